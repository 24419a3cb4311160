"""Stepwise Connect4 search with caller-supplied leaf values (include/zeroclone.h zc_c4_ext_*).

mcts.get_move (engine/mcts/src/mcts.cpp:102-160) pauses at every flush (:112-127) and hands
the pending leaves to `value.batch` (engine/value_functions.py:16-32).  `C4ValuedSearch`
drives the same loop for many games at once with the tree on the GPU:

    begin -> [select(f) -> value_fn(leaves, planes, counts) -> backup(f)] * n_flush -> end

`value_fn` returns one fp64 value per leaf slot (n_games * batch_size, leaf j of game i at
i*batch_size + j) for the leaf's side to move.  Two value functions are provided:

* `NetValue(model)` — the reference's network modes (value_functions.py:61-99, network.py):
  the planes are built on the device in state_to_tensor layout and fed straight into the
  fp16 model; no host round trip, so a whole move can be captured in one HIP graph
  (`C4ValuedSearch.capture`).
* `HostValue(value, backend)` — any reference-style Value object: the leaves go to the host
  as c4_backend states and `value.batch(states, backend=backend)` is called once per game
  per flush, as the reference does.  Slow, but it runs any plugin on the GPU tree search.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native


def _stream(dev) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _split_flushes(search, nfl: int, fns: list, first_game: int, select, evaluate_backup):
    """The flushes of k contiguous game parts, part i on stream i (stream 0: the current one;
    the others fork from it and join back), fns[i] the part's value / network function.  The
    parts share no tree, buffer or counter — select and backup of a part touch only its games
    and its slices of the leaf / plane / count / value buffers, and each fns[i] owns its
    network buffers — so the order of the launches across parts does not matter, and the GPU
    runs one part's search kernels beside another part's network.  select(first, n, f, leaves,
    planes, counts, stream); evaluate_backup(first, n, f, fn, leaves, planes, counts, values,
    stream) calls fn and backs its output up."""
    n, bs, k = search.n, search.bs, len(fns)
    main = torch.cuda.current_stream(search.dev)
    if getattr(search, "_side", None) is None or len(search._side) < k - 1:
        search._side = [torch.cuda.Stream(search.dev) for _ in range(k - 1)]
    streams = [main] + search._side[:k - 1]
    for st in streams[1:]:
        st.wait_stream(main)
    parts = []
    for i in range(k):
        lo, hi = i * n // k, (i + 1) * n // k
        if hi > lo:
            sl = slice(lo * bs, hi * bs)
            parts.append((lo, hi, streams[i], fns[i], search.leaves[sl] if search.leaves is not None else None,
                          search.planes[sl] if search.planes is not None else None, search.counts[lo:hi],
                          search.values[sl]))
    for f in range(nfl):
        for lo, hi, st, fn, lv, pv, cv, vv in parts:
            with torch.cuda.stream(st):
                select(first_game + lo, hi - lo, f, lv, pv, cv, st.cuda_stream)
                evaluate_backup(first_game + lo, hi - lo, f, fn, lv, pv, cv, vv, st.cuda_stream)
    for st in streams[1:]:
        main.wait_stream(st)


def _value_backup(sims: int, bs: int, backup):
    """evaluate_backup of a value search's part (_split_flushes): the part's network on its
    leaves (a short last flush on its nb leaves only, NetValue.rows), then backup(first, n,
    flush, values, stream)."""
    def evaluate_backup(first, m, f, fn, lv, pv, cv, vv, st):
        nb = min(bs, sims - f * bs)
        if nb < bs and hasattr(fn, "rows") and pv is not None:
            v = fn.rows(pv, m, bs, nb, vv)
        else:
            v = fn(lv, pv, cv)
        if v.data_ptr() != vv.data_ptr():
            vv.copy_(v.reshape(-1))
        backup(first, m, f, vv.data_ptr(), st)
    return evaluate_backup


class PolicyNet:
    """A policy + value network as a PUCT search's net_fn: net(planes) -> (values fp64 [rows],
    logits [rows, n_logits]).  It depends on the planes alone, so the search may call it on
    the n root positions of flush 0 (one leaf a game) instead of all n * batch_size slots."""
    roots_only = True

    def __init__(self, net):
        self.net = net

    def __call__(self, leaves, planes, counts):
        return self.net(planes)


def _puct_backup(bs: int, backup):
    """evaluate_backup of a PUCT search (part): fn on the flush's planes, then backup(first, n,
    flush, values, logits, logits_f16, stream, rows).  Flush 0 holds the roots only: a
    roots_only fn evaluates the n root positions alone (rows = 1)."""
    def evaluate_backup(first, m, f, fn, lv, pv, cv, vv, st):
        if f == 0 and getattr(fn, "roots_only", False):
            roots = pv.view(m, bs, *pv.shape[1:])[:, 0].contiguous()
            v, logits = fn(None, roots, cv)
            v = v.reshape(-1).to(torch.float64).contiguous()
            logits = logits.contiguous()
            backup(first, m, f, v.data_ptr(), logits.data_ptr(), logits.dtype == torch.float16, st, rows=1)
            return
        v, logits = fn(lv, pv, cv)
        if v.data_ptr() != vv.data_ptr():
            vv.copy_(v.reshape(-1))
        logits = logits.contiguous()
        backup(first, m, f, vv.data_ptr(), logits.data_ptr(), logits.dtype == torch.float16, st)
    return evaluate_backup


def _warm_parts(search, fns):
    """Each part's function once on its own slice, and a PolicyNet also at the roots flush's
    shape (graph capture warms kernels and buffers)."""
    k, n, bs = len(fns), search.n, search.bs
    for i, fn in enumerate(fns):
        lo, hi = i * n // k, (i + 1) * n // k
        fn(search.leaves[lo * bs:hi * bs] if search.leaves is not None else None,
           search.planes[lo * bs:hi * bs] if search.planes is not None else None, search.counts[lo:hi])
        if getattr(fn, "roots_only", False):
            fn(None, search.planes[lo * bs:hi * bs:bs].contiguous(), search.counts[lo:hi])


class C4ValuedSearch:
    def __init__(self, eng: "_native.NativeEngine", n_games: int, batch_size: int = 32,
                 planes_dtype: torch.dtype = torch.float16, leaves: bool = True, planes: bool = True):
        if batch_size > eng.max_batch:
            raise ValueError(f"batch_size {batch_size} > engine max_batch {eng.max_batch}")
        if n_games > eng.max_games:
            raise ValueError(f"{n_games} games > engine capacity {eng.max_games}")
        if planes_dtype not in (torch.float16, torch.float32):
            raise ValueError("planes_dtype must be float16 or float32")
        self.eng, self.n, self.bs = eng, n_games, batch_size
        self.dev = torch.device("cuda", eng.device)
        L = n_games * batch_size
        self.leaves = torch.zeros((L, 3), dtype=torch.int64, device=self.dev) if leaves else None
        self.planes = torch.zeros((L, 2, 6, 7), dtype=planes_dtype, device=self.dev) if planes else None
        self.counts = torch.zeros(n_games, dtype=torch.int32, device=self.dev)
        self.values = torch.zeros(L, dtype=torch.float64, device=self.dev)
        self.move = torch.zeros(n_games, dtype=torch.int32, device=self.dev)
        self.na = torch.zeros((n_games, 7), dtype=torch.int32, device=self.dev)
        self.stats = torch.zeros((n_games, _native.STATS_FIELDS), dtype=torch.int64, device=self.dev)

    def _ptr(self, t):
        return t.data_ptr() if t is not None else 0

    def enqueue(self, roots: torch.Tensor, sims: int, c: float, value_fn, first_game: int = 0):
        """Enqueue one whole move on torch's current stream (no host synchronisation unless
        value_fn makes one)."""
        if roots.shape != (self.n, 3) or roots.dtype != torch.int64 or not roots.is_contiguous():
            raise ValueError("roots must be a contiguous int64 [n_games, 3] tensor of zc_c4_state rows")
        if roots.device != self.dev:
            raise ValueError("roots must live on the engine's device")
        s = _stream(self.dev)
        e, n = self.eng, self.n
        e.c4_ext_begin(first_game, n, roots.data_ptr(), sims, c, self.bs, s)
        nfl = (sims + self.bs - 1) // self.bs
        if isinstance(value_fn, (list, tuple)):   # the games in parts on their own streams (_split_flushes)
            def select(first, m, f, lv, pv, cv, st):
                e.c4_ext_select(first, m, f, self._ptr(lv), self._ptr(pv), pv is None or pv.dtype == torch.float16,
                                cv.data_ptr(), st)
            _split_flushes(self, nfl, list(value_fn), first_game, select,
                           _value_backup(sims, self.bs, e.c4_ext_backup))
            nfl = 0
        for f in range(nfl):
            e.c4_ext_select(first_game, n, f, self._ptr(self.leaves), self._ptr(self.planes),
                            self.planes is None or self.planes.dtype == torch.float16, self.counts.data_ptr(), s)
            nb = min(self.bs, sims - f * self.bs)   # every game's pending leaves (0 after an error)
            if nb < self.bs and hasattr(value_fn, "rows") and self.planes is not None:
                v = value_fn.rows(self.planes, n, self.bs, nb, self.values)   # a short last flush
            else:
                v = value_fn(self.leaves, self.planes, self.counts)
            if v is not self.values:
                self.values.copy_(v.reshape(-1))
            e.c4_ext_backup(first_game, n, f, self.values.data_ptr(), _stream(self.dev))
        e.c4_ext_end(first_game, n, self.move.data_ptr(), self.na.data_ptr(), self.stats.data_ptr(),
                     _stream(self.dev))
        return self.move, self.na, self.stats

    def run(self, roots: torch.Tensor, sims: int, c: float, value_fn, first_game: int = 0):
        self.enqueue(roots, sims, c, value_fn, first_game)
        torch.cuda.current_stream(self.dev).synchronize()
        return self.move, self.na, self.stats

    def capture(self, roots: torch.Tensor, sims: int, c: float, value_fn, first_game: int = 0):
        """Capture one move into a HIP graph (value_fn must be capturable, e.g. NetValue).
        Returns the graph; graph.replay() re-runs the move on the current contents of
        `roots` and of the games' RNG streams."""
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):  # warm the value function's kernels outside capture
            _warm_parts(self, value_fn if isinstance(value_fn, (list, tuple)) else [value_fn])
        torch.cuda.current_stream(self.dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.enqueue(roots, sims, c, value_fn, first_game)
        return g


class NetValue:
    """Value('network_*') (value_functions.py:61-99): model(planes) in the planes' dtype;
    the [B, 1] output is the value for each leaf's side to move."""

    def __init__(self, model: torch.nn.Module):
        self.model = model

    @torch.no_grad()
    def __call__(self, leaves, planes, counts):
        return self.model(planes).reshape(-1).to(torch.float64)

    @torch.no_grad()
    def rows(self, planes, n: int, bs: int, nb: int, out):
        """A flush whose games all hold nb < bs pending leaves (the last flush of a search
        whose simulations are not a multiple of the batch): the network runs on those n*nb
        boards only, and their values land in out's first nb slots of each game (the others
        are never backed up).  Each board's value does not depend on its batch: the values
        are those of the full call."""
        sub = planes.view(n, bs, *planes.shape[1:])[:, :nb].reshape(n * nb, *planes.shape[1:])
        out.view(n, bs)[:, :nb].copy_(self.model(sub).reshape(n, nb).to(torch.float64))
        return out


class HostValue:
    """Any reference-style Value object: value.batch(states, backend=backend) per game per
    flush, on c4_backend states built from the device leaves.  With `eng`, Python's global
    `random` is game first_game + i's device stream during the call (the flush's expansion
    draws already taken, as in mcts.cpp:112-127), so a value object that draws from `random`
    gets the reference's numbers and the search continues after them."""

    def __init__(self, value, backend, eng=None, first_game: int = 0):
        self.value, self.backend, self.eng, self.first = value, backend, eng, first_game

    def __call__(self, leaves, planes, counts):
        from .engine._device import game_stream
        from .engine.games.connect4 import c4_backend as zb
        rows = leaves.cpu().numpy().view(np.uint64)
        cnt = counts.cpu().numpy()
        bs = rows.shape[0] // cnt.shape[0]
        out = np.zeros(rows.shape[0], np.float64)
        for i, k in enumerate(cnt):
            if k == 0:
                continue
            states = [zb.from_zc(int(r[0]), int(r[1]), int(r[2]) & 1) for r in rows[i * bs: i * bs + k]]
            if self.eng is None:
                v = self.value.batch(states, backend=self.backend)
            else:
                with game_stream(self.eng, self.first + i):
                    v = self.value.batch(states, backend=self.backend)
            out[i * bs: i * bs + k] = [float(x) for x in v]
        return torch.from_numpy(out).to(leaves.device)


class ChessValuedSearch:
    """Stepwise chess search (zc_chess_ext_*): the configs/chess_value.yaml path — a value
    network evaluates every flush's leaves (planes [n*bs, 17, 8, 8]) between the select and
    backup kernels.  Same protocol and value_fn contract as C4ValuedSearch."""

    def __init__(self, eng: "_native.NativeEngine", n_games: int, batch_size: int = 32,
                 planes_dtype: torch.dtype = torch.float16, leaves: bool = True, planes: bool = True,
                 policy: int = _native.ZC_POLICY_RANDOM, freedom: float = 0.0):
        if batch_size > eng.max_batch:
            raise ValueError(f"batch_size {batch_size} > engine max_batch {eng.max_batch}")
        if n_games > eng.max_games:
            raise ValueError(f"{n_games} games > engine capacity {eng.max_games}")
        self.eng, self.n, self.bs, self.policy, self.freedom = eng, n_games, batch_size, policy, freedom
        eng.chess_reserve()   # the tree arena exists before any graph capture
        self.dev = torch.device("cuda", eng.device)
        L = n_games * batch_size
        self.leaves = torch.zeros((L, 72), dtype=torch.uint8, device=self.dev) if leaves else None
        self.planes = torch.zeros((L, 17, 8, 8), dtype=planes_dtype, device=self.dev) if planes else None
        self.counts = torch.zeros(n_games, dtype=torch.int32, device=self.dev)
        self.values = torch.zeros(L, dtype=torch.float64, device=self.dev)
        self.move = torch.zeros(n_games, dtype=torch.int16, device=self.dev)
        self.na = torch.zeros((n_games, _native.CHESS_MAX_MOVES), dtype=torch.int32, device=self.dev)
        self.stats = torch.zeros((n_games, _native.STATS_FIELDS), dtype=torch.int64, device=self.dev)

    def enqueue(self, roots: torch.Tensor, sims: int, c: float, value_fn, first_game: int = 0):
        if roots.shape != (self.n, 72) or roots.dtype != torch.uint8 or not roots.is_contiguous():
            raise ValueError("roots must be a contiguous uint8 [n_games, 72] tensor of zc_chess_state rows")
        e, n = self.eng, self.n
        p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        e.chess_ext_begin(first_game, n, roots.data_ptr(), sims, c, self.bs, self.policy, self.freedom,
                          _stream(self.dev))
        nfl = (sims + self.bs - 1) // self.bs
        if isinstance(value_fn, (list, tuple)):   # the games in parts on their own streams (_split_flushes)
            def select(first, m, f, lv, pv, cv, st):
                e.chess_ext_select(first, m, f, p(lv), p(pv), pv is None or pv.dtype == torch.float16,
                                   cv.data_ptr(), st)
            _split_flushes(self, nfl, list(value_fn), first_game, select,
                           _value_backup(sims, self.bs, e.chess_ext_backup))
            nfl = 0
        for f in range(nfl):
            e.chess_ext_select(first_game, n, f, p(self.leaves), p(self.planes),
                               self.planes is None or self.planes.dtype == torch.float16, self.counts.data_ptr(),
                               _stream(self.dev))
            nb = min(self.bs, sims - f * self.bs)   # every game's pending leaves (0 after an error)
            if hasattr(value_fn, "flush_values"):   # values computed on the device from the tree itself
                v = value_fn.flush_values(first_game, n, f, _stream(self.dev))
            elif nb < self.bs and hasattr(value_fn, "rows") and self.planes is not None:
                v = value_fn.rows(self.planes, n, self.bs, nb, self.values)   # a short last flush
            else:
                v = value_fn(self.leaves, self.planes, self.counts)
            if v is not self.values:
                self.values.copy_(v.reshape(-1))
            e.chess_ext_backup(first_game, n, f, self.values.data_ptr(), _stream(self.dev))
        e.chess_ext_end(first_game, n, self.move.data_ptr(), self.na.data_ptr(), self.stats.data_ptr(),
                        _stream(self.dev))
        return self.move, self.na, self.stats

    def run(self, roots: torch.Tensor, sims: int, c: float, value_fn, first_game: int = 0):
        self.enqueue(roots, sims, c, value_fn, first_game)
        torch.cuda.current_stream(self.dev).synchronize()
        return self.move, self.na, self.stats

    capture = C4ValuedSearch.capture


class ChessPuctSearch:
    """AlphaZero-style PUCT search for chess (zc_chess_puct_*).

    net_fn(leaves, planes, counts) -> (values fp64 [n*bs], logits [n*bs, 4096] fp32/fp16,
    index from*64 + to).  Flush 0 evaluates the roots; Dirichlet(alpha) noise of weight eps
    goes on the root priors; end() picks by visits (temperature 0) or samples."""

    def __init__(self, eng: "_native.NativeEngine", n_games: int, batch_size: int = 32, c_puct: float = 1.5,
                 dirichlet_alpha: float = 0.3, dirichlet_eps: float = 0.25, seed: int = 0,
                 planes_dtype: torch.dtype = torch.float16, leaves: bool = True, planes_nhwc: bool = False):
        """planes_nhwc: the select kernel writes the planes in the MFMA tower's input layout, fp16
        [n * batch_size, 64, 32] (17 planes then zeros, square-major), so the network takes them
        without a conversion launch (MfmaPolicyValueNetwork with the convolutional head)."""
        if batch_size > eng.max_batch:
            raise ValueError(f"batch_size {batch_size} > engine max_batch {eng.max_batch}")
        if planes_nhwc and planes_dtype != torch.float16:
            raise ValueError("planes_nhwc needs fp16 planes")
        self.eng, self.n, self.bs = eng, n_games, batch_size
        self.c, self.alpha, self.eps, self.seed = c_puct, dirichlet_alpha, dirichlet_eps, seed
        eng.chess_reserve()   # the tree arena exists before any graph capture
        self.dev = torch.device("cuda", eng.device)
        L = n_games * batch_size
        self.planes_nhwc = planes_nhwc
        self.leaves = torch.zeros((L, 72), dtype=torch.uint8, device=self.dev) if leaves else None
        self.planes = torch.zeros((L, 64, 32) if planes_nhwc else (L, 17, 8, 8), dtype=planes_dtype, device=self.dev)
        self.counts = torch.zeros(n_games, dtype=torch.int32, device=self.dev)
        self.values = torch.zeros(L, dtype=torch.float64, device=self.dev)
        self.move = torch.zeros(n_games, dtype=torch.int16, device=self.dev)
        self.na = torch.zeros((n_games, _native.CHESS_MAX_MOVES), dtype=torch.int32, device=self.dev)
        self.prior = torch.zeros((n_games, _native.CHESS_MAX_MOVES), dtype=torch.float32, device=self.dev)
        self.stats = torch.zeros((n_games, _native.STATS_FIELDS), dtype=torch.int64, device=self.dev)
        # per-game search number: the Philox counter word of the root noise and the
        # temperature sample; each search adds 1 on the device (graph replays included)
        self.search_no = torch.zeros(n_games, dtype=torch.int32, device=self.dev)

    def enqueue(self, roots: torch.Tensor, sims: int, net_fn, temperature: float = 0.0, first_game: int = 0):
        """net_fn: one callable, or a list of k callables — then the games are split into k
        contiguous parts searched on k streams (`_enqueue_split`): one part's select, backup
        and policy GEMM overlap another part's tower.  The results are the same."""
        e, n = self.eng, self.n
        p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        nfl = _native.check(_native.lib().zc_chess_puct_flushes(int(sims), int(self.bs)))
        e.chess_puct_begin(first_game, n, roots.data_ptr(), sims, self.c, self.bs, self.alpha, self.eps, self.seed,
                           self.search_no.data_ptr(), stream=_stream(self.dev))
        if isinstance(net_fn, (list, tuple)):
            self._enqueue_split(nfl, list(net_fn), first_game)
            e.chess_puct_end(first_game, n, temperature, self.move.data_ptr(), self.na.data_ptr(),
                             self.prior.data_ptr(), self.stats.data_ptr(), _stream(self.dev))
            return self.move, self.na, self.stats
        evaluate_backup = _puct_backup(self.bs, e.chess_puct_backup)
        for f in range(nfl):
            e.chess_puct_select(first_game, n, f, p(self.leaves), p(self.planes),
                                self.planes.dtype == torch.float16, self.counts.data_ptr(), _stream(self.dev),
                                planes_nhwc=self.planes_nhwc)
            evaluate_backup(first_game, n, f, net_fn, self.leaves, self.planes, self.counts, self.values,
                            _stream(self.dev))
        e.chess_puct_end(first_game, n, temperature, self.move.data_ptr(), self.na.data_ptr(), self.prior.data_ptr(),
                         self.stats.data_ptr(), _stream(self.dev))
        return self.move, self.na, self.stats

    def _enqueue_split(self, nfl: int, fns: list, first_game: int):
        """The search split over len(fns) streams (_split_flushes): one part's select and
        backup beside another part's tower."""
        e = self.eng

        def select(first, n, f, lv, pv, cv, s):
            e.chess_puct_select(first, n, f, lv.data_ptr() if lv is not None else 0, pv.data_ptr(),
                                pv.dtype == torch.float16, cv.data_ptr(), s, planes_nhwc=self.planes_nhwc)

        _split_flushes(self, nfl, fns, first_game, select, _puct_backup(self.bs, e.chess_puct_backup))

    def run(self, roots, sims, net_fn, temperature: float = 0.0, first_game: int = 0):
        self.enqueue(roots, sims, net_fn, temperature, first_game)
        torch.cuda.current_stream(self.dev).synchronize()
        return self.move, self.na, self.stats

    def capture(self, roots, sims, net_fn, temperature: float = 0.0, first_game: int = 0):
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            _warm_parts(self, net_fn if isinstance(net_fn, (list, tuple)) else [net_fn])
        torch.cuda.current_stream(self.dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.enqueue(roots, sims, net_fn, temperature, first_game)
        return g


class C4PuctSearch:
    """AlphaZero-style PUCT search for Connect4 (zc_c4_puct_*, SURVEY §8 a21 on the target
    game): the chess PUCT search's selection, virtual loss, Dirichlet root noise and
    temperature on the Connect4 rules.

    net_fn(leaves, planes, counts) -> (values fp64 [n*bs], logits [n*bs, 7] fp32/fp16, one per
    column) — e.g. `lambda l, p, c: net(p)` with nets.MfmaPolicyValueNetwork over
    PolicyValueNetwork(in_planes=2, board=(6, 7), n_logits=7)."""

    def __init__(self, eng: "_native.NativeEngine", n_games: int, batch_size: int = 32, c_puct: float = 1.5,
                 dirichlet_alpha: float = 0.3, dirichlet_eps: float = 0.25, seed: int = 0,
                 planes_dtype: torch.dtype = torch.float16, leaves: bool = True):
        if batch_size > eng.max_batch:
            raise ValueError(f"batch_size {batch_size} > engine max_batch {eng.max_batch}")
        self.eng, self.n, self.bs = eng, n_games, batch_size
        self.c, self.alpha, self.eps, self.seed = c_puct, dirichlet_alpha, dirichlet_eps, seed
        self.dev = torch.device("cuda", eng.device)
        L = n_games * batch_size
        self.leaves = torch.zeros((L, 3), dtype=torch.int64, device=self.dev) if leaves else None
        self.planes = torch.zeros((L, 2, 6, 7), dtype=planes_dtype, device=self.dev)
        self.counts = torch.zeros(n_games, dtype=torch.int32, device=self.dev)
        self.values = torch.zeros(L, dtype=torch.float64, device=self.dev)
        self.move = torch.zeros(n_games, dtype=torch.int32, device=self.dev)
        self.na = torch.zeros((n_games, 7), dtype=torch.int32, device=self.dev)
        self.prior = torch.zeros((n_games, 7), dtype=torch.float32, device=self.dev)
        self.stats = torch.zeros((n_games, _native.STATS_FIELDS), dtype=torch.int64, device=self.dev)
        self.search_no = torch.zeros(n_games, dtype=torch.int32, device=self.dev)   # as ChessPuctSearch
        # the tree arena exists before any graph capture
        z = torch.zeros((1, 3), dtype=torch.int64, device=self.dev)
        eng.c4_puct_begin(0, 0, z.data_ptr(), 2, c_puct, batch_size, dirichlet_alpha, dirichlet_eps, seed)

    def enqueue(self, roots: torch.Tensor, sims: int, net_fn, temperature: float = 0.0, first_game: int = 0):
        e, n = self.eng, self.n
        p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        nfl = _native.check(_native.lib().zc_chess_puct_flushes(int(sims), int(self.bs)))
        e.c4_puct_begin(first_game, n, roots.data_ptr(), sims, self.c, self.bs, self.alpha, self.eps, self.seed,
                        self.search_no.data_ptr(), stream=_stream(self.dev))
        if isinstance(net_fn, (list, tuple)):   # split over streams, as ChessPuctSearch
            def select(first, m, f, lv, pv, cv, s):
                e.c4_puct_select(first, m, f, lv.data_ptr() if lv is not None else 0, pv.data_ptr(),
                                 pv.dtype == torch.float16, cv.data_ptr(), s)

            _split_flushes(self, nfl, list(net_fn), first_game, select, _puct_backup(self.bs, e.c4_puct_backup))
            nfl = 0
        evaluate_backup = _puct_backup(self.bs, e.c4_puct_backup)
        for f in range(nfl):
            e.c4_puct_select(first_game, n, f, p(self.leaves), p(self.planes), self.planes.dtype == torch.float16,
                             self.counts.data_ptr(), _stream(self.dev))
            evaluate_backup(first_game, n, f, net_fn, self.leaves, self.planes, self.counts, self.values,
                            _stream(self.dev))
        e.c4_puct_end(first_game, n, temperature, self.move.data_ptr(), self.na.data_ptr(), self.prior.data_ptr(),
                      self.stats.data_ptr(), _stream(self.dev))
        return self.move, self.na, self.stats

    run = ChessPuctSearch.run
    capture = ChessPuctSearch.capture
