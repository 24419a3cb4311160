"""Device-resident self-play, its trajectories, and the multi-GPU trajectory exchange.

`C4SelfPlay` / `ChessSelfPlay` are the batched form of scripts/train.py:simulate_games
(:151-170) + Engine.play_mcts_parallel (engine/engine.py:131-138): G games live on one GPU;
one `step()` searches every game, plays the chosen moves and evaluates them
(Engine.play_move/_evaluate) on the device.  Game slot g of rank r is global slot r*G + g
and draws from its own CPython MT19937 stream seeded seed + global slot id, so per-game
results do not depend on the number of GPUs.

Trajectories never leave the device while games are played (`Trajectories`,
zc_traj_record_async): every position is appended to its slot's game in HBM; a finished game
is labelled exactly as Engine.get_dataset (engine.py:60-89) labels it and copied to a
device pool, and its slot restarts from the opening (or goes idle once simulate_games'
quota of games has started).  `take()` returns the pool's games in start order as device
tensors; `gather_positions` all-gathers every rank's positions (counts first, then a padded
payload) over torch.distributed — RCCL over xGMI on the GPUs, gloo on CPU — the one
collective of the scale-out path; `ReplayBuffer` is
scripts/train.py:_update_replay (:27-50) over device tensors.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import os

import numpy as np
import torch

from . import _native

ONGOING = _native.ZC_C4_ONGOING
IDLE = _native.ZC_SLOT_IDLE
_UNLIMITED = 1 << 62


def dataset_labels(n_states: int, result: int) -> np.ndarray:
    """Engine.get_dataset's labels for one finished history of n_states positions
    (initial ... terminal): factor starts at 0 (draw) or -1, alternates sign, and the
    per-game list is appended REVERSED (engine.py:72-81)."""
    factor = 0 if result == 0 else -1
    entry = []
    for _ in range(n_states):
        entry.append(factor)
        factor = -factor
    return np.asarray(list(reversed(entry)), dtype=np.float32)


def planes(positions: np.ndarray) -> np.ndarray:
    """Compact rows -> c4_backend.state_to_tensor planes [n, 2, 6, 7] (side to move first)."""
    n = positions.shape[0]
    out = np.zeros((n, 2, 6, 7), np.float32)
    s0 = positions[:, 0].astype(np.uint64)
    s1 = positions[:, 1].astype(np.uint64)
    turn = (positions[:, 2] & 1).astype(np.int64)
    for r in range(6):
        for c in range(7):
            bit = np.uint64(1) << np.uint64(7 * c + (5 - r))
            x = (s0 & bit) != 0
            o = (s1 & bit) != 0
            out[:, 0, r, c] = np.where(turn == 0, x, o)
            out[:, 1, r, c] = np.where(turn == 0, o, x)
    return out


@dataclass
class TrajBatch:
    """Finished games taken from a `Trajectories` pool, in start order (device tensors).

    rows   [n, row_bytes // 8] int64  positions (zc_c4_state / zc_chess_state records)
    labels [n] int32                  Engine.get_dataset label of each position
    moves  [n] int16                  move played from it (-1 at a game's last position)
    games  [k, 5] int64               game number, slot, result, first row, positions
    """
    rows: torch.Tensor
    labels: torch.Tensor
    moves: torch.Tensor
    games: torch.Tensor

    def results(self) -> list[int]:
        return [int(r) for r in self.games[:, 2].cpu().tolist()]


class Trajectories:
    """Per-slot game histories and the pool of finished games, all in HBM (zc_traj_record_async).

    `max_len` positions per game (Connect4: 43), room for `games_cap` finished games and
    `pool_cap` positions until the next `take()`."""

    def __init__(self, n_slots: int, init_row: torch.Tensor, max_len: int, games_cap: int, pool_cap: int,
                 device: torch.device):
        init = init_row.reshape(-1).contiguous().view(torch.uint8)
        if init.numel() % 8:
            raise ValueError("row size must be a multiple of 8 bytes")
        self.n, self.W, self.max_len, self.dev = n_slots, init.numel() // 8, max_len, device
        self.init = init.view(torch.int64).to(device).clone()
        self.hist = torch.zeros((n_slots, max_len, self.W), dtype=torch.int64, device=device)
        self.hmoves = torch.zeros((n_slots, max_len), dtype=torch.int16, device=device)
        self.slot = torch.zeros((n_slots, 4), dtype=torch.int32, device=device)
        self.ctl = torch.zeros(8, dtype=torch.int64, device=device)
        self._alloc_pool(games_cap, pool_cap)
        self.start(None)

    def _alloc_pool(self, games_cap: int, pool_cap: int):
        if getattr(self, "pinned", False):
            # a captured step graph has this pool's pointers baked into its record kernel:
            # replacing the buffers would leave the graph writing into freed memory
            raise RuntimeError(f"the trajectory pool ({self.games_cap} games, {self.pool_cap} positions) is held by "
                               f"a captured step graph and cannot grow to ({games_cap}, {pool_cap}); construct the "
                               "self-play pool with a larger games_cap before capture_step()")
        self.games_cap, self.pool_cap = int(games_cap), int(pool_cap)
        self.pool = torch.zeros((self.pool_cap, self.W), dtype=torch.int64, device=self.dev)
        self.labels = torch.zeros(self.pool_cap, dtype=torch.int32, device=self.dev)
        self.pool_moves = torch.zeros(self.pool_cap, dtype=torch.int16, device=self.dev)
        self.games = torch.zeros((self.games_cap, 4), dtype=torch.int64, device=self.dev)
        b = _native.TrajBuffers()
        b.row_bytes, b.max_len, b.pool_cap, b.games_cap = 8 * self.W, self.max_len, self.pool_cap, self.games_cap
        for f, t in (("d_hist", self.hist), ("d_hmoves", self.hmoves), ("d_slot", self.slot), ("d_pool", self.pool),
                     ("d_labels", self.labels), ("d_pool_moves", self.pool_moves), ("d_games", self.games),
                     ("d_ctl", self.ctl), ("d_init", self.init)):
            setattr(b, f, t.data_ptr())
        self._buf = b

    def _grow_pool(self, games_cap: int, pool_cap: int):
        """A larger pool holding the positions and game records reserved so far."""
        ctl = self.ctl.cpu().tolist()
        npos, ngames = int(ctl[_native.ZC_TRAJ_POSITIONS]), int(ctl[_native.ZC_TRAJ_GAMES])
        old = (self.pool, self.labels, self.pool_moves, self.games)
        self._alloc_pool(games_cap, pool_cap)
        self.pool[:npos] = old[0][:npos]
        self.labels[:npos] = old[1][:npos]
        self.pool_moves[:npos] = old[2][:npos]
        self.games[:ngames] = old[3][:ngames]

    def ensure_room(self):
        """Grow the pool (on demand, keeping its contents) so that the next step cannot
        overflow it: a slot's game that finishes at that step has at most its current
        history length + 1 positions, so the worst case is known before the step — far less
        than quota x max_len.  One small device read; simulate_games calls it per step."""
        act = self.slot[:, 1] >= 0
        need = torch.stack([(self.slot[:, 0].to(torch.int64) + 1)[act].sum(), act.sum().to(torch.int64)])
        ctl = self.ctl[[_native.ZC_TRAJ_POSITIONS, _native.ZC_TRAJ_GAMES]]
        npos, ngames = (int(x) for x in (ctl + need).tolist())
        if npos > self.pool_cap or ngames > self.games_cap:
            self._grow_pool(max(ngames, self.games_cap, 2 * self.games_cap if ngames > self.games_cap else 0),
                            max(npos, self.pool_cap, 2 * self.pool_cap if npos > self.pool_cap else 0))

    def start(self, quota: int | None, games_cap: int | None = None):
        """Slot g plays game g (g < quota) or idles; the pool is emptied.  quota None = no
        limit (every finished game's slot starts another).  With a quota the game records are
        sized for it and the positions grow on demand (`ensure_room` before each step), so
        simulate_games never drops a game (round 4 reserved quota x max_len positions up
        front: 2,049 rows per chess game)."""
        q = _UNLIMITED if quota is None else int(quota)
        self.quota = q
        need_g = max(int(games_cap or 0), q if quota is not None else 0)
        if need_g > self.games_cap:
            self._alloc_pool(need_g, self.pool_cap)
        ids = torch.arange(self.n, dtype=torch.int32, device=self.dev)
        self.slot.zero_()
        self.slot[:, 0] = 1
        self.slot[:, 1] = torch.where(ids < min(q, self.n), ids, torch.full_like(ids, -1))
        self.hist[:, 0] = self.init
        self.ctl.zero_()
        self.ctl[_native.ZC_TRAJ_NEXT] = min(q, self.n)
        self.ctl[_native.ZC_TRAJ_QUOTA] = q

    def record(self, d_states: int, moves: torch.Tensor, results: torch.Tensor, flags: torch.Tensor | None = None,
               rep: torch.Tensor | None = None, stream: int = 0):
        _native.check(_native.lib().zc_traj_record_async(
            self.n, ctypes.byref(self._buf), ctypes.c_void_p(d_states), ctypes.c_void_p(moves.data_ptr()),
            ctypes.c_void_p(results.data_ptr()), ctypes.c_void_p(flags.data_ptr() if flags is not None else None),
            ctypes.c_void_p(rep.data_ptr() if rep is not None else None), ctypes.c_void_p(stream or None)))

    def record_steps(self, d_states: int, moves: torch.Tensor, results: torch.Tensor, steps: int,
                     reached: torch.Tensor | None = None, stream: int = 0):
        """record() for `steps` consecutive [steps][n] self-play outputs in one call
        (zc_traj_record_steps_async: four launches whatever `steps` is); only the steps
        k < *reached are read.  Needs the unlimited quota."""
        if self.quota != _UNLIMITED:
            raise ValueError("multi-step recording needs the unlimited quota (start(None))")
        need = ctypes.c_int64(0)
        _native.check(_native.lib().zc_traj_steps_scratch_bytes(self.n, int(steps), ctypes.byref(need)))
        if getattr(self, "_scratch", None) is None or self._scratch.numel() < need.value:
            self._scratch = torch.empty(max(need.value, 16), dtype=torch.uint8, device=self.dev)
        _native.check(_native.lib().zc_traj_record_steps_async(
            self.n, ctypes.byref(self._buf), ctypes.c_void_p(d_states), ctypes.c_void_p(moves.data_ptr()),
            ctypes.c_void_p(results.data_ptr()), int(steps),
            ctypes.c_void_p(reached.data_ptr() if reached is not None else None),
            ctypes.c_void_p(self._scratch.data_ptr()), self._scratch.numel(), ctypes.c_void_p(stream or None)))

    def finished(self) -> int:
        """Games finished since start() (one device read); raises at once if the pool has
        overflowed (a game was dropped), rather than at take()."""
        fin, ov = (int(x) for x in self.ctl[[_native.ZC_TRAJ_FINISHED, _native.ZC_TRAJ_OVERFLOW]].tolist())
        if ov:
            self.take()   # raises with the overflow's cause
        return fin

    def take(self) -> TrajBatch:
        """The pooled games, sorted by game number (start order), as device tensors; the pool
        is emptied (slots keep their games in progress)."""
        ctl = self.ctl.cpu().tolist()
        if ctl[_native.ZC_TRAJ_OVERFLOW]:
            raise RuntimeError("trajectory pool overflow: " + ("pool full (take() more often or raise games_cap) "
                                                               if ctl[_native.ZC_TRAJ_OVERFLOW] & 1 else "")
                               + ("a game longer than max_len " if ctl[_native.ZC_TRAJ_OVERFLOW] & 2 else "")
                               + ("the quota ran out inside a multi-step record" if ctl[_native.ZC_TRAJ_OVERFLOW] & 4
                                  else ""))
        k, n = int(ctl[_native.ZC_TRAJ_GAMES]), int(ctl[_native.ZC_TRAJ_POSITIONS])
        g = self.games[:k]
        order = torch.argsort(g[:, 0])
        g = g[order]
        lens = g[:, 3]
        starts = torch.cumsum(lens, 0) - lens
        idx = torch.repeat_interleave(g[:, 2] - starts, lens, output_size=n) + torch.arange(n, device=self.dev)
        games = torch.stack([g[:, 0], g[:, 1] >> 32, (g[:, 1] & 0xFFFFFFFF) - 1, starts, lens], dim=1)
        out = TrajBatch(self.pool[idx].clone(), self.labels[idx].clone(), self.pool_moves[idx].clone(), games)
        self.ctl[_native.ZC_TRAJ_POSITIONS] = 0
        self.ctl[_native.ZC_TRAJ_GAMES] = 0
        return out


def _room(traj, stream: int | None = None):
    """Before a step under a game quota: grow the trajectory pool so the step cannot overflow
    it (not while a step is being captured into a graph: the unlimited quota is the graphs'
    case, and their pool is pinned).  `stream`: the stream the step runs on (None: torch's
    current one).  The control read and the pool copy run ON that stream, so the read sees the
    previous step's record kernel finished and the copy is ordered before the next one."""
    if traj is None or traj.quota == _UNLIMITED or torch.cuda.is_current_stream_capturing():
        return
    cur = torch.cuda.current_stream(traj.dev)
    if stream is None or stream == cur.cuda_stream:
        traj.ensure_room()
        return
    with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=traj.dev)):
        traj.ensure_room()


def _warm(search, fn, sims: int):
    """Each part's network once on its own slice of the search's buffers (and at a PolicyNet's
    roots shape: valued._warm_parts), and once at the short last flush's shape
    (NetValue.rows) when the simulations are not a multiple of the batch: kernels loaded and
    buffers allocated before a graph capture."""
    from .valued import _warm_parts
    fns = list(fn) if isinstance(fn, (list, tuple)) else [fn]
    _warm_parts(search, fns)
    nb, k, n, bs = sims % search.bs, len(fns), search.n, search.bs
    for i, f in enumerate(fns):
        lo, hi = i * n // k, (i + 1) * n // k
        if nb and hasattr(f, "rows"):
            f.rows(search.planes[lo * bs:hi * bs], hi - lo, bs, nb, search.values[lo * bs:hi * bs])


class C4SelfPlay:
    """Connect4 self-play pool on one GPU: search (zc_c4_search_async) + play/evaluate
    (zc_c4_play_async) + trajectory recording (zc_traj_record_async), all stream-ordered,
    no host synchronisation per step.  With `net=` the search takes its leaf values from a
    value network (C4ValuedSearch, C2(iii)); with `puct_net=` it is the PUCT search with a
    policy + value network (C4PuctSearch), moves sampled at `temperature`;
    both step() only (the network runs between kernels) and capture_step() into one graph."""

    MAX_LEN = 43   # the opening + at most 42 moves

    def __init__(self, games: int, sims: int, c: float = 1.4, batch_size: int = 32, seed: int = 0,
                 rank: int = 0, device: int = 0, record: bool = True, games_cap: int | None = None,
                 net=None, puct_net=None, temperature: float = 1.0, puct_seed: int = 1, streams: int = 1):
        self.G, self.sims, self.c, self.bs = games, sims, c, batch_size
        self.dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.eng = _native.NativeEngine(max_games=games, max_sims=sims, max_batch=batch_size,
                                        device=self.dev.index or 0)
        self.first_id = rank * games
        self.eng.seed(0, [seed + self.first_id + g for g in range(games)])
        self.roots = torch.zeros((games, 3), dtype=torch.int64, device=self.dev)
        self.moves = torch.zeros(games, dtype=torch.int32, device=self.dev)
        self.moves16 = torch.zeros(games, dtype=torch.int16, device=self.dev)
        self.na = torch.zeros((games, 7), dtype=torch.int32, device=self.dev)
        self.stats = torch.zeros((games, _native.STATS_FIELDS), dtype=torch.int64, device=self.dev)
        self.results = torch.zeros(games, dtype=torch.int32, device=self.dev)
        self.record = record
        self.traj = None
        if record:
            cap = games_cap or max(8 * games, 1024)
            self.traj = Trajectories(games, torch.zeros(24, dtype=torch.uint8), self.MAX_LEN, cap,
                                     cap * self.MAX_LEN, self.dev)
        self.totals = torch.zeros(2, dtype=torch.int64, device=self.dev)   # expansions, depth sum since reset
        self.carry_pending = False   # run_pooled(carry=True) left moves in flight (drain() finishes them)
        self.vs = self.value_fn = self.ps = self.net_fn = None
        self.temperature = float(temperature)
        if net is not None:
            from .valued import C4ValuedSearch, NetValue
            self.vs = C4ValuedSearch(self.eng, games, batch_size, leaves=False)
            self.value_fn = NetValue(net)
            if streams > 1:   # the games in parts on their own streams (valued._split_flushes)
                self.value_fn = [NetValue(net.replica() if hasattr(net, "replica") else net) for _ in range(streams)]
        if puct_net is not None:
            from .valued import C4PuctSearch, PolicyNet
            self.ps = C4PuctSearch(self.eng, games, batch_size, seed=puct_seed, leaves=False)
            self.net_fn = PolicyNet(puct_net)
            if streams > 1:
                self.net_fn = [PolicyNet(puct_net.replica()) for _ in range(streams)]

    def start(self, quota: int | None = None):
        """Every slot back to the opening; with a quota, slots beyond it idle and finished
        slots start new games only while fewer than `quota` have started."""
        if self.carry_pending:   # the games restart: their carried moves are dropped
            # (after every stream's launches: the carry launch may have run on a caller's stream)
            torch.cuda.synchronize(self.dev)
            self.eng.c4_carry_discard(0, self.G, torch.cuda.current_stream(self.dev).cuda_stream)
            self.carry_pending = False
        self.roots.zero_()
        if self.traj is not None:
            self.traj.start(quota, games_cap=quota)

    def step(self, stream: int | None = None) -> torch.Tensor:
        """One move for every game (on torch's current stream unless given); returns the
        per-game results tensor (ONGOING = 2, IDLE = 3).  Finished games restart from the
        opening."""
        _room(self.traj, stream)
        self.step_search(stream)
        return self.step_finish(stream)

    def run(self, moves: int, stream: int | None = None, kernel_done=None) -> torch.Tensor:
        """`moves` moves for every game in ONE launch (zc_c4_selfplay_async: each game at its
        own pace, finished games refilled from the opening in the kernel), then the
        trajectory recording of every step, in step order — the same games, pool and labels
        as `moves` calls of step().  Needs the unlimited quota (start(None)): with a quota the
        refill depends on other slots' finishes, which step() decides once per step.
        Returns the per-step results [moves, G]; self.stats sums the moves' counters."""
        if self.traj is not None and self.traj.quota != _UNLIMITED:
            raise ValueError("run() plays without a game quota; use step() under simulate_games' quota")
        if self.vs is not None or self.ps is not None:
            raise ValueError("run() fuses the rollout search; network modes step()")
        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        if getattr(self, "_run_k", None) != moves:
            self._run_states = torch.zeros((moves, self.G, 3), dtype=torch.int64, device=self.dev)
            self._run_moves = torch.zeros((moves, self.G), dtype=torch.int16, device=self.dev)
            self._run_results = torch.zeros((moves, self.G), dtype=torch.int32, device=self.dev)
            self._run_k = moves
        self.eng.c4_selfplay_async(self.roots.data_ptr(), self.G, self.sims, self.c, self.bs, moves,
                                   self._run_states.data_ptr(), self._run_moves.data_ptr(),
                                   self._run_results.data_ptr(), self.stats.data_ptr(), stream=s)
        self.carry_pending = False   # carried moves were resumed first
        if kernel_done is not None:   # an event recorded after the launch, before the recording
            kernel_done.record()
        if self.record:
            self.traj.record_steps(self._run_states.data_ptr(), self._run_moves, self._run_results, moves, stream=s)
        self.results.copy_(self._run_results[-1])
        return self._run_results

    def run_pooled(self, budget: int, moves_cap: int, stream: int | None = None, kernel_done=None,
                   carry: bool = False) -> torch.Tensor:
        """`budget` moves shared by all games in ONE launch (zc_c4_selfplay_pooled_async): each
        game takes its next move from a device counter while the budget lasts, at most
        `moves_cap` moves.  A throughput schedule, not the reference's: scripts/train.py:151-170
        is lockstep (one move per unfinished game per call).  Game i's k-th move is the k-th move
        run() would play;
        how many moves each game gets follows the games' pace.  The trajectory recording
        replays the steps in order (slots without a k-th move: ZC_SLOT_SKIP, untouched).
        carry=True (zc_c4_selfplay_carry_async): once the budget is spent the in-flight moves
        stop at their next flush and carry over — the next run()/run_pooled() resumes them
        first; drain() finishes them; step() and the lockstep searches refuse until then.
        Returns the per-step results [moves_cap, G]; self.stats sums the launch's counters."""
        if self.traj is not None and self.traj.quota != _UNLIMITED:
            raise ValueError("run_pooled() plays without a game quota; use step() under simulate_games' quota")
        if self.vs is not None or self.ps is not None:
            raise ValueError("run_pooled() fuses the rollout search; network modes step()")
        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        if getattr(self, "_run_k", None) != moves_cap:
            self._run_states = torch.zeros((moves_cap, self.G, 3), dtype=torch.int64, device=self.dev)
            self._run_moves = torch.zeros((moves_cap, self.G), dtype=torch.int16, device=self.dev)
            self._run_results = torch.zeros((moves_cap, self.G), dtype=torch.int32, device=self.dev)
            self._run_k = moves_cap
        if getattr(self, "_ticket", None) is None:
            self._ticket = torch.zeros(2, dtype=torch.int32, device=self.dev)   # counter, most moves played
        self.eng.c4_selfplay_pooled_async(self.roots.data_ptr(), self.G, self.sims, self.c, self.bs, moves_cap,
                                          budget, self._ticket.data_ptr(), self._run_states.data_ptr(),
                                          self._run_moves.data_ptr(), self._run_results.data_ptr(),
                                          self.stats.data_ptr(), stream=s, carry=carry)
        self.carry_pending = bool(carry)
        if kernel_done is not None:
            kernel_done.record()
        if self.record:
            self.traj.record_steps(self._run_states.data_ptr(), self._run_moves, self._run_results, moves_cap,
                                   reached=self._ticket[1:], stream=s)
        return self._run_results

    def drain(self, stream: int | None = None) -> torch.Tensor:
        """Finish the moves run_pooled(carry=True) left in flight (a pooled launch with no
        budget: each carried move is resumed and finished, nothing new starts), recorded like
        any launch's moves.  Returns that launch's per-step results."""
        return self.run_pooled(0, 1, stream=stream)

    def step_search(self, stream: int | None = None) -> torch.Tensor:
        """The search half of a step (zc_c4_search_async); returns the results tensor the
        finish half will fill."""
        if self.carry_pending:
            raise RuntimeError("moves carried over by run_pooled(carry=True) are in flight: drain() first")
        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        if self.ps is not None or self.vs is not None:
            if self.ps is not None:
                mv, _, st = self.ps.enqueue(self.roots, self.sims, self.net_fn, temperature=self.temperature)
            else:
                mv, _, st = self.vs.enqueue(self.roots, self.sims, self.c, self.value_fn)
            self.moves.copy_(mv)
            self.stats.copy_(st)
        else:
            self.eng.c4_search_async(self.roots.data_ptr(), self.G, self.sims, self.c, self.bs,
                                     self.moves.data_ptr(), self.na.data_ptr(), self.stats.data_ptr(), stream=s)
        self.totals += self.stats[:, :2].sum(0)
        return self.results

    def adopt(self, other: "C4SelfPlay"):
        """Take over another pool's games in progress (positions and their recorded
        histories, game numbers; this pool's streams and pool stay its own) — e.g. a
        network-mode pool starting from a burned-in rollout pool's mixed game ages."""
        if self.carry_pending:   # its carried searches belong to the roots being replaced
            raise RuntimeError("moves carried over by run_pooled(carry=True) are in flight: drain() first")
        self.roots.copy_(other.roots)
        if self.traj is not None and other.traj is not None:
            t, o = self.traj, other.traj
            t.hist.copy_(o.hist)
            t.hmoves.copy_(o.hmoves)
            t.slot.copy_(o.slot)
            t.ctl[_native.ZC_TRAJ_NEXT] = o.ctl[_native.ZC_TRAJ_NEXT]

    def capture_step(self):
        """One whole step (search with its network, play, record) as a HIP graph; each
        replay plays the next move of every game."""
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):   # the network's kernels warmed outside the capture
            if self.ps is not None:
                _warm(self.ps, self.net_fn, self.sims)
            elif self.vs is not None:
                _warm(self.vs, self.value_fn, self.sims)
        torch.cuda.current_stream(self.dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.step()
        if self.traj is not None:
            self.traj.pinned = True   # the graph holds the pool's buffers from now on
        return g

    def step_finish(self, stream: int | None = None) -> torch.Tensor:
        """Play + evaluate the searched moves, record the positions, refill finished games."""
        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        self.eng.c4_play_async(self.roots.data_ptr(), self.G, self.moves.data_ptr(), self.results.data_ptr(),
                               reset=not self.record, stream=s)
        if self.record:
            self.moves16.copy_(self.moves)
            self.traj.record(self.roots.data_ptr(), self.moves16, self.results, stream=s)
        return self.results

    def take(self) -> TrajBatch:
        return self.traj.take()

    def take_positions(self) -> torch.Tensor:
        """Positions of the games finished since the last take, in start order: [n, 3] int64
        device rows (stones X, stones O, turn | Engine.get_dataset label << 32)."""
        return positions_of(self.take())

    def finished_games(self, batch: TrajBatch | None = None):
        """Host view of taken games (tests / inspection): (global slot id, moves, result,
        positions [n, 3] with labels) per game, in start order."""
        b = batch if batch is not None else self.take()
        return _host_games(b, self.first_id, lambda m: int(m))

    def close(self):
        self.eng.close()


def positions_of(b: TrajBatch) -> torch.Tensor:
    """A Connect4 TrajBatch as the exchange's rows: [n, 3] int64 (stones X, stones O,
    turn | Engine.get_dataset label << 32), on the batch's device."""
    rows = b.rows.clone()
    rows[:, 2] = (rows[:, 2] & 1) | (b.labels.to(torch.int64) << 32)
    return rows


def _host_games(b: TrajBatch, first_id: int, move_fn):
    rows, labels, moves = b.rows.cpu().numpy(), b.labels.cpu().numpy(), b.moves.cpu().numpy()
    out = []
    for gno, slot, res, off, n in b.games.cpu().numpy().tolist():
        pos = rows[off:off + n].copy()
        if pos.shape[1] == 3:
            pos[:, 2] = (pos[:, 2] & 1) | (labels[off:off + n].astype(np.int64) << 32)
        out.append((first_id + slot, [move_fn(m) for m in moves[off:off + n - 1]], res, pos))
    return out


class ChessSelfPlay:
    """Device-resident chess self-play: the chess form of `C4SelfPlay`.  G games live on one
    GPU as zc_chess_state rows; one `step()` searches every game — Value('crude_chess_score')
    in the search kernel, a value network between the stepwise select and backup kernels
    (`net=`), or the PUCT search with a policy + value network (`puct_net=`)
    — then ONE kernel plays the chosen moves, tests the new positions (check_win, stalemate,
    the fifty-move rule) and both sides' move histories (the repetition half of check_draw,
    chess_backend.cpp:416-441; histories in HBM) and refills finished games
    (zc_chess_play_step_async), and the recorder pools the finished games
    (zc_traj_record_async: Engine._evaluate's results, engine.py:148-153).  With the crude
    score, `run(K)` / `run_pooled(budget, cap)` play K moves per game (or a shared budget) in
    ONE launch (zc_chess_selfplay*_async) — the same games as K steps.  Nothing is read back
    per step; errors (a game longer than the history capacity, a search out of tree
    capacity, no move at a live root) are collected on the device and raised by `check()` /
    `take()`.  `capture_step()` records a whole step (search, network, play, record) in one
    HIP graph."""

    def __init__(self, games: int, sims: int, c: float = 1.4, batch_size: int = 32, seed: int = 0,
                 rank: int = 0, device: int = 0, policy: int = _native.ZC_POLICY_IMMEDIATE_VALUE,
                 freedom: float = 3.0, net=None, init_fen: str | None = None, games_cap: int | None = None,
                 hist_cap: int = 1024, puct_net=None, temperature: float = 1.0, puct_seed: int = 1,
                 puct_streams: int = 1, streams: int = 1):
        self.G, self.sims, self.c, self.bs = games, sims, c, batch_size
        self.policy, self.freedom = int(policy), float(freedom)
        self.dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.eng = _native.NativeEngine(max_games=games, max_sims=sims, max_batch=batch_size,
                                        device=self.dev.index or 0)
        self.eng.chess_reserve()
        self.first_id = rank * games
        self.eng.seed(0, [seed + self.first_id + g for g in range(games)])
        init = _native.chess_from_fen(init_fen) if init_fen else _native.chess_init()
        self.init_row = torch.from_numpy(np.frombuffer(init.tobytes(), np.uint8).reshape(1, 72).copy()).to(self.dev)
        self.roots = self.init_row.repeat(games, 1).contiguous()
        self.moves = torch.zeros(games, dtype=torch.int16, device=self.dev)
        self.na = torch.zeros((games, _native.CHESS_MAX_MOVES), dtype=torch.int32, device=self.dev)
        self.stats = torch.zeros((games, _native.STATS_FIELDS), dtype=torch.int64, device=self.dev)
        self.post = torch.zeros_like(self.roots)
        self.results = torch.zeros(games, dtype=torch.int32, device=self.dev)
        self.totals = torch.zeros(2, dtype=torch.int64, device=self.dev)   # expansions, depth sum since reset
        self.vs = self.value_fn = self.ps = self.net_fn = None
        self.temperature = float(temperature)
        if net is not None:
            from .valued import ChessValuedSearch, NetValue
            self.vs = ChessValuedSearch(self.eng, games, batch_size, leaves=False, policy=self.policy,
                                        freedom=self.freedom)
            self.value_fn = NetValue(net)
            if streams > 1:   # the games in parts on their own streams (valued._split_flushes)
                self.value_fn = [NetValue(net.replica() if hasattr(net, "replica") else net) for _ in range(streams)]
        if puct_net is not None:
            from .valued import ChessPuctSearch, PolicyNet
            # a network with the convolutional head takes the planes in its input layout straight
            # from the select kernel (no conversion launch per flush)
            self.ps = ChessPuctSearch(self.eng, games, batch_size, seed=puct_seed, leaves=False,
                                      planes_nhwc=bool(getattr(puct_net, "conv_head", False))
                                      and os.environ.get("ZC_PUCT_NHWC", "1") != "0")   # 0: A/B runs only
            self.net_fn = PolicyNet(puct_net)
            if puct_streams > 1:   # the games in parts on their own streams (valued._split_flushes)
                self.net_fn = [PolicyNet(puct_net.replica()) for _ in range(puct_streams)]
        self.hist_cap = hist_cap  # moves per side
        self.hist = torch.zeros((games, 2, self.hist_cap), dtype=torch.int16, device=self.dev)
        self.hlen = torch.zeros((games, 2), dtype=torch.int32, device=self.dev)
        self.err = torch.zeros(3, dtype=torch.int32, device=self.dev)
        b = _native.ChessPlayBuffers()
        b.d_roots, b.d_init, b.d_hist = self.roots.data_ptr(), self.init_row.data_ptr(), self.hist.data_ptr()
        b.d_hist_len, b.hist_cap, b.d_err = self.hlen.data_ptr(), self.hist_cap, self.err.data_ptr()
        self._pb = b
        max_len = 2 * self.hist_cap + 1
        cap = games_cap or max(8 * games, 1024)
        self.traj = Trajectories(games, self.init_row[0], max_len, cap, cap * 160, self.dev)

    def start(self, quota: int | None = None):
        self.roots.copy_(self.init_row.expand_as(self.roots))
        self.hlen.zero_()
        self.traj.start(quota, games_cap=quota)

    def _stream(self, stream):
        return stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream

    def step(self, stream: int | None = None) -> torch.Tensor:
        """One move for every game; returns the per-game results tensor (ONGOING = 2,
        IDLE = 3).  Finished games restart from the initial position."""
        _room(self.traj, stream)
        s = self._stream(stream)
        if self.ps is not None:
            mv, _, st = self.ps.enqueue(self.roots, self.sims, self.net_fn, temperature=self.temperature)
        elif self.vs is not None:
            mv, _, st = self.vs.enqueue(self.roots, self.sims, self.c, self.value_fn)
        else:
            self.eng.chess_search_async(0, self.G, self.roots.data_ptr(), self.sims, self.c, self.bs, self.policy,
                                        self.freedom, self.moves.data_ptr(), self.na.data_ptr(),
                                        self.stats.data_ptr(), s)
            mv, st = self.moves, self.stats
        if mv is not self.moves:
            self.moves.copy_(mv)
            self.stats.copy_(st)
        _native.check(_native.lib().zc_chess_play_step_async(
            self.G, ctypes.byref(self._pb), ctypes.c_void_p(self.moves.data_ptr()),
            ctypes.c_void_p(self.stats.data_ptr()), ctypes.c_void_p(self.post.data_ptr()),
            ctypes.c_void_p(self.results.data_ptr()), ctypes.c_void_p(s)))
        self.traj.record(self.post.data_ptr(), self.moves, self.results, stream=s)
        self.totals += self.stats[:, :2].sum(0)
        return self.results

    def adopt(self, other: "ChessSelfPlay"):
        """Take over another pool's games in progress: positions, both sides' move histories
        (the repetition draw), recorded histories and game numbers (same hist_cap)."""
        if other.hist_cap != self.hist_cap:
            raise ValueError("adopt() needs the same hist_cap")
        self.roots.copy_(other.roots)
        self.hist.copy_(other.hist)
        self.hlen.copy_(other.hlen)
        t, o = self.traj, other.traj
        t.hist.copy_(o.hist)
        t.hmoves.copy_(o.hmoves)
        t.slot.copy_(o.slot)
        t.ctl[_native.ZC_TRAJ_NEXT] = o.ctl[_native.ZC_TRAJ_NEXT]

    def capture_step(self):
        """One whole step (search with its network, play, record) as a HIP graph; each
        replay plays the next move of every game."""
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):   # the network's kernels warmed outside the capture
            if self.ps is not None:
                _warm(self.ps, self.net_fn, self.sims)
            elif self.vs is not None:
                _warm(self.vs, self.value_fn, self.sims)
        torch.cuda.current_stream(self.dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.step()
        if self.traj is not None:
            self.traj.pinned = True   # the graph holds the pool's buffers from now on
        return g

    def _run_buffers(self, moves: int):
        if getattr(self, "_run_k", None) != moves:
            self._run_states = torch.zeros((moves, self.G, 72), dtype=torch.uint8, device=self.dev)
            self._run_moves = torch.zeros((moves, self.G), dtype=torch.int16, device=self.dev)
            self._run_results = torch.zeros((moves, self.G), dtype=torch.int32, device=self.dev)
            self._run_k = moves

    def run(self, moves: int, stream: int | None = None, kernel_done=None) -> torch.Tensor:
        """Crude score: `moves` moves for every game in ONE launch (zc_chess_selfplay_async),
        then the multi-step recording — the same games, pool and labels as `moves` calls of
        step().  Returns the per-step results [moves, G]; self.stats sums the moves."""
        return self._launch(moves, None, stream, kernel_done)

    def run_pooled(self, budget: int, moves_cap: int, stream: int | None = None, kernel_done=None) -> torch.Tensor:
        """Crude score: `budget` moves shared by the games in ONE launch (at most moves_cap
        each; a throughput schedule, the reference's train.py is lockstep).  Game i's k-th
        move is the k-th move run() would play."""
        return self._launch(moves_cap, budget, stream, kernel_done)

    def _launch(self, moves, budget, stream, kernel_done):
        if self.vs is not None or self.ps is not None:
            raise ValueError("run()/run_pooled() fuse the crude-score search; network modes step()")
        if self.traj.quota != _UNLIMITED:
            raise ValueError("run() plays without a game quota; use step() under simulate_games' quota")
        s = self._stream(stream)
        self._run_buffers(moves)
        args = [self.eng.handle, 0, self.G, ctypes.byref(self._pb), self.sims, self.c, self.bs, self.policy,
                self.freedom, moves]
        outs = [ctypes.c_void_p(self._run_states.data_ptr()), ctypes.c_void_p(self._run_moves.data_ptr()),
                ctypes.c_void_p(self._run_results.data_ptr()), ctypes.c_void_p(self.stats.data_ptr()),
                ctypes.c_void_p(s)]
        reached = None
        if budget is None:
            _native.check(_native.lib().zc_chess_selfplay_async(*args, *outs))
        else:
            if getattr(self, "_ticket", None) is None:
                self._ticket = torch.zeros(2, dtype=torch.int32, device=self.dev)
            reached = self._ticket[1:]
            _native.check(_native.lib().zc_chess_selfplay_pooled_async(
                *args, int(budget), ctypes.c_void_p(self._ticket.data_ptr()), *outs))
        if kernel_done is not None:
            kernel_done.record()
        self.traj.record_steps(self._run_states.data_ptr(), self._run_moves, self._run_results, moves,
                               reached=reached, stream=s)
        return self._run_results

    def check(self):
        e = self.err.cpu().tolist()
        if e[0]:
            raise RuntimeError(f"a game exceeded {self.hist_cap} moves per side")
        if e[1] & 2:
            raise RuntimeError(f"a played position's legal-move list overflowed {_native.CHESS_MAX_MOVES} moves "
                               "(the game was not judged)")
        if e[1]:
            raise RuntimeError("chess search exceeded the tree's child-slot pool or depth limit")
        if e[2]:
            raise RuntimeError("no legal move at a non-terminal root")

    def take(self) -> TrajBatch:
        self.check()
        return self.traj.take()

    def finished_games(self, batch: TrajBatch | None = None):
        """(global slot id, moves ((fr, fc, tr, tc), value), result, rows [n, 9] int64) per
        game, in start order (host copies)."""
        b = batch if batch is not None else self.take()
        return _host_games(b, self.first_id, lambda m: _native.unpack_chess_move(int(m) & 0xFFFF))

    def close(self):
        self.eng.close()


def simulate_games(pool, total_games: int, max_steps: int | None = None, check_every: int = 4) -> list[int]:
    """scripts/train.py:simulate_games (:151-170) on a device pool (C4SelfPlay or
    ChessSelfPlay): games 0..min(total, G)-1 start in slots 0.., a finished game's slot starts
    the next game while fewer than `total_games` have started, and every started game is
    played to its end.  Returns the results by game number (start order), as the
    reference's `final` list; the games' trajectories stay in the pool (`pool.take()`)."""
    if total_games < 0:
        raise ValueError("total_games must be >= 0")
    pool.start(total_games)
    steps = 0
    while total_games and (steps % check_every or pool.traj.finished() < total_games):
        if max_steps is not None and steps >= max_steps:
            raise RuntimeError(f"{pool.traj.finished()} of {total_games} games finished in {max_steps} steps")
        pool.step()   # with a quota, step() grows the trajectory pool first (ensure_room)
        steps += 1
    pool.last_batch = pool.take()
    res = pool.last_batch.results()
    assert len(res) == total_games, (len(res), total_games)
    return res


def schedule_hyperparams(cycle: int, *, games_cap: int = 2000, sims_cap: int = 800, init_lr: float = 3e-4,
                         lr_decay: float = 0.95, lr_floor: float = 1e-5) -> dict:
    """scripts/train.py:schedule_hyperparams (:173-188): the self-play games, simulations per
    move and exploration constant of training cycle `cycle`, and its learning rate."""
    games = min(games_cap, 500 * (cycle + 1))
    sims = int(min(100 * (1.2 ** cycle), sims_cap))
    c_val = max(1.25, 2.5 * (0.97 ** cycle))
    lr = max(init_lr * (lr_decay ** cycle), lr_floor)
    return {"games": games, "simulations": sims, "c_puct": c_val, "lr": lr}


def gather_positions(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather variable-length [n_r, ...] position rows from every rank (rank order; e.g.
    [n, 3] int64 Connect4 rows with labels, or chess rows): an all_gather of the counts,
    then of payloads padded to the largest count."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)


class ReplayBuffer:
    """scripts/train.py:_update_replay (:27-50): the training set of a cycle = a uniform
    sample (without replacement) of 30 % of everything seen before, then all new data.

    Works on numpy arrays or device tensors (the pooled positions stay on the GPU: the old
    data is concatenated and indexed on the device).  The sample indices come from numpy's
    GLOBAL generator, `np.random.choice(len(old), k, replace=False)`, exactly the
    reference's call — so after the same `np.random.seed` the same rows are drawn; pass
    `seed` for a private generator instead."""

    def __init__(self, frac_old: float = 0.30, seed: int | None = None):
        self.frac_old = frac_old
        self.states, self.values = [], []
        self.rng = np.random.default_rng(seed) if seed is not None else None

    @staticmethod
    def _cat(xs):
        return torch.cat(xs, dim=0) if torch.is_tensor(xs[0]) else np.concatenate(xs, axis=0)

    def update(self, states_new, values_new):
        if not self.states:
            self.states.append(states_new)
            self.values.append(values_new)
            return states_new, values_new
        old_s, old_v = self._cat(self.states), self._cat(self.values)
        k = int(self.frac_old * len(old_s))
        if k > 0:
            idx = (self.rng.choice(len(old_s), k, replace=False) if self.rng is not None
                   else np.random.choice(len(old_s), k, replace=False))
            if torch.is_tensor(old_s):
                idx = torch.from_numpy(idx).to(old_s.device)
            ss, sv = old_s[idx], old_v[idx]
        else:
            ss, sv = old_s[:0], old_v[:0]
        self.states.append(states_new)
        self.values.append(values_new)
        return self._cat([ss, states_new]), self._cat([sv, values_new])
