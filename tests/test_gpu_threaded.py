"""The drop-in get_move under the reference's threaded caller (SURVEY.md §8(b) "Threading").

The reference's Engine fans `mcts.get_move` out over a ThreadPoolExecutor
(/root/reference/engine/engine.py:119-138) with the GIL released around the search
(engine/mcts/src/bindings_mcts.cpp:11); its network Value coalesces requests from all those
threads on one worker thread (engine/value_functions.py:20-32, 61-99).  INTEGRATION.md §1 tells
a user to swap engine/mcts for zeroclone_amd.engine.mcts and keep that Engine, so this is the
path a drop-in user runs.  `RefShapedEngine` below restates that fan-out around
zeroclone_amd.engine.mcts.get_move.

Checked for Connect4 (random_rollout on the device; a host value drawing from `random`; a
reference-shaped network value blocking on a batch worker thread; a host value that itself
calls get_move — re-entry) and chess (crude_chess_score on the device):
  * no deadlock (the fan-out finishes within a timeout);
  * every move is legal in its position;
  * the top-level calls consumed Python's global stream as consecutive blocks (each call's
    entry state is the previous call's exit state: mcts.trace, recorded inside the search
    lock), and replaying every call serially from its recorded entry state gives the same
    move and the same exit state;
  * another Python thread keeps running while a long device search is in flight (the GIL is
    released).
"""
import queue
import random
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from fallback_values import ShuffleValue

pytestmark = pytest.mark.gpu

TIMEOUT = 240


class RefShapedEngine:
    """engine/engine.py:119-138's play_mcts / play_mcts_parallel around the drop-in get_move
    (per-game states, values[turn], a terminal check before the search, the move played
    after; the legality check takes Connect4's (col, 0) moves, unlike the reference's
    _is_legal)."""

    def __init__(self, backend, value, policy, states):
        self.backend, self.policy = backend, policy
        self.values = [value, value]
        self.states = list(states)
        self.results = {}

    def _evaluate(self, s):
        if self.backend.check_win(s):
            return s.turn * 2 - 1
        if self.backend.check_draw(s):
            return 0
        return None

    def play_mcts(self, idx, sims, c, bs):
        from zeroclone_amd.engine import mcts
        s = self.states[idx]
        r = self._evaluate(s)
        if r is not None:
            return r
        mv = mcts.get_move(s, self.values[s.turn], self.policy, self.backend, sims, c, bs)
        if mv not in self.backend.get_legal_moves(s):
            raise AssertionError(f"illegal move {mv}")
        self.states[idx] = self.backend.play_move(s, mv)
        return self._evaluate(self.states[idx])

    def play_mcts_parallel(self, idxs, sims, c, bs, max_workers=8):
        out = {}
        with ThreadPoolExecutor(max_workers=max_workers) as ex:
            futs = {ex.submit(self.play_mcts, i, sims, c, bs): i for i in idxs}
            for f in futs:
                out[futs[f]] = f.result(timeout=TIMEOUT)
        return out


class QueueNetValue:
    """A network Value shaped like the reference's (value_functions.py:20-32, 61-99): batch()
    puts each leaf's state_to_tensor planes on a request queue with a reply queue and blocks on
    the replies; a daemon worker drains up to batch_size requests from ALL threads, stacks
    them and evaluates them on the GPU.  The "network" is an integer-weight linear layer in
    float64 followed by tanh: its sums are exact, so a leaf's value does not depend on which
    requests shared its batch (the serial replay can reproduce it)."""

    def __init__(self, batch_size=64):
        g = torch.Generator().manual_seed(11)
        self.w = torch.randint(-9, 10, (84,), generator=g).double().cuda()
        self.batch_size = batch_size
        self.req = queue.Queue()
        self.batches = []
        threading.Thread(target=self._worker, daemon=True).start()

    def _worker(self):
        while True:
            batch = [self.req.get()]
            while len(batch) < self.batch_size:
                try:
                    batch.append(self.req.get_nowait())
                except queue.Empty:
                    break
            arrs, qs = zip(*batch)
            x = torch.from_numpy(np.stack(arrs).reshape(len(arrs), -1).astype(np.float64)).cuda()
            out = torch.tanh((x @ self.w) / 16.0).cpu().tolist()
            self.batches.append(len(batch))
            for q, v in zip(qs, out):
                q.put(v)

    def batch(self, states, **kw):
        backend = kw["backend"]
        qs = []
        for s in states:
            q = queue.Queue()
            self.req.put((np.asarray(backend.state_to_tensor(s), np.float32), q))
            qs.append(q)
        return [q.get(timeout=TIMEOUT) for q in qs]


class NestedValue:
    """A host value that calls get_move itself (re-entry on the same thread, mid-search):
    each flush runs a 24-simulation rollout search from its first leaf and folds the chosen
    column into the values.  Before round 5 the nested call would have reused — and could
    have regrown — the engine holding the outer search's tree."""

    def batch(self, states, **kw):
        from zeroclone_amd.engine import Policy, Value, mcts
        backend = kw["backend"]
        first = states[0]
        col = -1
        if not backend.check_win(first) and not backend.check_draw(first):
            col = mcts.get_move(first, Value("random_rollout"), Policy("random"), backend, 24, 1.4, 8)[0]
        return [((sum(ch != " " for row in s.board for ch in row) * 7 + col) % 13 - 6) / 7.0 for s in states]


def c4_positions(n, seed):
    from zeroclone_amd.engine.games.connect4 import c4_backend as c4
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        s = c4.create_init_state()
        for _ in range(rng.randrange(0, 14)):
            if c4.check_win(s) or c4.check_draw(s):
                break
            s = c4.play_move(s, rng.choice(sorted(c4.get_legal_moves(s))))
        if not c4.check_win(s) and not c4.check_draw(s):
            out.append(s)
    return out


def chess_positions(n, seed):
    from zeroclone_amd.engine.games.chess import chess_backend as cb
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        s = cb.create_init_state()
        for _ in range(rng.randrange(0, 8)):
            moves = cb.get_legal_moves(s)
            if not moves:
                break
            s = cb.play_move(s, rng.choice(moves))
        if cb.get_legal_moves(s) and not cb.check_draw(s):
            out.append(s)
    return out


def _plugins(kind):
    from zeroclone_amd.engine import Policy, Value
    from zeroclone_amd.engine.games.chess import chess_backend as cb
    from zeroclone_amd.engine.games.connect4 import c4_backend as c4
    if kind == "c4_rollout":
        return c4, Value("random_rollout"), Policy("random"), c4_positions(16, 1), (160, 32)
    if kind == "c4_host_value":
        return c4, ShuffleValue(), Policy("random"), c4_positions(16, 2), (96, 16)
    if kind == "c4_queue_net":
        return c4, QueueNetValue(), Policy("random"), c4_positions(16, 3), (128, 32)
    if kind == "c4_nested":
        return c4, NestedValue(), Policy("random"), c4_positions(16, 4), (64, 16)
    if kind == "chess_crude":
        return cb, Value("crude_chess_score"), Policy("random"), chess_positions(16, 5), (96, 32)
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["c4_rollout", "c4_host_value", "c4_queue_net", "c4_nested", "chess_crude"])
def test_threaded_fanout_is_a_serialisation_of_get_move(kind):
    from zeroclone_amd.engine import mcts
    backend, value, policy, states, (sims, bs) = _plugins(kind)
    eng = RefShapedEngine(backend, value, policy, states)
    random.seed(4321)
    s0 = random.getstate()
    mcts.trace = []
    done = {}

    def run():
        for _ in range(2):
            done.setdefault("rounds", []).append(eng.play_mcts_parallel(range(len(states)), sims, 1.4, bs))

    try:
        t = threading.Thread(target=run, daemon=True)
        t.start()
        t.join(TIMEOUT)
        assert not t.is_alive(), f"{kind}: the threaded fan-out did not finish in {TIMEOUT} s (deadlock?)"
        trace = mcts.trace
    finally:
        mcts.trace = None
    assert len(done["rounds"]) == 2
    top = [e for e in trace if e[0] == 0]
    assert len(top) == 2 * len(states) - sum(r is not None for r in done["rounds"][0].values())
    if kind == "c4_nested":
        assert len(trace) > len(top)            # the nested searches ran (and are in the trace)
    if kind == "c4_queue_net":
        assert sum(value.batches) > 0
    # the calls took the one global stream as consecutive blocks ...
    assert top[0][1] == s0
    for a, b in zip(top, top[1:]):
        assert b[1] == a[2]
    # ... and each equals a serial get_move from its recorded entry state
    for depth, entry, exit_, mv, st in top:
        assert mv in backend.get_legal_moves(st)
        random.setstate(entry)
        assert mcts.get_move(st, value, policy, backend, sims, 1.4, bs) == mv
        assert random.getstate() == exit_


def test_get_move_releases_the_gil():
    """A long device search (one Connect4 game, 30,000 simulations) in the main thread: a
    pure-Python counter thread keeps at least a quarter of its idle rate meanwhile."""
    from zeroclone_amd.engine import Policy, Value, mcts
    from zeroclone_amd.engine.games.connect4 import c4_backend as c4
    st = c4.create_init_state()
    value, policy = Value("random_rollout"), Policy("random")
    random.seed(9)
    mcts.get_move(st, value, policy, c4, 30000, 1.4, 32)      # warm: engine growth, code load
    stop = threading.Event()
    count = [0]

    def spin():
        while not stop.is_set():
            count[0] += 1

    th = threading.Thread(target=spin, daemon=True)
    th.start()
    t0, c0 = time.perf_counter(), count[0]
    time.sleep(0.1)
    idle_rate = (count[0] - c0) / (time.perf_counter() - t0)
    t0, c0 = time.perf_counter(), count[0]
    random.seed(10)
    mcts.get_move(st, value, policy, c4, 30000, 1.4, 32)
    dt = time.perf_counter() - t0
    busy_rate = (count[0] - c0) / dt
    stop.set()
    th.join(5)
    print(f"search {dt * 1e3:.1f} ms; counter {busy_rate:.3g}/s during vs {idle_rate:.3g}/s idle")
    assert dt > 0.005
    assert busy_rate > 0.25 * idle_rate


def test_reentry_matches_the_oracle():
    """A nested get_move (a host value calling it mid-search, on the same thread) against the
    oracle doing the same: the outer search's flush callback runs the oracle's get_move on the
    SAME stream (the reference's nested call draws from the one global `random`).  Outer
    move, root choice and the stream afterwards must agree; before round 5 the nested call
    reused the engine that held the outer search's tree."""
    import oracle
    from zeroclone_amd.engine import Policy, mcts
    from zeroclone_amd.engine.games.connect4 import c4_backend as c4
    for k, st in enumerate(c4_positions(6, 77)):
        board = "".join("." if ch == " " else ch for row in st.board for ch in row)
        mt = oracle.MT(500 + k)

        def cb(boards, turns):
            col = -1
            if not oracle.check_win(boards[0], turns[0]) and not oracle.check_draw(boards[0]):
                col = oracle.get_move_mt(boards[0], turns[0], mt, 24, 1.4, 8)[0]
            return [((sum(ch != "." for ch in b) * 7 + col) % 13 - 6) / 7.0 for b in boards]
        want, _, _ = oracle.get_move_valued(board, st.turn, mt, 200, 1.4, 16, cb)
        random.seed(500 + k)
        got = mcts.get_move(st, NestedValue(), Policy("random"), c4, 200, 1.4, 16)
        assert got == (want, 0), k
        assert random.getrandbits(32) == mt.u32(), k
