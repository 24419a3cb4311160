"""`get_move` — drop-in for the reference's search core (engine/mcts/__init__.py,
engine/mcts/src/bindings_mcts.cpp:9-11, engine/mcts/src/mcts.cpp:102-160).

    get_move(state, value, policy, backend, simulations=1000, c=1.4, batch_size=32) -> move

The whole search runs on the GPU (libzeroclone_amd.so; paths in _search.py).  Every random
number is drawn from Python's global `random` stream, in the reference's order, and the
stream is handed back advanced by exactly what the reference would have consumed — so
`random.seed(s); get_move(...)` returns the reference's move and leaves `random` in the
reference's state.  The GIL is released during device calls (ctypes).

Supported plugins: the Connect4 and chess backends (this package's, or the reference's —
states with the same fields), Policy('random') / Policy('immediate_value') on the device, any
other policy callable (called on the host at each expansion, the tree still on the device:
_search.c4_host_policy_moves / chess_host_policy_moves), and any value object:
Value('random_rollout') runs on the device (Connect4: inside the search kernel; chess: a
rollout kernel between the select and backup kernels, the leaves' move histories rebuilt from
the root's and the path), Value('crude_chess_score') inside the chess search kernel, network
values on the device between the select and backup kernels, and any other object's
value.batch(states, backend=backend) on the host once per flush, exactly where the reference
calls it (mcts.cpp:116) — with Python's `random` handed the game's device stream for the
call (_device.game_stream), so a value that draws random numbers draws the reference's, and
chess leaves carrying their move histories.

Any other game backend (the six functions of engine/README.md:17-24) searches with the tree
on the device (zc_gen_*) and the backend, policy and value called on the host, in the
reference's order, drawing from Python's `random` themselves (_search.generic_moves).
There is no CPU search.

Threads (the reference fans get_move out from a ThreadPoolExecutor with the GIL released,
engine/engine.py:131-138, engine/mcts/src/bindings_mcts.cpp:11): calls from several threads
are serialised by the scratch engine's lock, each call taking Python's global `random`
at its start and handing it back advanced at its end, so the threads' calls consume the one
global stream as consecutive blocks — one of the interleavings the reference's shared stream
allows.  The GIL is released while the device works (ctypes calls and stream waits), so
other threads — a network batcher, the callers' own work — keep running.  Re-entry: a host
plugin that calls get_move during a search (same thread) gets a separate engine per nesting
level (_device.scratch(depth=...)), so the outer search's tree is not touched.

`trace`: None, or a list to which every call appends (depth, random state at entry,
random state at exit, move, state) inside its lock — the record the threaded tests replay.
"""
from __future__ import annotations

import random
import threading

from . import _device, _search

__all__ = ["get_move"]

trace = None
_tls = threading.local()


def _plugin_check(state, value, policy, backend):
    game = _search.game_of(backend, state)
    _search.policy_of(policy)
    _search.value_kind(value)
    # every combination runs: e.g. crude_chess_score on Connect4 goes to the host value path
    # and fails where the reference's does (chr() of a board row, value_functions.py:54)
    return game


def get_move(state, value, policy, backend, simulations=1000, c=1.4, batch_size=32):
    game = _plugin_check(state, value, policy, backend)
    if simulations < 1:
        raise ValueError("simulations must be >= 1 (the reference indexes moves[-1] here)")
    if batch_size < 1:
        raise ValueError("batch_size must be >= 1")
    depth = getattr(_tls, "depth", 0)
    ge = _device.scratch(simulations, batch_size, depth=depth)
    _tls.depth = depth + 1
    try:
        with ge.lock:
            entry = random.getstate() if trace is not None else None
            mv = _get_move_locked(ge, game, state, value, policy, backend, simulations, c, batch_size)
            if trace is not None:
                trace.append((depth, entry, random.getstate(), mv, state))
            return mv
    finally:
        _tls.depth = depth


def _get_move_locked(ge, game, state, value, policy, backend, simulations, c, batch_size):
    eng = ge.ensure(1, simulations, batch_size)
    if game == "generic":   # any backend: the tree on the device, the plugins on the host
        return _search.generic_moves(eng, state, simulations, c, batch_size, value, policy, backend)
    if _search.policy_of(policy)[0] == _search.HOST_POLICY:
        if game == "connect4":
            from .games.connect4 import c4_backend as c4
            return _search.c4_host_policy_moves(eng, [0], _device.c4_roots([state], c4), simulations, c,
                                                batch_size, value, policy, backend)[0]
        mv = _search.chess_host_policy_moves(eng, [0], [state], simulations, c, batch_size, value, policy,
                                             backend)[0]
        if mv is None:
            raise ValueError("root has no legal move (the reference indexes moves[-1] here)")
        return mv
    mt, idx, ver, gauss = _device.python_random_state()
    eng.set_rng_state(0, mt, idx)
    eng.py_gauss = {0: gauss}
    if game == "connect4":
        from .games.connect4 import c4_backend as c4
        mv = _search.c4_moves(eng, [0], _device.c4_roots([state], c4), simulations, c, batch_size, value,
                              backend)[0]
    else:
        mv = _search.chess_moves(eng, [0], [state], simulations, c, batch_size, value, policy, backend)[0]
        if mv is None:
            raise ValueError("root has no legal move (the reference indexes moves[-1] here)")
    mt, idx = eng.get_rng_state(0)
    _device.set_python_random_state(mt, idx, ver, eng.py_gauss.get(0, gauss))
    return mv
