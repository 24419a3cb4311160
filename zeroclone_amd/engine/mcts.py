"""`get_move` — drop-in for the reference's search core (engine/mcts/__init__.py,
engine/mcts/src/bindings_mcts.cpp:9-11, engine/mcts/src/mcts.cpp:102-160).

    get_move(state, value, policy, backend, simulations=1000, c=1.4, batch_size=32) -> move

The whole search runs on the GPU (zc_c4_search_games in libzeroclone_amd.so).  Every random
number is drawn from Python's global `random` stream, in the reference's order, and the
stream is handed back advanced by exactly what the reference would have consumed — so
`random.seed(s); get_move(...)` returns the reference's move and leaves `random` in the
reference's state.  The GIL is released during the device call (ctypes).

Supported plugins: the Connect4 backend (this package's c4_backend, or any module with the
reference c4_backend's State layout) and Policy('random').  Value('random_rollout') runs
entirely on the device (zc_c4_search_games); any other value object runs through the
stepwise search (zc_c4_ext_*, zeroclone_amd/valued.py): the tree stays on the GPU and
value.batch(states, backend=backend) is called on the host once per flush, exactly where
the reference calls it (mcts.cpp:116).  Such a value function must not draw from `random`
(the reference's NN and crude-score values do not).  Anything else raises
NotImplementedError: there is no CPU search.
"""
from __future__ import annotations

import numpy as np

from . import _device

__all__ = ["get_move"]


def _plugin_check(state, value, policy, backend):
    from .games.connect4 import c4_backend as c4
    game = getattr(backend, "ZC_GAME", None)
    if game is None and getattr(backend, "__name__", "").endswith("c4_backend") and c4.is_state(state):
        game = "connect4"
    if game != "connect4":
        raise NotImplementedError(f"backend {getattr(backend, '__name__', backend)!r}: only Connect4 runs on the "
                                  "MI355X search path so far (see DESIGN.md)")
    pname = getattr(policy, "name", None)
    if pname != "random":
        raise NotImplementedError(f"policy {pname!r}: only Policy('random') is implemented on the GPU")
    if not callable(getattr(value, "batch", None)):
        raise NotImplementedError("value objects must provide .batch(states, backend=) (value_functions.py:20)")
    return c4


def _device_rollouts(value) -> bool:
    return getattr(value, "name", None) == "random_rollout" and not hasattr(value, "_req_q")


def get_move(state, value, policy, backend, simulations=1000, c=1.4, batch_size=32):
    c4 = _plugin_check(state, value, policy, backend)
    if simulations < 1:
        raise ValueError("simulations must be >= 1 (the reference indexes moves[-1] here)")
    if batch_size < 1:
        raise ValueError("batch_size must be >= 1")
    roots = _device.c4_roots([state], c4)
    ge = _device.scratch(simulations, batch_size)
    with ge.lock:
        eng = ge.ensure(1, simulations, batch_size)
        mt, idx, ver, gauss = _device.python_random_state()
        eng.set_rng_state(0, mt, idx)
        if _device_rollouts(value):
            mv, _, _ = eng.c4_search_games([0], roots, simulations, c, batch_size)
        else:
            mv = _valued_search(eng, roots, simulations, c, batch_size, value, backend)
        mt, idx = eng.get_rng_state(0)
        _device.set_python_random_state(mt, idx, ver, gauss)
    return (int(mv[0]), 0)


def _valued_search(eng, roots, sims, c, bs, value, backend):
    import torch
    from ..valued import C4ValuedSearch, HostValue
    vs = C4ValuedSearch(eng, 1, bs, planes=False)
    r = torch.from_numpy(roots.view(np.int64).reshape(1, 3).copy()).to(vs.dev)
    mv, _, st = vs.run(r, sims, c, HostValue(value, backend))
    st = st.cpu().numpy()
    if st[0, 5]:
        raise ValueError(f"invalid root for the search (status {int(st[0, 5])})")
    return mv.cpu().numpy()
