"""Leaf evaluators with the reference's interface (engine/value_functions.py:8-130).

`Value('random_rollout')` runs on the GPU: `batch(states, backend=)` rolls the states out
in order on one CPython-compatible MT19937 stream taken from (and returned to) Python's
global `random` module — the same numbers, consumed in the same order, as the reference's
`[self(s) for s in states]` (value_functions.py:20-22, 35-45).  Inside `mcts.get_move` /
`Engine` the value object is not called at all: its name selects the fused on-device
rollout of the search kernel.
"""
from __future__ import annotations

from . import _device

SUPPORTED = ("random_rollout",)


class Value:
    def __init__(self, name, **kwargs):
        self.name = name
        self.init_args = kwargs
        if name not in SUPPORTED:
            raise NotImplementedError(
                f"value function {name!r} is not implemented on the MI355X path yet "
                f"(supported: {', '.join(SUPPORTED)}); see DESIGN.md 'Out of scope / next'")

    def __call__(self, state, **kwargs):
        return self.batch([state], **kwargs)[0]

    def batch(self, states, **kwargs):
        backend = (self.init_args | kwargs).get("backend")
        return getattr(self, self.name)(list(states), backend)

    def random_rollout(self, states, backend):
        if getattr(backend, "ZC_GAME", None) != "connect4" and not _looks_like_c4(backend, states):
            raise NotImplementedError("random_rollout is implemented for the Connect4 backend only")
        from .games.connect4 import c4_backend as c4
        if not states:
            return []
        ge = _device.scratch(1, 32)
        with ge.lock:
            eng = ge.ensure(1, 1, 32)
            mt, idx, ver, gauss = _device.python_random_state()
            eng.set_rng_state(0, mt, idx)
            vals, _ = eng.c4_rollouts(_device.c4_roots(states, c4), game=0)
            mt, idx = eng.get_rng_state(0)
            _device.set_python_random_state(mt, idx, ver, gauss)
        return [int(v) for v in vals]


def _looks_like_c4(backend, states):
    from .games.connect4 import c4_backend as c4
    return getattr(backend, "__name__", "").endswith("c4_backend") and all(c4.is_state(s) for s in states)
