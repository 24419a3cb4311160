"""Device-side plumbing shared by the reference-API modules: engine ownership with capacity
growth, Python `random` <-> per-game MT19937 stream hand-off, state conversion."""
from __future__ import annotations

import random
import threading

import numpy as np

from .. import _native

_lock = threading.RLock()
_scratch = {}


class GrowingEngine:
    """A NativeEngine that is re-created larger when a request exceeds its capacity; the
    games' random streams are carried over, so growth is invisible to callers."""

    def __init__(self, games: int = 1, sims: int = 1, batch: int = 32, device: int = 0):
        self.device = device
        self.eng = None
        self.cap = (0, 0, 0)
        self.seeded = {}
        self.lock = threading.RLock()
        self.ensure(games, sims, batch)

    def ensure(self, games: int, sims: int, batch: int) -> _native.NativeEngine:
        with self.lock:
            g0, s0, b0 = self.cap
            if self.eng is not None and games <= g0 and sims <= s0 and batch <= b0:
                return self.eng
            g = max(games, 2 * g0 if games > g0 else g0, 1)
            s = max(sims, s0)
            b = max(batch, b0)
            saved = {}
            if self.eng is not None:
                for game in range(g0):
                    saved[game] = self.eng.get_rng_state(game)
                self.eng.close()
            self.eng = _native.NativeEngine(max_games=g, max_sims=s, max_batch=b, device=self.device)
            for game, (mt, idx) in saved.items():
                self.eng.set_rng_state(game, mt, idx)
            self.cap = (g, s, b)
            return self.eng


def scratch(sims: int, batch: int, device: int = 0, depth: int = 0) -> GrowingEngine:
    """One-game engine for calls that consume Python's global `random` (get_move, Value).
    `depth` is the caller's get_move nesting level on its thread: a host plugin (policy,
    value, backend) that itself calls get_move in the middle of a search gets the engine of
    the next level, so the outer search's tree — and its engine's capacity — stay untouched.
    Do not call `ensure` on another level's engine while a search runs on it."""
    key = device if depth == 0 else (device, "nested", depth)
    with _lock:
        ge = _scratch.get(key)
        if ge is None:
            ge = _scratch[key] = GrowingEngine(1, sims, batch, device)
    return ge


def value_engine(device: int = 0) -> GrowingEngine:
    """The one-game engine of direct Value.batch calls (Value('random_rollout') on a list of
    states): separate from the get_move scratch engine, since a host plugin may call such a
    Value in the middle of a search on the scratch engine (growing it there would destroy the
    search's tree)."""
    with _lock:
        key = ("value", device)
        ge = _scratch.get(key)
        if ge is None:
            ge = _scratch[key] = GrowingEngine(1, 1, 1, device)
        return ge


def python_random_state():
    version, internal, gauss = random.getstate()
    return np.asarray(internal[:624], dtype=np.uint32), int(internal[624]), version, gauss


def set_python_random_state(mt, idx, version, gauss):
    random.setstate((version, tuple(int(x) for x in mt) + (int(idx),), gauss))


class game_stream:
    """Python's global `random` becomes engine game g's device stream for the duration of the
    block — a host plugin called where the reference calls it (value.batch once per flush,
    mcts.cpp:116) draws the words the reference would draw, after the device's own — then the
    advanced stream goes back to the device and Python's previous state is restored.
    random.gauss's cached second value travels with the game (eng.py_gauss)."""

    def __init__(self, eng, g: int):
        self.eng, self.g = eng, int(g)

    def __enter__(self):
        self.saved = random.getstate()
        mt, idx = self.eng.get_rng_state(self.g)
        gauss = getattr(self.eng, "py_gauss", {}).get(self.g)
        set_python_random_state(mt, idx, self.saved[0], gauss)
        return self

    def __exit__(self, *exc):
        mt, idx, _, gauss = python_random_state()
        random.setstate(self.saved)
        if exc[0] is None:
            self.eng.set_rng_state(self.g, mt, idx)
            if not hasattr(self.eng, "py_gauss"):
                self.eng.py_gauss = {}
            self.eng.py_gauss[self.g] = gauss
        return False


def c4_roots(states, c4) -> np.ndarray:
    out = np.zeros(len(states), _native.C4_STATE_DTYPE)
    for i, s in enumerate(states):
        s0, s1, t = c4.to_zc(s)
        out[i]["stones"] = (s0, s1)
        out[i]["turn"] = t
    return out
