"""`Engine` — the reference's multi-game orchestrator (engine/engine.py:10-161), with the
search of every game running on the GPU.

Same constructor, state list, history, dataset labelling and method names.  Differences,
all deliberate and documented in DESIGN.md:

* `play_mcts_parallel(idxs, ...)` is ONE batched device search over all those games (the
  reference fans out Python threads, engine.py:131-138); results have the same shape.
* Random numbers: every game owns a CPython-compatible MT19937 stream on the device,
  seeded `random.seed(config['seed'] + idx)` (default seed 0), so a game's moves do not
  depend on which other games are searched with it or on thread timing.  With
  `rng: global` in the config the engine instead consumes Python's global `random`, game by
  game in index order — the reference's serial behaviour.
* `play_move` accepts Connect4 moves: the reference's `_is_legal` unpacks `mv[0]` as a chess
  4-tuple and raises TypeError for `(col, 0)` (engine.py:155-157).
* Chess games search on the device too (crude_chess_score in-kernel; network values between
  the select and backup kernels); the game's move histories stay on the host State.
"""
from __future__ import annotations

import importlib
from dataclasses import dataclass, field
from typing import Any, Callable, Optional, Sequence

import yaml

from . import _device
from .policy_functions import Policy
from .value_functions import Value


@dataclass
class History:
    states: list[Any] = field(default_factory=list)
    result: Optional[int] = None


class Engine:
    def __init__(self, config: str | dict, *, value_functions: Sequence[Callable] | None = None, device: int = 0):
        if isinstance(config, str):
            with open(config, "r") as fh:
                self.config = yaml.safe_load(fh)
        else:
            self.config = config
        # engine.py:26 imports engine.games.<game>.<backend>; a dotted `backend` names any module
        name = self.config["backend"]
        self.backend = importlib.import_module(
            name if "." in name else f"zeroclone_amd.engine.games.{self.config['game']}.{name}")
        self.policy = Policy(name=self.config.get("policy_functions"), **self.config.get("policy", {}))
        if value_functions is None:
            val = Value(self.config.get("value_function"), **self.config.get("value", {}))
            self.values = [val, val]
        else:
            if len(value_functions) != 2:
                raise ValueError("value_functions must have length 2")
            self.values = list(value_functions)
        init_state = self.backend.create_init_state()
        self.threads = self.config.get("threads", 1)
        self.states = [init_state for _ in range(self.threads)]
        self.history = [History(states=[init_state], result=None) for _ in range(self.threads)]
        self.seed = int(self.config.get("seed", 0))
        self.rng_mode = self.config.get("rng", "per_game")
        if self.rng_mode not in ("per_game", "global"):
            raise ValueError("config 'rng' must be 'per_game' or 'global'")
        self.device = device
        self._dev = None
        self._seeded = 0   # games [0, _seeded) have their streams on the device

    # ------------------------------------------------------------------ basic functions
    def add_game(self, init_state=None):
        state = init_state or self.backend.create_init_state()
        self.states.append(state)
        self.history.append(History(states=[state], result=None))
        return len(self.states) - 1

    def get_state(self, idx=0):
        return self.states[idx]

    def get_hist(self, idx=0):
        return list(self.history[idx].states)

    # ------------------------------------------------------------------ dataset helper
    def get_dataset(self):
        """Finished games' positions with side-to-move labels (engine.py:60-89)."""
        import numpy as np
        state_arrays, labels = [], []
        for h in self.history:
            if h.result is None:
                continue
            factor = 0 if h.result == 0 else -1
            entry = []
            for s in h.states:
                state_arrays.append(self.backend.state_to_tensor(s).astype(np.float32))
                entry.append(factor)
                factor = -factor
            labels += list(reversed(entry))
        if not state_arrays:
            dummy = self.backend.state_to_tensor(self.backend.create_init_state())
            return np.empty((0,) + dummy.shape, dtype=np.float32), np.empty((0,), dtype=np.float32)
        return np.stack(state_arrays, axis=0), np.array(labels, dtype=np.float32)

    # ------------------------------------------------------------------ game play
    def legal_moves(self, idx=0):
        return self.backend.get_legal_moves(self.states[idx])

    def play_move(self, move, idx=0):
        if not self._is_legal(move, idx):
            raise ValueError("Illegal move")
        new_state = self.backend.play_move(self.states[idx], move)
        self.states[idx] = new_state
        hist = self.history[idx]
        hist.states.append(new_state)
        hist.result = self._evaluate(new_state)
        return hist.result

    def play_moves_parallel(self, moves, max_workers=None):
        return {idx: self.play_move(mv, idx) for idx, mv in moves.items()}

    def play_mcts(self, idx=0, simulations=1000, c=1.4):
        return self.play_mcts_parallel([idx], simulations, c)[idx]

    def play_mcts_parallel(self, idxs, simulations=1000, c=1.4, max_workers=None, batch_size=32):
        results, live = {}, []
        for idx in idxs:
            term = self._evaluate(self.states[idx])
            if term is not None:
                self.history[idx].result = term
                results[idx] = term
            else:
                live.append(idx)
        if live:
            moves = self._search(live, simulations, c, batch_size)
            for idx in live:
                results[idx] = self.play_move(moves[idx], idx)
        return {idx: results[idx] for idx in idxs}

    def reset_all_games(self):
        init_state = self.backend.create_init_state()
        self.states = [init_state for _ in range(self.threads)]
        self.history = [History(states=[init_state], result=None) for _ in range(self.threads)]

    # ------------------------------------------------------------------ internals
    def _evaluate(self, state):
        if self.backend.check_win(state):
            return state.turn * 2 - 1
        if self.backend.check_draw(state):
            return 0
        return None

    def _is_legal(self, mv, idx=0) -> bool:
        legal = self.legal_moves(idx)
        if mv in legal:
            return True
        try:   # chess-style moves: compare the coordinate part (engine.py:155-157)
            return any(m[0] == mv[0] for m in legal)
        except (TypeError, IndexError):
            return False

    def _search(self, idxs, simulations, c, batch_size):
        from . import _search
        from .mcts import _plugin_check, get_move
        game = None
        for v in {id(v): v for v in self.values}.values():
            game = _plugin_check(self.states[idxs[0]], v, self.policy, self.backend)
        if self.rng_mode == "global" or game == "generic" or _search.policy_of(self.policy)[0] == _search.HOST_POLICY:
            return {i: get_move(self.states[i], self.values[self.states[i].turn], self.policy, self.backend,
                                simulations, c, batch_size) for i in idxs}
        need = max(idxs) + 1
        if self._dev is None:
            self._dev = _device.GrowingEngine(max(need, 64), simulations, batch_size, self.device)
        moves = {}
        with self._dev.lock:
            eng = self._dev.ensure(need, simulations, batch_size)
            if need > self._seeded:
                eng.seed(self._seeded, [self.seed + g for g in range(self._seeded, need)])
                self._seeded = need
            # Engine.play_mcts uses values[state.turn] (engine.py:126): one device search per
            # value object, over contiguous runs of game indices
            groups = {}
            for i in sorted(idxs):
                v = self.values[self.states[i].turn]
                groups.setdefault(id(v), (v, []))[1].append(i)
            for value, ids in groups.values():
                if game == "connect4" and _search.value_kind(value) == "rollout":
                    roots = _device.c4_roots([self.states[i] for i in ids], self.backend)
                    moves.update(zip(ids, _search.c4_moves(eng, ids, roots, simulations, c, batch_size, value,
                                                           self.backend)))
                    continue
                for run in _runs(ids):
                    st = [self.states[i] for i in run]
                    if game == "connect4":
                        mv = _search.c4_moves(eng, run, _device.c4_roots(st, self.backend), simulations, c,
                                              batch_size, value, self.backend)
                    else:
                        mv = _search.chess_moves(eng, run, st, simulations, c, batch_size, value, self.policy,
                                                 self.backend)
                    moves.update(zip(run, mv))
        return moves


def _runs(ids):
    out, cur = [], [ids[0]]
    for i in ids[1:]:
        if i == cur[-1] + 1:
            cur.append(i)
        else:
            out.append(cur)
            cur = [i]
    out.append(cur)
    return out
