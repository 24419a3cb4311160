"""Device-resident Connect4 self-play and the multi-GPU trajectory exchange.

`C4SelfPlay` is the batched form of scripts/train.py:simulate_games (:151-170) +
Engine.play_mcts_parallel (engine/engine.py:131-138): G games live on one GPU as bitboards;
one `step()` searches every game (zc_c4_search_async), plays the chosen moves and
evaluates them (zc_c4_play_async, Engine.play_move/_evaluate), and restarts finished games
from the opening — the refill the reference does with add_game.  Game slot g of rank r is
global game r*G + g and draws from its own CPython MT19937 stream seeded seed + global id,
so per-game results do not depend on the number of GPUs.

Finished games are labelled exactly as Engine.get_dataset (engine.py:60-89) labels them and
kept as compact positions (zc_c4_state rows: stones X, stones O, turn | label << 32).
`gather_positions` all-gathers every rank's finished positions (counts first, then a padded
payload) over torch.distributed — RCCL over xGMI on the GPUs, gloo on CPU — the one
collective of the scale-out path.  `ReplayBuffer` is
scripts/train.py:_update_replay (:27-50).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native

ONGOING = _native.ZC_C4_ONGOING


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


class C4SelfPlay:
    def __init__(self, games: int, sims: int, c: float = 1.4, batch_size: int = 32, seed: int = 0,
                 rank: int = 0, device: int = 0, record: bool = True):
        self.G, self.sims, self.c, self.bs = games, sims, c, batch_size
        self.dev = torch.device("cuda", device)
        self.eng = _native.NativeEngine(max_games=games, max_sims=sims, max_batch=batch_size, device=device)
        self.first_id = rank * games
        self.eng.seed(0, [seed + self.first_id + g for g in range(games)])
        self.roots = torch.zeros((games, 3), dtype=torch.int64, device=self.dev)
        self.moves = torch.zeros(games, dtype=torch.int32, device=self.dev)
        self.na = torch.zeros((games, 7), dtype=torch.int32, device=self.dev)
        self.stats = torch.zeros((games, _native.STATS_FIELDS), dtype=torch.int64, device=self.dev)
        self.results = torch.zeros(games, dtype=torch.int32, device=self.dev)
        self.record = record
        # current game of every slot: positions so far (host copies, appended per step)
        self._hist = [[] for _ in range(games)]
        self.finished = []   # (global game id, move list, result, positions[n,3])
        self._moves = [[] for _ in range(games)]

    def step(self) -> torch.Tensor:
        """One move for every game (on torch's current stream); returns the per-game results
        tensor (ONGOING = 2).  Finished games restart from the opening."""
        s = torch.cuda.current_stream(self.dev).cuda_stream
        before = self.roots.clone() if self.record else None
        self.eng.c4_search_async(self.roots.data_ptr(), self.G, self.sims, self.c, self.bs, self.moves.data_ptr(),
                                 self.na.data_ptr(), self.stats.data_ptr(), stream=s)
        self.eng.c4_play_async(self.roots.data_ptr(), self.G, self.moves.data_ptr(), self.results.data_ptr(),
                               reset=False, stream=s)
        if self.record:
            self._collect(before)
        else:
            self._refill()
        return self.results

    def _refill(self):
        done = self.results != ONGOING
        self.roots[done] = 0

    def _collect(self, before: torch.Tensor):
        pre = before.cpu().numpy()
        post = self.roots.cpu().numpy()
        res = self.results.cpu().numpy()
        mv = self.moves.cpu().numpy()
        for g in range(self.G):
            if not self._hist[g]:
                self._hist[g].append(pre[g].copy())
            self._moves[g].append(int(mv[g]))
            self._hist[g].append(post[g].copy())
            if res[g] != ONGOING:
                pos = np.stack(self._hist[g]).astype(np.int64)
                lab = dataset_labels(len(pos), int(res[g]))
                pos[:, 2] = (pos[:, 2] & 1) | (lab.astype(np.int64) << 32)
                self.finished.append((self.first_id + g, self._moves[g], int(res[g]), pos))
                self._hist[g], self._moves[g] = [], []
        self._refill()

    def take_positions(self):
        """Positions of the games finished since the last call: [n, 3] int64 rows with the
        Engine.get_dataset label in the high half of column 2."""
        rows = [f[3] for f in self.finished]
        self.finished = []
        return np.concatenate(rows) if rows else np.zeros((0, 3), np.int64)

    def close(self):
        self.eng.close()


class ChessSelfPlay:
    """Device-resident chess self-play: the chess form of `C4SelfPlay`.  G games live on one
    GPU as zc_chess_state rows; one `step()` searches every game (Value('crude_chess_score')
    in the search kernel, or a value network between the stepwise select and backup
    kernels), plays the chosen moves (zc_chess_play_async) and tests the new positions
    (zc_chess_terminal_async: check_win, stalemate, fifty-move rule) on the device, and
    restarts finished games from the initial position.  The repetition half of check_draw
    (chess_backend.cpp:416-441: both sides' move histories end in >= 3 repeats of a block of
    >= 2 moves) runs on the device too: each side's moves are appended to a per-game history
    on the GPU and zc_chess_repetition_async tests both after every step.  Results follow Engine._evaluate (engine.py:148-153): check_win -> turn*2-1
    of the position after the move, a draw -> 0.  Game slot g of rank r is global game r*G+g
    with its own CPython MT19937 stream seeded seed + global id, as in C4SelfPlay."""

    def __init__(self, games: int, sims: int, c: float = 1.4, batch_size: int = 32, seed: int = 0,
                 rank: int = 0, device: int = 0, policy: int = _native.ZC_POLICY_IMMEDIATE_VALUE,
                 freedom: float = 3.0, net=None, init_fen: str | None = None):
        self.G, self.sims, self.c, self.bs = games, sims, c, batch_size
        self.policy, self.freedom = int(policy), float(freedom)
        self.dev = torch.device("cuda", device)
        self.eng = _native.NativeEngine(max_games=games, max_sims=sims, max_batch=batch_size, device=device)
        self.eng.chess_reserve()
        self.first_id = rank * games
        self.eng.seed(0, [seed + self.first_id + g for g in range(games)])
        init = _native.chess_from_fen(init_fen) if init_fen else _native.chess_init()
        self.init_row = torch.from_numpy(np.frombuffer(init.tobytes(), np.uint8).reshape(1, 72).copy()).to(self.dev)
        self.init_turn = int(np.asarray(init["turn"]).reshape(-1)[0])
        self.roots = self.init_row.repeat(games, 1).contiguous()
        self.moves = torch.zeros(games, dtype=torch.int16, device=self.dev)
        self.na = torch.zeros((games, _native.CHESS_MAX_MOVES), dtype=torch.int32, device=self.dev)
        self.stats = torch.zeros((games, _native.STATS_FIELDS), dtype=torch.int64, device=self.dev)
        self.flags = torch.zeros(games, dtype=torch.int32, device=self.dev)
        self.vs = self.value_fn = None
        if net is not None:
            from .valued import ChessValuedSearch, NetValue
            self.vs = ChessValuedSearch(self.eng, games, batch_size, leaves=False, policy=self.policy,
                                        freedom=self.freedom)
            self.value_fn = NetValue(net)
        self.hist_cap = 1024  # moves per side; a longer game raises
        self.hist = torch.zeros((games, 2, self.hist_cap), dtype=torch.int16, device=self.dev)
        self.hlen = torch.zeros((games, 2), dtype=torch.int32, device=self.dev)
        self.turn = torch.full((games,), self.init_turn, dtype=torch.int64, device=self.dev)
        self.rep = torch.zeros(games, dtype=torch.int32, device=self.dev)
        self._slots = torch.arange(games, device=self.dev)
        self._turn = [self.init_turn] * games
        self._moves = [[] for _ in range(games)]
        self.finished = []   # (global game id, move list, result)

    def step(self) -> np.ndarray:
        """One move for every game; returns the per-game results (ONGOING = 2).  Finished
        games restart from the initial position."""
        s = torch.cuda.current_stream(self.dev).cuda_stream
        if self.vs is None:
            self.eng.chess_search_async(0, self.G, self.roots.data_ptr(), self.sims, self.c, self.bs, self.policy,
                                        self.freedom, self.moves.data_ptr(), self.na.data_ptr(),
                                        self.stats.data_ptr(), s)
        else:
            mv, _, st = self.vs.run(self.roots, self.sims, self.c, self.value_fn)
            self.moves.copy_(mv)
            self.stats.copy_(st)
        self.eng.chess_play_async(self.G, self.roots.data_ptr(), self.moves.data_ptr(), self.roots.data_ptr(), s)
        self.eng.chess_terminal_async(self.G, self.roots.data_ptr(), self.flags.data_ptr(), s)
        # play_move's history push (the mover's deque), then both sides' repetition test
        at = self.hlen[self._slots, self.turn].clamp(max=self.hist_cap - 1).long()
        self.hist[self._slots, self.turn, at] = self.moves
        self.hlen[self._slots, self.turn] += 1
        self.turn ^= 1
        _native.check(_native.lib().zc_chess_repetition_async(self.G, self.hist_cap, self.hist.data_ptr(),
                                                              self.hlen.data_ptr(), self.rep.data_ptr(), s))
        mv = self.moves.cpu().numpy().view(np.uint16)
        fl = self.flags.cpu().numpy()
        rep = self.rep.cpu().numpy()
        if int(self.hlen.max().item()) > self.hist_cap:
            raise RuntimeError(f"a game exceeded {self.hist_cap} moves per side")
        if (self.stats[:, 5] == _native.ZC_STATUS_CAPACITY).any():
            raise RuntimeError("chess search exceeded the tree's child-slot pool or depth limit")
        res = np.full(self.G, ONGOING, np.int32)
        done = []
        draw_flags = _native.ZC_CHESS_STALEMATE | _native.ZC_CHESS_FIFTY
        for g in range(self.G):
            if mv[g] == 0xFFFF:
                raise RuntimeError(f"game slot {g}: no legal move at a non-terminal root")
            self._moves[g].append(_native.unpack_chess_move(int(mv[g])))
            self._turn[g] ^= 1
            if fl[g] & _native.ZC_CHESS_WIN:
                res[g] = self._turn[g] * 2 - 1
            elif fl[g] & draw_flags or rep[g] == 3:
                res[g] = 0
            if res[g] != ONGOING:
                self.finished.append((self.first_id + g, self._moves[g], int(res[g])))
                self._moves[g] = []
                self._turn[g] = self.init_turn
                done.append(g)
        if done:
            d = torch.tensor(done, dtype=torch.int64, device=self.dev)
            self.roots[d] = self.init_row
            self.hlen[d] = 0
            self.turn[d] = self.init_turn
        return res

    def close(self):
        self.eng.close()


def simulate_games(pool, total_games: int, max_steps: int | None = None) -> list[int]:
    """scripts/train.py:simulate_games (:151-170) on a device pool (C4SelfPlay or
    ChessSelfPlay): step every game until `total_games` games have finished; returns their
    results in completion order (slot order within a step), while their trajectories are in
    `pool.finished`.  The reference starts min(total, threads) games and adds one per finished
    game while fewer than `total_games` have started; the pool keeps every slot playing, so
    games still running when the quota is met are surplus and not counted."""
    if total_games < 0:
        raise ValueError("total_games must be >= 0")
    out: list[int] = []
    steps = 0
    while len(out) < total_games:
        if max_steps is not None and steps >= max_steps:
            raise RuntimeError(f"{len(out)} of {total_games} games finished in {max_steps} steps")
        r = pool.step()
        r = r.cpu().numpy() if torch.is_tensor(r) else np.asarray(r)
        out.extend(int(v) for v in r[r != ONGOING])
        steps += 1
    return out[:total_games]


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
    """All-gather variable-length [n_r, 3] int64 position rows from every rank (rank order):
    an all_gather of the counts, then of payloads padded to the largest count."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    pad = torch.zeros((m, 3), dtype=torch.int64, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)


class ReplayBuffer:
    """scripts/train.py:_update_replay (:27-50): the training set of a cycle = all new data +
    a uniform sample (without replacement) of 30 % of everything seen before."""

    def __init__(self, frac_old: float = 0.30, seed: int | None = None):
        self.frac_old = frac_old
        self.states, self.values = [], []
        self.rng = np.random.default_rng(seed)

    def update(self, states_new: np.ndarray, values_new: np.ndarray):
        if not self.states:
            self.states.append(states_new)
            self.values.append(values_new)
            return states_new, values_new
        old_s = np.concatenate(self.states, axis=0)
        old_v = np.concatenate(self.values, axis=0)
        k = int(self.frac_old * len(old_s))
        if k > 0:
            idx = self.rng.choice(len(old_s), k, replace=False)
            ss, sv = old_s[idx], old_v[idx]
        else:
            ss, sv = old_s[:0], old_v[:0]
        self.states.append(states_new)
        self.values.append(values_new)
        return np.concatenate([ss, states_new], axis=0), np.concatenate([sv, values_new], axis=0)
