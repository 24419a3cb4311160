"""Device self-play (search + play + refill on the GPU) against the oracle playing the same
games with the same per-slot streams; plus the 1-GPU form of the trajectory gather."""
import numpy as np
import pytest
import torch

import oracle
from zeroclone_amd.selfplay import C4SelfPlay, dataset_labels

pytestmark = pytest.mark.gpu


def oracle_games(seed, n_games, sims, c=1.4, bs=32):
    mt = oracle.MT(seed)
    games = []
    for _ in range(n_games):
        b, t = "." * 42, 0
        moves = []
        while True:
            col, _, _ = oracle.get_move_mt(b, t, mt, sims, c, bs)
            moves.append(col)
            b, t = oracle.play(b, t, col)
            if oracle.check_win(b, t):
                games.append((moves, t * 2 - 1))
                break
            if oracle.check_draw(b):
                games.append((moves, 0))
                break
    return games


def test_selfplay_matches_oracle_games_with_refill():
    G, sims, seed = 48, 60, 77
    sp = C4SelfPlay(G, sims, seed=seed, rank=1)   # rank 1: global ids G..2G-1
    per_slot = {g: [] for g in range(G)}
    for _ in range(70):
        sp.step()
        for gid, moves, res, pos in sp.finished:
            per_slot[gid - G].append((moves, res, pos))
        sp.finished = []
    torch.cuda.synchronize()
    checked = 0
    for g in range(G):
        if not per_slot[g]:
            continue
        exp = oracle_games(seed + G + g, len(per_slot[g]), sims)
        for (moves, res, pos), (emoves, eres) in zip(per_slot[g], exp):
            assert moves == emoves and res == eres
            assert pos.shape[0] == len(moves) + 1
            assert np.array_equal((pos[:, 2] >> 32).astype(np.float32), dataset_labels(len(pos), res))
            checked += 1
    assert checked >= G   # every slot finished at least one game on average
    sp.close()
