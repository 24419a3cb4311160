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


MATE_IN_ONE = "r1bqkbnr/pppp1ppp/2n5/4p3/2B1P3/5Q2/PPPP1PPP/RNB1K1NR w KQkq - 2 3"   # Qxf7#
FIFTY_NEXT = "4k3/8/8/8/8/8/8/4K2R w K - 49 30"   # every move reaches the fifty-move draw


@pytest.mark.parametrize("fen", [None, MATE_IN_ONE, FIFTY_NEXT])
def test_chess_selfplay_matches_engine(fen):
    """The device chess pool plays the same games as Engine.play_mcts_parallel (crude score,
    immediate_value(3), per-game streams seed + idx): same positions after every move, same
    results; a finished game restarts from the initial position while Engine's stays over."""
    from zeroclone_amd.engine import Engine
    from zeroclone_amd.engine.games.chess import chess_backend as cb
    from zeroclone_amd.selfplay import ChessSelfPlay
    G, sims, seed = 8, 48, 5
    sp = ChessSelfPlay(G, sims, seed=seed, init_fen=fen)
    e = Engine({"game": "chess", "backend": "chess_backend", "value_function": "crude_chess_score",
                "policy_functions": "immediate_value", "policy": {"policy_freedom": 3}, "threads": G, "seed": seed})
    if fen:
        for i in range(G):
            e.states[i] = cb.state_from_fen(fen)
            e.history[i].states = [e.states[i]]
    init = sp.init_row.cpu().numpy()[0]
    alive = [True] * G
    finished = 0
    for _ in range(6):
        res = sp.step()
        er = e.play_mcts_parallel([g for g in range(G) if alive[g]], simulations=sims, c=1.4)
        rows = sp.roots.cpu().numpy()
        for g in range(G):
            if not alive[g]:
                continue
            exp = er[g] if er[g] is not None else 2
            assert int(res[g]) == exp, (g, res[g], er[g])
            if exp != 2:
                alive[g] = False
                finished += 1
                assert np.array_equal(rows[g], init)   # refilled
            else:
                want = np.frombuffer(cb.to_zc(e.states[g]).tobytes(), np.uint8)
                assert np.array_equal(rows[g][:67], want[:67])
    assert len(sp.finished) >= finished
    if fen == FIFTY_NEXT:
        assert finished == G and all(r == 0 for _, _, r in sp.finished[:G])
    sp.close()


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


def test_simulate_games_quota():
    """train.py:simulate_games on the device pool: exactly `total` results, each a game the
    pool recorded, in completion order."""
    from zeroclone_amd.selfplay import simulate_games
    sp = C4SelfPlay(16, 40, seed=3)
    res = simulate_games(sp, 24, max_steps=200)
    assert len(res) == 24 and set(res) <= {-1, 0, 1}
    assert [f[2] for f in sp.finished[:24]] == res
    assert simulate_games(sp, 0) == []
    sp.close()
