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
        res = sp.step().cpu().numpy()
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
    games = sp.finished_games()
    assert len(games) >= finished
    for gid, moves, res, rows in games:   # the recorded trajectory replays through the rules
        assert rows.shape == (len(moves) + 1, 9)
        assert np.array_equal(rows[0].view(np.uint8), init)
    if fen == FIFTY_NEXT:
        assert finished == G and all(r == 0 for _, _, r, _ in games[:G])
    sp.close()


def test_selfplay_matches_oracle_games_with_refill():
    G, sims, seed = 48, 60, 77
    sp = C4SelfPlay(G, sims, seed=seed, rank=1)   # rank 1: global ids G..2G-1
    per_slot = {g: [] for g in range(G)}
    for k in range(70):
        sp.step()
        if k % 25 == 24:   # take part-way: games in progress stay in their slots
            for gid, moves, res, pos in sp.finished_games():
                per_slot[gid - G].append((moves, res, pos))
    for gid, moves, res, pos in sp.finished_games():
        per_slot[gid - G].append((moves, res, pos))
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
    """train.py:simulate_games on the device pool: games 0..G-1 start in slots 0..G-1, a
    finished slot starts the next game only while fewer than `total` have started, every
    started game is played to its end: exactly `total` games, results by game number, each
    game the oracle's game for its slot's stream."""
    from zeroclone_amd.selfplay import simulate_games
    G, sims, seed, total = 16, 40, 3, 24
    sp = C4SelfPlay(G, sims, seed=seed)
    res = simulate_games(sp, total, max_steps=400)
    games = sp.finished_games(sp.last_batch)
    assert len(res) == total and len(games) == total and set(res) <= {-1, 0, 1}
    assert [g[2] for g in games] == res
    assert sorted(sp.last_batch.games[:, 0].cpu().tolist()) == list(range(total))
    assert [g[0] for g in games[:G]] == list(range(G))   # game g < G starts in slot g
    per_slot = {}
    for gid, moves, r, pos in games:
        per_slot.setdefault(gid, []).append((moves, r))
    for slot, got in per_slot.items():
        assert got == oracle_games(seed + slot, len(got), sims), slot
    # a shorter quota than the pool: surplus slots idle from the start
    res = simulate_games(sp, 5, max_steps=400)
    assert len(res) == 5 and [g[0] for g in sp.finished_games(sp.last_batch)] == list(range(5))
    assert simulate_games(sp, 0) == []
    sp.close()


def test_quota_steps_on_a_side_stream_grow_the_pool_in_order():
    """step(stream=s) under a quota with a pool too small for it: the pool grows between
    steps (ensure_room) on s itself, so the growth reads the counts after the previous
    step's record kernel and copies the pool before the next one writes — no game is dropped
    or corrupted, every game is the oracle's game for its slot."""
    G, sims, seed, total = 12, 24, 41, 20
    sp = C4SelfPlay(G, sims, seed=seed, games_cap=2)   # 2 x 43 positions: must grow on the way
    side = torch.cuda.Stream(sp.dev)
    side.wait_stream(torch.cuda.current_stream(sp.dev))
    sp.start(total)
    cap0 = sp.traj.pool_cap
    for _ in range(200):   # no host synchronisation between the steps
        sp.step(stream=side.cuda_stream)
    side.synchronize()
    assert sp.traj.pool_cap > cap0
    games = sp.finished_games()
    assert len(games) == total
    per_slot = {}
    for gid, moves, r, pos in games:
        assert pos.shape[0] == len(moves) + 1
        assert np.array_equal((pos[:, 2] >> 32).astype(np.float32), dataset_labels(len(pos), r))
        per_slot.setdefault(gid, []).append((moves, r))
    for slot, got in per_slot.items():
        assert got == oracle_games(seed + slot, len(got), sims), slot
    sp.close()


def test_record_labels_and_take_positions():
    """Pooled labels are Engine.get_dataset's (engine.py:60-89) and take_positions carries
    them in the high half of column 2, on the device."""
    sp = C4SelfPlay(64, 24, seed=9)
    for _ in range(45):
        sp.step()
    b = sp.take()
    assert b.games.shape[0] >= 64
    labels = b.labels.cpu().numpy()
    for gno, slot, r, off, n in b.games.cpu().numpy().tolist():
        assert np.array_equal(labels[off:off + n].astype(np.float32), dataset_labels(n, r))
        assert b.moves[off + n - 1].item() == -1
    for _ in range(45):
        sp.step()
    rows = sp.take_positions()
    assert rows.is_cuda and rows.shape[1] == 3 and rows.shape[0] > 0
    sp.close()
