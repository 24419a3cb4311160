"""The reference-API layer on the chess path: mcts.get_move with the reference's plugins
(crude_chess_score, immediate_value) against the reference's own outputs, Engine self-play
against the oracle, and the network value modes end to end."""
import random

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def test_get_move_crude_chess_is_a_drop_in(golden):
    from zeroclone_amd.engine import Policy, Value, mcts
    from zeroclone_amd.engine.games.chess import chess_backend as cb
    value = Value("crude_chess_score")
    for c in golden("chess_get_move.json")["cases"][:10]:
        st = cb.state_from_fen(c["fen"])
        pol = Policy("immediate_value", policy_freedom=c["freedom"]) if c["policy"] == "immediate_value" \
            else Policy("random")
        random.seed(c["seed"])
        mv = mcts.get_move(st, value, pol, cb, c["sims"], c["c"], c["bs"])
        assert list(mv[0]) + [mv[1]] == c["move"]
        assert random.getrandbits(32) == c["next_word"]


def test_engine_chess_selfplay_matches_oracle():
    """Engine(crude_chess config) — per-game streams random.seed(seed + idx); the reference's
    Engine reads `policy_functions` (engine.py:27), so the YAML's policy_function is unused
    and the policy is random with policy_freedom kwargs.  Three moves of two games."""
    from zeroclone_amd.engine import Engine
    cfg = {"game": "chess", "backend": "chess_backend", "value_function": "crude_chess_score",
           "policy_function": "immediate_value", "threads": 2, "mcts": {"simulations": 120, "c_puct": 1.4},
           "policy": {"policy_freedom": 3}, "seed": 5}
    e = Engine(cfg)
    for _ in range(3):
        e.play_mcts_parallel([0, 1], simulations=120, c=1.4)
    for g in range(2):
        mt = oracle.MT(5 + g)
        s = oracle.chess_init()
        for k in range(3):
            best, moves, _ = oracle.chess_get_move(s, mt, 120, 1.4, 32, "random", 0.0)
            h = e.history[g].states[k + 1]
            s = oracle.chess_play(s, moves[best])
            assert bytes(s.board) == bytes(h.board), (g, k)


def test_network_value_modes_run_on_device():
    """Value('network_latest', model_type=...) — the reference's ValueNetwork template with a
    random init, fp16 on the GPU — drives get_move for chess (17 planes) and Connect4
    (2 planes); the move is legal and Python's random stream advanced as the oracle's would
    be for the same policy draws."""
    from zeroclone_amd.engine import Policy, Value, mcts
    from zeroclone_amd.engine.games.chess import chess_backend as cb
    from zeroclone_amd.engine.games.connect4 import c4_backend as c4
    v = Value("network_latest", model_type="chess_value")
    st = cb.create_init_state()
    random.seed(3)
    mv = mcts.get_move(st, v, Policy("random"), cb, 64, 1.4, 32)
    assert mv in cb.get_legal_moves(st)
    vals = v.batch([st, cb.play_move(st, mv)], backend=cb)
    assert all(-1.0 <= x <= 1.0 for x in vals)
    v4 = Value("network_latest", model_type="connect4_value")
    s4 = c4.create_init_state()
    mv4 = mcts.get_move(s4, v4, Policy("random"), c4, 64, 1.4, 32)
    assert mv4 in c4.get_legal_moves(s4)
