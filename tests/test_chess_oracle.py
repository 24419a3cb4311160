"""The chess oracle (oracle/chess_oracle.c) against the reference's own outputs
(tests/golden/chess_*.json, generated from engine/games/chess compiled unmodified)."""
import numpy as np
import pytest

import oracle


def test_perft_matches_reference(golden):
    for case in golden("chess_perft.json")["perft"]:
        s = oracle.chess_from_fen(case["fen"])
        for d, n in enumerate(case["counts"], start=1):
            assert oracle.chess_perft(s, d) == n, (case["name"], d)


def test_perft_start_depth5():
    assert oracle.chess_perft(oracle.chess_init(), 5) == 4865351


def test_ordered_move_lists_with_capture_values(golden):
    cases = golden("chess_movelists.json")["cases"]
    assert len(cases) >= 250
    for case in cases:
        got = oracle.chess_moves(oracle.chess_from_json(case["state"]))
        assert [list(m) for m in got] == case["moves"]


def test_play_move(golden):
    for case in golden("chess_play.json")["cases"]:
        s = oracle.chess_from_json(case["state"])
        o = oracle.chess_play(s, case["move"])
        a = case["after"]
        assert bytes(o.board).decode("latin-1") == a["board"]
        b = case["state"]   # the fixture's "before" state carries only its history lengths
        assert (o.turn, o.fifty, o.castle) == (a["turn"], a["fifty"], a["castle"])
        assert (o.nhw, o.nhb) == (a["nhw"] - b["nhw"], a["nhb"] - b["nhb"])
        mv = case["move"]
        head = "%d%d%d%d%d" % (mv[0], mv[1], mv[2], mv[3], int(mv[4]))
        assert (a["hw_head"] if s.turn == 0 else a["hb_head"]) == head


def test_terminal_flags(golden):
    cases = golden("chess_terminal.json")["cases"]
    assert sum(c["win"] for c in cases) >= 10 and sum(c["draw"] for c in cases) >= 20
    for case in cases:
        s = oracle.chess_from_json(case["state"])
        assert oracle.chess_win(s) == case["win"], case.get("note", case.get("fen"))
        assert oracle.chess_draw(s) == case["draw"], case.get("note", case.get("fen"))
        if "expect" in case:  # the reference's own test expectations (tests/test_cb.py:105-116)
            assert [case["win"], case["draw"]] == case["expect"]


def test_state_to_tensor(golden):
    for case in golden("chess_tensor.json")["cases"]:
        t = oracle.chess_tensor(oracle.chess_from_json(case["state"]))
        bits = np.unpackbits(np.frombuffer(bytes.fromhex(case["bits"]), np.uint8))[: 17 * 64]
        np.testing.assert_array_equal((t.reshape(-1) != 0).astype(np.uint8), bits)
        assert list(t.shape) == case["shape"]


def test_chess_search_matches_reference(golden):
    """Chess get_move (crude_chess_score, immediate_value / random policy) vs the reference."""
    for case in golden("chess_get_move.json")["cases"]:
        s = oracle.chess_from_fen(case["fen"])
        mt = oracle.MT(case["seed"])
        best, moves, na = oracle.chess_get_move(s, mt, case["sims"], case["c"], case["bs"], case["policy"],
                                                case["freedom"])
        assert [list(m) for m in moves] == case["root_moves"]
        assert na == case["root_na"], case["fen"]
        assert list(moves[best]) == case["move"]
        assert mt.drawn == case["consumed"]
        assert mt.u32() == case["next_word"]


def test_chess_selfplay_batch_equals_get_move_play_judge():
    """zcc_selfplay_batch (bench.py's chess CPU baseline) = per game, per move: get_move
    (crude_chess_score, immediate_value(3)), play the best move, refill at a finished game —
    the same stream consumption as the step-by-step oracle calls, from mixed positions."""
    import copy
    import numpy as np
    rng = np.random.default_rng(3)
    states = []
    for _ in range(6):
        s = oracle.chess_init()
        for _ in range(int(rng.integers(0, 30))):
            ms = oracle.chess_moves(s)
            if not ms or oracle.chess_draw(s):
                break
            s = oracle.chess_play(s, ms[int(rng.integers(len(ms)))])
        states.append(s)
    rows = np.zeros((len(states), 72), np.uint8)
    for i, s in enumerate(states):
        rows[i, :64] = list(s.board)
        rows[i, 64:67] = (s.turn, s.fifty, s.castle)
    mts = [oracle.MT(40 + i) for i in range(len(states))]
    ref = [copy.deepcopy(m) for m in mts]
    K, S = 5, 60
    exp = oracle.chess_selfplay_batch(rows, mts, K, S, 1.4, 16, threads=3)
    assert (exp > 0).all() and (exp <= K * S).all()
    for i, s in enumerate(states):
        s = oracle.chess_state(bytes(rows[i, :64]).decode("latin-1"), int(rows[i, 64]), int(rows[i, 65]),
                               int(rows[i, 66]))
        for _ in range(K):
            best, ms, _ = oracle.chess_get_move(s, ref[i], S, 1.4, 16, "immediate_value", 3.0)
            s = oracle.chess_play(s, ms[best])
            if not oracle.chess_moves(s) or oracle.chess_draw(s):
                s = oracle.chess_init()
        assert ref[i].state() == mts[i].state(), i
