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
