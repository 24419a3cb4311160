"""GPU parity of the host-policy fallback: mcts.get_move with an arbitrary
policy callable — the tree on the device (zc_c4_hp_walk / zc_c4_hp_expand + the stepwise
backup), the policy called on the host at every expansion (mcts.cpp:65-78).  Checked against
the reference's own compiled get_move (tests/golden/c4_get_move_hostpolicy.json, generator
tests/golden/gen_golden_hostpolicy.py): the move, EVERY policy call (untried columns in list
order and the pick), the leaves evaluated, and the state of Python's `random` afterwards
(the policies and Value('random_rollout') share it)."""
import random

import pytest

import c4_policies as P
from c4_values import bits_from_rows, hash_value
from zeroclone_amd.engine import Engine, Policy, Value, mcts
from zeroclone_amd.engine.games.connect4 import c4_backend as c4

pytestmark = pytest.mark.gpu


def dec(s):
    return [[(" " if ch == "." else ch) for ch in s[r * 7:(r + 1) * 7]] for r in range(6)]


class HashValue:
    def __init__(self):
        self.leaves = 0

    def batch(self, states, **kw):
        self.leaves += len(states)
        return [hash_value(*bits_from_rows(s.board), s.turn) for s in states]


class CountingValue:
    def __init__(self, inner):
        self.inner, self.leaves = inner, 0

    def batch(self, states, **kw):
        self.leaves += len(states)
        return self.inner.batch(states, **kw)


def test_host_policy_get_move_matches_reference(golden):
    cases = golden("c4_get_move_hostpolicy.json")["cases"]
    assert len(cases) >= 12
    for c in cases:
        st = c4.State(dec(c["board"]), c["turn"])
        pol = P.Recording(P.make(c["policy"]))
        val = CountingValue(Value("random_rollout")) if c["value"] == "random_rollout" else HashValue()
        random.seed(c["seed"])
        mv = mcts.get_move(st, val, pol, c4, c["sims"], c["c"], c["bs"])
        key = (c["policy"], c["value"], c["seed"])
        assert pol.calls == c["calls"], key
        assert mv == (c["move"], 0), key
        assert val.leaves == c["leaves"], key
        assert random.getrandbits(32) == c["next_word"], key


def test_policy_errors_behave_like_the_reference():
    st = c4.create_init_state()
    # an action that is not among the untried moves: list.index raises ValueError (mcts.cpp:68)
    with pytest.raises(ValueError):
        mcts.get_move(st, HashValue(), lambda moves: (9, 0), c4, 10, 1.4, 4)
    # a policy's own exception propagates
    def boom(moves):
        raise KeyError("policy failure")
    with pytest.raises(KeyError):
        mcts.get_move(st, HashValue(), boom, c4, 10, 1.4, 4)


def test_builtin_policies_stay_on_the_device():
    from zeroclone_amd import _native
    from zeroclone_amd.engine import _search
    assert _search.policy_of(Policy("random"))[0] == _native.ZC_POLICY_RANDOM
    assert _search.policy_of(Policy("immediate_value", policy_freedom=2))[0] == _native.ZC_POLICY_IMMEDIATE_VALUE
    assert _search.policy_of(P.last_move)[0] == _search.HOST_POLICY

    class Greedy(Policy):
        def random(self, moves, args):   # overriding a built-in rule makes it a host policy
            return moves[0]
    assert _search.policy_of(Greedy("random"))[0] == _search.HOST_POLICY


def test_engine_with_a_host_policy_plays_the_reference_move(golden):
    # Engine.play_mcts with a host policy searches on Python's global stream (get_move), even
    # in the per-game stream mode, and plays the reference's move (play_mcts: batch 32)
    c = next(x for x in golden("c4_get_move_hostpolicy.json")["cases"]
             if x["board"] == "." * 42 and x["value"] == "random_rollout" and x["bs"] == 32
             and x["policy"] == "last_move")
    eng = Engine({"game": "connect4", "backend": "c4_backend", "value_function": "random_rollout", "threads": 1})
    eng.policy = P.make(c["policy"])
    random.seed(c["seed"])
    eng.play_mcts(0, c["sims"], c["c"])
    after = eng.states[0]
    col = c["move"]
    assert after.board[5][col] == "X" and sum(ch != " " for row in after.board for ch in row) == 1
    assert random.getrandbits(32) == c["next_word"]


def test_chess_host_policy_get_move_matches_reference(golden):
    """Chess: the reference's compiled get_move with the reference chess backend and
    Value('crude_chess_score') (tests/golden/chess_get_move_hostpolicy.json) — every policy
    call (size, pick and a checksum of the untried list in order), move, leaves, and Python's
    `random` afterwards."""
    from zeroclone_amd.engine.games.chess import chess_backend as cb
    cases = golden("chess_get_move_hostpolicy.json")["cases"]
    assert len(cases) >= 16
    for c in cases:
        st = cb.state_from_fen(c["fen"])
        pol = P.ChessRecording(P.make(c["policy"]))
        val = CountingValue(Value("crude_chess_score"))
        random.seed(c["seed"])
        mv = mcts.get_move(st, val, pol, cb, c["sims"], c["c"], c["bs"])
        key = (c["fen"], c["policy"], c["seed"])
        assert pol.calls == c["calls"], key
        assert list(mv[0]) + [mv[1]] == c["move"], key
        assert val.leaves == c["leaves"], key
        assert random.getrandbits(32) == c["next_word"], key
