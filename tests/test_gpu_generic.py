"""mcts.get_move with a game backend the device knows nothing about.  The
toy backends of tests/toy_games (tic-tac-toe; a subtraction game whose moves are strings in
a tuple) run through this package's get_move — the tree on the device (zc_gen_*), the
backend, policy and value called on the host — and must reproduce the reference's compiled
get_move on the committed goldens (tests/golden/gen_golden_generic.py): the move, every
policy call (untried moves in list order, the pick), every flush's leaves in pending order,
and Python's `random` stream afterwards (/root/reference engine/mcts/src/mcts.cpp:47-160,
engine/value_functions.py:35-45, engine/policy_functions.py:10-12)."""
import random

import pytest

from toy_games import pile_backend, plugins, ttt_backend

pytestmark = pytest.mark.gpu

GAMES = {"ttt": ttt_backend, "pile": pile_backend}


def _state(game, enc):
    if game == "ttt":
        return ttt_backend.State(tuple(enc[:9]), enc[9])
    return pile_backend.State(enc[0], enc[1])


def _jsonish(x):
    if isinstance(x, (list, tuple)):
        return [_jsonish(y) for y in x]
    return x


def test_generic_get_move_matches_reference(golden):
    from zeroclone_amd.engine import mcts
    from zeroclone_amd.engine.policy_functions import Policy
    from zeroclone_amd.engine.value_functions import Value
    cases = golden("generic_get_move.json")["cases"]
    assert len(cases) >= 12
    for c in cases:
        be = GAMES[c["game"]]
        inner = Policy("random") if c["policy"] == "random" else plugins.POLICIES[c["policy"]]
        pol = plugins.Recording(inner)
        v = Value("random_rollout") if c["value"] == "random_rollout" else plugins.HashValue(be.encode)
        val = plugins.RecordingValue(v, be.encode)
        random.seed(c["seed"])
        mv = mcts.get_move(_state(c["game"], c["state"]), val, pol, be, c["sims"], c["c"], c["bs"])
        key = (c["game"], c["seed"])
        assert _jsonish(pol.calls) == c["calls"], key
        assert _jsonish(val.flushes) == c["flushes"], key
        assert mv == c["move"], key
        assert random.getrandbits(32) == c["next_word"], key


def test_generic_engine_plays_a_game():
    """Engine over a backend module named by its dotted path: play_mcts drives the
    any-backend search to the end of a tic-tac-toe game; each move is the one get_move gives
    from the same Python random state."""
    from zeroclone_amd.engine import Engine, mcts
    e = Engine({"game": "ttt", "backend": "toy_games.ttt_backend", "value_function": "random_rollout",
                "policy_functions": "random", "threads": 1})
    random.seed(3)
    res = None
    for _ in range(9):
        st = random.getstate()
        state = e.get_state(0)
        exp = mcts.get_move(state, e.values[state.turn], e.policy, e.backend, 60, 1.4, 32)
        random.setstate(st)
        res = e.play_mcts(0, simulations=60, c=1.4)
        assert e.get_hist(0)[-1] == ttt_backend.play_move(state, exp)
        if res is not None:
            break
    assert res in (-1, 0, 1)


def test_generic_tree_grows_its_slot_pool():
    """A backend with wide nodes: the move-slot pool grows (zc_gen_reserve) mid-search and the
    search still finishes with every simulation backed up."""
    from zeroclone_amd.engine import mcts
    from toy_games import wide_backend
    random.seed(1)
    mv = mcts.get_move(wide_backend.create_init_state(), plugins.HashValue(wide_backend.encode),
                       plugins.last_move, wide_backend, 300, 1.4, 16)
    assert mv in wide_backend.get_legal_moves(wide_backend.create_init_state())
