"""GPU tests of the reference-API layer: get_move / Value / Engine are drop-ins for the
reference's, including the state of Python's global `random` afterwards."""
import random

import numpy as np
import pytest

import oracle
from zeroclone_amd.engine import Engine, Policy, Value, mcts
from zeroclone_amd.engine.games.connect4 import c4_backend as c4

pytestmark = pytest.mark.gpu


def dec(s):
    return [[(" " if ch == "." else ch) for ch in s[r * 7:(r + 1) * 7]] for r in range(6)]


def test_get_move_is_a_drop_in(golden):
    value, policy = Value("random_rollout"), Policy("random")
    for c in golden("c4_get_move.json")["cases"]:
        st = c4.State(dec(c["board"]), c["turn"])
        random.seed(c["seed"])
        mv = mcts.get_move(st, value, policy, c4, c["sims"], c["c"], c["bs"])
        assert mv == (c["move"], 0)
        assert mv in c4.get_legal_moves(st)
        # Python's random continues exactly where the reference leaves it
        assert random.getrandbits(32) == c["next_word"], (c["seed"], c["sims"], c["bs"])


def test_value_batch_is_the_reference_rollout(golden):
    v = Value("random_rollout")
    for c in golden("c4_rollout.json")["cases"][:60]:
        st = c4.State(dec(c["board"]), c["turn"])
        random.seed(c["seed"])
        assert v(st, backend=c4) == c["value"]
        r = random.Random(c["seed"])
        for _ in range(c["consumed"]):
            r.getrandbits(32)
        assert random.getstate() == r.getstate()
    # several states in one batch consume one stream in order
    cases = golden("c4_rollout.json")["cases"][:20]
    random.seed(123)
    got = v.batch([c4.State(dec(c["board"]), c["turn"]) for c in cases], backend=c4)
    mt = oracle.MT(123)
    import ctypes
    exp = [oracle.lib().zco_rollout(c["board"].encode(), c["turn"], ctypes.byref(mt.s)) for c in cases]
    assert got == exp


def test_engine_global_rng_replays_reference_selfplay(golden):
    for g in golden("c4_selfplay.json")["games"]:
        e = Engine({"game": "connect4", "backend": "c4_backend", "value_function": "random_rollout",
                    "threads": 1, "rng": "global"})
        random.seed(g["seed"])
        moves, res = [], None
        while res is None:
            before = e.get_state(0)
            res = e.play_mcts(0, g["sims"], g["c"])
            after = e.get_state(0)
            col = next(cc for cc in range(7) for r in range(6) if before.board[r][cc] != after.board[r][cc])
            moves.append(col)
        assert moves == g["moves"]
        assert res == g["result"]


def test_engine_parallel_per_game_streams():
    n, sims = 24, 120
    e = Engine({"game": "connect4", "backend": "c4_backend", "value_function": "random_rollout",
                "threads": n, "seed": 1000})
    boards = [("." * 42, 0)] * n
    res = e.play_mcts_parallel(list(range(n)), sims, 1.4)
    assert set(res) == set(range(n)) and all(r is None for r in res.values())
    # each game's move = the oracle's move for seed 1000+idx (first move of the game)
    omv, _, _ = oracle.get_move_batch(["." * 42] * n, [0] * n, [1000 + i for i in range(n)], sims, 1.4, 32)
    for i in range(n):
        after = e.get_state(i)
        col = next(c for c in range(7) if after.board[5][c] != " ")
        assert col == omv[i]
    # a subset searched alone gives the same second moves as searched together with others
    e2 = Engine({"game": "connect4", "backend": "c4_backend", "value_function": "random_rollout",
                 "threads": n, "seed": 1000})
    e2.play_mcts_parallel(list(range(n)), sims, 1.4)
    e.play_mcts_parallel([3, 5, 7], sims, 1.4)
    e2.play_mcts_parallel(list(range(n)), sims, 1.4)
    for i in (3, 5, 7):
        assert e.get_state(i) == e2.get_state(i)


def test_integration_md_ctypes_stub_works(golden):
    """The ctypes stub shown in INTEGRATION.md §2 runs as written and is a drop-in."""
    import os
    import re
    from conftest import REPO
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = [b for b in re.findall(r"```python\n(.*?)```", text, re.S) if "zc_ctypes" in b][0]
    block = block.replace("/path/to/zeroclone_amd/libzeroclone_amd.so",
                          os.path.join(REPO, "zeroclone_amd", "libzeroclone_amd.so"))
    ns = {}
    exec(compile(block, "INTEGRATION.md", "exec"), ns)
    for c in golden("c4_get_move.json")["cases"][:40]:
        st = c4.State(dec(c["board"]), c["turn"])
        random.seed(c["seed"])
        assert ns["get_move"](st, None, None, None, c["sims"], c["c"], c["bs"]) == (c["move"], 0)
        assert random.getrandbits(32) == c["next_word"]
