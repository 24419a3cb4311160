#!/usr/bin/env python3
"""Golden get_move outputs for game backends the device does not know.

Runs ONLY in the build container: drives the reference's compiled mcts.get_move
(oracle/_ref, `make -C oracle ref`) with the toy backends of tests/toy_games (tic-tac-toe,
a subtraction game whose moves are strings in a tuple), the reference's own
Policy('random') and Value('random_rollout') (engine/policy_functions.py,
engine/value_functions.py, imported by path: the rollout then plays the toy game through
its backend) or the plugins of tests/toy_games/plugins.py.  Recorded per case: the move,
every policy call (untried moves in list order, the pick), every flush's leaves, and the
next word of Python's stream.

Usage: make -C oracle ref && python tests/golden/gen_golden_generic.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import gen_golden as G  # noqa: E402
from toy_games import pile_backend, plugins, ttt_backend  # noqa: E402

GAMES = {"ttt": ttt_backend, "pile": pile_backend}


def main():
    mcts, _, vf, pf = G.load_reference()

    def run(game, state, seed, sims, bs, c, pname, vname):
        be = GAMES[game]
        inner = pf.Policy("random") if pname == "random" else plugins.POLICIES[pname]
        pol = plugins.Recording(inner)
        v = vf.Value("random_rollout") if vname == "random_rollout" else plugins.HashValue(be.encode)
        val = plugins.RecordingValue(v, be.encode)
        random.seed(seed)
        mv = mcts.get_move(state, val, pol, be, sims, c, bs)
        return {"game": game, "state": be.encode(state), "seed": seed, "sims": sims, "bs": bs, "c": c,
                "policy": pname, "value": vname, "move": mv, "calls": pol.calls, "flushes": val.flushes,
                "next_word": random.getrandbits(32)}

    cases = []
    T = ttt_backend
    mids = [T.create_init_state()]
    for seq in ([4], [0, 4, 8], [4, 0, 2, 6], [0, 1, 3, 4, 2]):   # the last one: X has already won
        s = T.create_init_state()
        for m in seq:
            s = T.play_move(s, m)
        mids.append(s)
    k = 0
    for i, st in enumerate(mids):
        for pname, vname, sims, bs, c in (("random", "random_rollout", 200, 8, 1.4), ("last_move", "hash", 150, 32, 1.4),
                                          ("shuffled_first", "random_rollout", 120, 1, 0.7),
                                          ("random", "hash", 400, 16, 2.0)):
            cases.append(run("ttt", st, 500 + k, sims, bs, c, pname, vname))
            k += 1
    P = pile_backend
    for i, pile in enumerate((21, 10, 5)):
        st = P.State(pile, i & 1)
        cases.append(run("pile", st, 900 + i, 150, 8, 1.4, "random", "random_rollout"))
        cases.append(run("pile", st, 910 + i, 90, 4, 1.4, "shuffled_first", "hash"))
    meta = {"generator": "tests/golden/gen_golden_generic.py", "backends": "tests/toy_games"}
    json.dump({"meta": meta, "cases": cases}, open(os.path.join(HERE, "generic_get_move.json"), "w"))
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
