#!/usr/bin/env python3
"""Golden get_move outputs with a caller-supplied value function (stepwise search parity).

Runs ONLY in the build container: drives the reference's compiled mcts.get_move (oracle/_ref)
with Policy('random'), the reference c4_backend, and a Value object whose .batch returns
tests/c4_values.hash_value of each leaf — a deterministic, full-precision fp64 value, so the
root visit counts pin the order of the fp64 backups (mcts.cpp:86-96) and the flush protocol
(:112-127).  Root Na is recovered with the same tagging proxies as gen_golden.py.

Usage: make -C oracle ref && python tests/golden/gen_golden_valued.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import gen_golden as G  # noqa: E402
from c4_values import bits_from_rows, hash_value  # noqa: E402


class HashValue:
    def __init__(self):
        self.counts = {}
        self.leaves = 0
        self.calls = 0

    def batch(self, states, **kw):
        self.calls += 1
        out = []
        for s in states:
            self.counts[s.tag] = self.counts.get(s.tag, 0) + 1
            s0, s1 = bits_from_rows(s.board)
            out.append(hash_value(s0, s1, s.turn))
        self.leaves += len(states)
        return out


def main():
    mcts, c4, vf, pf = G.load_reference()
    policy = pf.Policy("random")
    tagb = G.TagBackend(c4)

    def run(st, seed, sims, bs, c):
        val = HashValue()
        root = G.TState(st.board, st.turn, None)
        random.seed(seed)
        mv = mcts.get_move(root, val, policy, tagb, sims, c, bs)
        after = random.getstate()
        order_ = [m[0] for m in list(c4.get_legal_moves(st))]
        return {"board": G.enc(st.board), "turn": st.turn, "seed": seed, "sims": sims, "bs": bs, "c": c,
                "move": mv[0], "order": order_, "root_na": [val.counts.get(col, 0) for col in order_],
                "leaves": val.leaves, "flushes": val.calls, "consumed": G.consumed_since(seed, after),
                "next_word": random.getrandbits(32)}

    cases = []
    init = c4.create_init_state()
    for seed in range(8):
        cases.append(run(init, seed, 100, 32, 1.4))
    for seed in range(4):
        cases.append(run(init, seed, 800, 32, 1.4))
    for seed in range(4):
        cases.append(run(init, 40 + seed, 100, 1, 1.4))
    prng = random.Random(123)
    mids = G.random_positions(c4, 12, prng, 2, 30)
    for i, st in enumerate(mids):
        cases.append(run(st, 300 + i, 200, 16, 1.4))
    deep = G.random_positions(c4, 6, random.Random(321), 30, 40)
    for i, st in enumerate(deep):
        cases.append(run(st, 400 + i, 300, 32, 1.4))
    cases.append(run(init, 11, 50, 32, 1.4))    # one partial flush
    cases.append(run(init, 12, 333, 64, 0.0))
    cases.append(run(init, 13, 257, 100, 2.5))
    won = []
    prng = random.Random(8)
    while len(won) < 3:
        st = G.random_positions(c4, 1, prng, 7, 30, allow_terminal=True)[0]
        if c4.check_win(st) and c4.get_legal_moves(st):
            won.append(st)
    for i, st in enumerate(won):
        cases.append(run(st, 500 + i, 200, 32, 1.4))
    meta = {"generator": "tests/golden/gen_golden_valued.py", "value": "tests/c4_values.hash_value"}
    json.dump({"meta": meta, "cases": cases}, open(os.path.join(HERE, "c4_get_move_valued.json"), "w"))
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
