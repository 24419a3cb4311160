#!/usr/bin/env python3
"""Golden get_move outputs with arbitrary policy callables (the §8(b) host-policy fallback).

Runs ONLY in the build container: drives the reference's compiled mcts.get_move
(oracle/_ref, built from /root/reference by `make -C oracle ref`) with the policies of
tests/c4_policies.py, the reference c4_backend, and either the reference's
Value('random_rollout') (so policy and rollouts share Python's stream) or the deterministic
hash value of tests/c4_values.py.  Recorded per case: the move, every policy call (untried
columns in list order and the pick), the leaves, and the next word of Python's stream.

Usage: make -C oracle ref && python tests/golden/gen_golden_hostpolicy.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import c4_policies as P  # noqa: E402
import gen_golden as G  # noqa: E402
from gen_golden_valued import HashValue  # noqa: E402


def main():
    mcts, c4, vf, _ = G.load_reference()
    tagb = G.TagBackend(c4)

    def run(st, seed, sims, bs, c, pname, vname):
        pol = P.Recording(P.make(pname))
        val = G.RecordingValue(vf.Value("random_rollout")) if vname == "random_rollout" else HashValue()
        root = G.TState(st.board, st.turn, None)
        random.seed(seed)
        mv = mcts.get_move(root, val, pol, tagb, sims, c, bs)
        order_ = [m[0] for m in list(c4.get_legal_moves(st))]
        return {"board": G.enc(st.board), "turn": st.turn, "seed": seed, "sims": sims, "bs": bs, "c": c,
                "policy": pname, "value": vname, "move": mv[0], "calls": pol.calls,
                "root_na": [val.counts.get(col, 0) for col in order_], "order": order_, "leaves": val.leaves,
                "next_word": random.getrandbits(32)}

    cases = []
    init = c4.create_init_state()
    for i, pname in enumerate(P.POLICIES):
        cases.append(run(init, 10 + i, 100, 32, 1.4, pname, "random_rollout"))
        cases.append(run(init, 20 + i, 60, 1, 1.4, pname, "hash"))
    mids = G.random_positions(c4, 6, random.Random(77), 4, 28)
    for i, st in enumerate(mids):
        pname = list(P.POLICIES)[i % 3]
        cases.append(run(st, 30 + i, 150, 16, 1.4, pname, "random_rollout" if i % 2 else "hash"))
    meta = {"generator": "tests/golden/gen_golden_hostpolicy.py", "policies": "tests/c4_policies.py"}
    json.dump({"meta": meta, "cases": cases}, open(os.path.join(HERE, "c4_get_move_hostpolicy.json"), "w"))
    print(len(cases), "cases")
    chess_main(mcts, vf)


def chess_main(mcts, vf):
    """Chess: the reference's compiled chess backend, Value('crude_chess_score')."""
    import gen_golden_chess as GC
    cb = GC.load_ref()

    def run(fen, seed, sims, bs, c, pname):
        st = cb.state_from_fen(fen)
        pol = P.ChessRecording(P.make(pname))
        val = G.RecordingValue(vf.Value("crude_chess_score"))
        val.counts = {}
        random.seed(seed)
        mv = mcts.get_move(st, _Counting(val), pol, cb, sims, c, bs)
        return {"fen": fen, "seed": seed, "sims": sims, "bs": bs, "c": c, "policy": pname,
                "move": list(mv[0]) + [mv[1]], "calls": pol.calls, "leaves": val.leaves,
                "next_word": random.getrandbits(32)}

    cases = []
    fens = [GC.FENS["start"], GC.FENS["kiwipete"], GC.FENS["pos4"],
            "r1bqkbnr/pppp1ppp/2n5/4p3/2B1P3/5Q2/PPPP1PPP/RNB1K1NR w KQkq - 2 3"]
    for i, fen in enumerate(fens):
        for k, pname in enumerate(P.CHESS_POLICIES):
            cases.append(run(fen, 100 + 10 * i + k, 48 + 16 * k, (8, 16, 32, 5)[k], 1.4, pname))
    json.dump({"meta": {"generator": "tests/golden/gen_golden_hostpolicy.py", "policies": "tests/c4_policies.py",
                        "value": "crude_chess_score"}, "cases": cases},
              open(os.path.join(HERE, "chess_get_move_hostpolicy.json"), "w"))
    print(len(cases), "chess cases")


class _Counting:
    """Value.batch pass-through that counts leaves (the reference's states carry no tag)."""

    def __init__(self, rec):
        self.rec = rec

    def batch(self, states, **kw):
        self.rec.leaves += len(states)
        return self.rec.inner.batch(states, **kw)


if __name__ == "__main__":
    main()
