#!/usr/bin/env python3
"""Golden chess get_move outputs from the reference (SURVEY.md §8c fixture 9).

Runs ONLY in the build container: the reference's compiled mcts.get_move (oracle/_ref) with
the reference chess backend (oracle/_ref/chess_backend*.so), Value('crude_chess_score') and
Policy('immediate_value', policy_freedom=3) — configs/crude_chess.yaml — or Policy('random').
Root visit counts come out through plugin seams only: states are wrapped in a tagging proxy
(the root's children carry their move) and a recording Value counts leaves per tag before
delegating to the reference Value.batch.  Neither wrapper touches `random`.

Usage: make -C oracle ref && python tests/golden/gen_golden_chess_search.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402
import gen_golden_chess as GC  # noqa: E402


class Tagged:
    __slots__ = ("s", "tag")

    def __init__(self, s, tag):
        self.s, self.tag = s, tag

    @property
    def board(self):
        return self.s.board

    @property
    def turn(self):
        return self.s.turn


class TagChess:
    def __init__(self, cb):
        self.cb = cb

    def get_legal_moves(self, ts):
        return self.cb.get_legal_moves(ts.s)

    def play_move(self, ts, m):
        return Tagged(self.cb.play_move(ts.s, m), ts.tag if ts.tag is not None else tuple(m[0]))

    def check_win(self, ts):
        return self.cb.check_win(ts.s)

    def check_draw(self, ts):
        return self.cb.check_draw(ts.s)

    def state_to_tensor(self, ts):
        return self.cb.state_to_tensor(ts.s)


class Recording:
    def __init__(self, inner):
        self.inner = inner
        self.counts = {}
        self.leaves = 0

    def batch(self, states, **kw):
        for s in states:
            self.counts[s.tag] = self.counts.get(s.tag, 0) + 1
        self.leaves += len(states)
        return self.inner.batch(states, **kw)


def main():
    mcts, _, vf, pf = G.load_reference()
    cb = GC.load_ref()
    tb = TagChess(cb)

    def run(fen, seed, sims, bs, c, policy, freedom):
        st = cb.state_from_fen(fen)
        pol = pf.Policy("immediate_value", policy_freedom=freedom) if policy == "immediate_value" else pf.Policy("random")
        rec = Recording(vf.Value("crude_chess_score"))
        random.seed(seed)
        mv = mcts.get_move(Tagged(st, None), rec, pol, tb, sims, c, bs)
        after = random.getstate()
        root_moves = cb.get_legal_moves(st)
        return {"fen": fen, "seed": seed, "sims": sims, "bs": bs, "c": c, "policy": policy, "freedom": freedom,
                "move": list(mv[0]) + [mv[1]],
                "root_moves": [list(m[0]) + [m[1]] for m in root_moves],
                "root_na": [rec.counts.get(tuple(m[0]), 0) for m in root_moves],
                "leaves": rec.leaves, "consumed": G.consumed_since(seed, after),
                "next_word": random.getrandbits(32)}

    fens = list(GC.FENS.values()) + [
        "r1bqkbnr/pppp1ppp/2n5/4p3/2B1P3/5Q2/PPPP1PPP/RNB1K1NR w KQkq - 2 3",   # mate in one (Qxf7#)
        "6k1/5ppp/8/8/8/8/5PPP/3R2K1 w - - 0 1",                                # back-rank mate
        "4k3/8/8/8/8/8/8/4K2R w K - 0 1",
    ]
    cases = []
    for i, fen in enumerate(fens):
        cases.append(run(fen, 10 + i, 100, 32, 1.4, "immediate_value", 3))
        cases.append(run(fen, 30 + i, 100, 8, 1.4, "random", 0))
    for seed in range(4):
        cases.append(run(GC.FENS["start"], seed, 400, 32, 1.4, "immediate_value", 3))
    cases.append(run(GC.FENS["kiwipete"], 7, 400, 32, 1.4, "immediate_value", 3))
    cases.append(run(GC.FENS["start"], 8, 64, 1, 1.4, "immediate_value", 3))
    cases.append(run(GC.FENS["pos4"], 9, 300, 64, 2.0, "random", 0))
    cases.append(run(GC.FENS["pos5"], 11, 250, 32, 0.5, "immediate_value", 0))
    json.dump({"meta": {"generator": "tests/golden/gen_golden_chess_search.py",
                        "config": "configs/crude_chess.yaml (crude_chess_score, immediate_value, policy_freedom 3)"},
               "cases": cases}, open(os.path.join(HERE, "chess_get_move.json"), "w"))
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
