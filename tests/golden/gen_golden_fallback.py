#!/usr/bin/env python3
"""Golden outputs for the §8(b) fallback: plugins whose semantics involve Python's `random`
beyond the built-in Connect4 paths.

Runs ONLY in the build container: the reference's compiled mcts.get_move (oracle/_ref) with
the reference's chess backend (oracle/_ref/chess_backend*.so) and the reference's own
Value / Policy (engine/value_functions.py, engine/policy_functions.py) imported by path.

  chess_rollouts  Value('random_rollout').batch(states, backend=chess_backend) called
                  directly (value_functions.py:35-45 on the chess rules): per state the
                  value and the plies played (a counting backend proxy), then the next word
                  of Python's stream.  States with histories: repetition-prone shuffles,
                  fifty-move counters near 50, bare-king and minor-piece endings.
  chess_search    get_move with Value('random_rollout') on chess (Policy random /
                  immediate_value): move, root visit counts (tagging proxy), leaves, the
                  rollout values in flush order, next word.
  c4_hostvalue    get_move on Connect4 with value objects that draw from `random`
                  (tests/fallback_values.py) and the built-in Policy('random').
  chess_hostvalue the same on chess, incl. a value reading the leaves' move histories.

Usage: make -C oracle ref && python tests/golden/gen_golden_fallback.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import fallback_values as FV  # noqa: E402
import gen_golden as G  # noqa: E402
import gen_golden_chess as GC  # noqa: E402


class Tagged:
    """A reference chess State with the root action it descends from (None at the root)."""
    __slots__ = ("s", "tag")

    def __init__(self, s, tag):
        self.s, self.tag = s, tag

    def __getattr__(self, name):
        return getattr(self.s, name)


class TagChess:
    def __init__(self, cb):
        self.cb = cb
        self.plays = 0

    def get_legal_moves(self, ts):
        return self.cb.get_legal_moves(ts.s)

    def play_move(self, ts, m):
        self.plays += 1
        return Tagged(self.cb.play_move(ts.s, m), ts.tag if ts.tag is not None else tuple(m[0]))

    def check_win(self, ts):
        return self.cb.check_win(ts.s)

    def check_draw(self, ts):
        return self.cb.check_draw(ts.s)

    def state_to_tensor(self, ts):
        return self.cb.state_to_tensor(ts.s)


class Recording:
    """Counts leaves per root tag and logs the values returned, before/after delegating."""

    def __init__(self, inner):
        self.inner = inner
        self.counts = {}
        self.leaves = 0
        self.values = []

    def batch(self, states, **kw):
        for s in states:
            self.counts[s.tag] = self.counts.get(s.tag, 0) + 1
        self.leaves += len(states)
        v = self.inner.batch(states, **kw)
        self.values += [float(x) for x in v]
        return v


def enc_state(s):
    e = GC.enc_state(s)
    e["hw"] = GC.enc_hist(s.hist_white)
    e["hb"] = GC.enc_hist(s.hist_black)
    return e


def play_line(cb, st, moves):
    """Plays ((fr, fc, tr, tc) ...) coordinate moves, matching them against the legal list."""
    for frm in moves:
        legal = {tuple(m[0]): m for m in cb.get_legal_moves(st)}
        st = cb.play_move(st, legal[frm])
    return st


def random_play(cb, st, rng, plies):
    for _ in range(plies):
        if cb.check_win(st) or cb.check_draw(st):
            break
        st = cb.play_move(st, rng.choice(list(cb.get_legal_moves(st))))
    return st


def rollout_states(cb):
    start = cb.create_init_state()
    shuffle = [(7, 6, 5, 5), (0, 6, 2, 5), (5, 5, 7, 6), (2, 5, 0, 6)]   # Ng1-f3 Ng8-f6 Nf3-g1 Nf6-g8
    out = [start,
           play_line(cb, start, shuffle * 2),             # one period short of a repetition draw
           play_line(cb, start, shuffle * 2 + shuffle[:3]),
           play_line(cb, start, [(6, 4, 4, 4), (1, 4, 3, 4)] + shuffle * 2)]
    rng = random.Random(5)
    for plies in (10, 40, 80, 120):
        out.append(random_play(cb, start, rng, plies))
    for fen in ("4k3/8/8/8/8/8/8/4K2R w K - 0 1", "8/8/4k3/8/8/3QK3/8/8 b - - 0 1",
                "8/8/8/4k3/8/8/2N5/4K3 w - - 0 1",      # insufficient material: no legal move
                "4k3/8/8/8/8/8/4P3/4K3 w - - 47 1",     # fifty counter near 50
                "6k1/5ppp/8/8/8/8/5PPP/3R2K1 w - - 0 1", GC.FENS["kiwipete"], GC.FENS["pos3"]):
        out.append(cb.state_from_fen(fen))
    return out


def main():
    mcts, c4, vf, pf = G.load_reference()
    cb = GC.load_ref()
    tb = TagChess(cb)
    fx = {"meta": {"generator": "tests/golden/gen_golden_fallback.py", "values": "tests/fallback_values.py"}}

    # ---- Value('random_rollout').batch on chess, called directly
    rol = vf.Value("random_rollout")
    sts = rollout_states(cb)
    cases = []
    for seed, idx in ((1, list(range(len(sts)))), (2, [0, 1, 2, 3]), (3, [1, 1, 2, 2, 3]),
                      (4, [9, 10, 11, 12]), (5, [4, 5, 6, 7])):
        states = [Tagged(sts[i], None) for i in idx]
        random.seed(seed)
        vals, plies = [], []
        for s in states:   # one at a time: the plies of each rollout (Value.batch == this loop)
            tb.plays = 0
            vals.append(float(rol.batch([s], backend=tb)[0]))
            plies.append(tb.plays)
        cases.append({"seed": seed, "states": [enc_state(sts[i]) for i in idx], "values": vals, "plies": plies,
                      "next_word": random.getrandbits(32)})
    fx["chess_rollouts"] = cases
    print(len(cases), "rollout batches, plies", [c["plies"] for c in cases])

    # ---- get_move with Value('random_rollout') on chess
    def run_chess(st, seed, sims, bs, c, policy, freedom, value):
        pol = pf.Policy("immediate_value", policy_freedom=freedom) if policy == "immediate_value" else pf.Policy("random")
        rec = Recording(value)
        random.seed(seed)
        mv = mcts.get_move(Tagged(st, None), rec, pol, tb, sims, c, bs)
        root_moves = cb.get_legal_moves(st)
        return {"state": enc_state(st), "seed": seed, "sims": sims, "bs": bs, "c": c, "policy": policy,
                "freedom": freedom, "move": list(mv[0]) + [mv[1]],
                "root_moves": [list(m[0]) + [m[1]] for m in root_moves],
                "root_na": [rec.counts.get(tuple(m[0]), 0) for m in root_moves],
                "leaves": rec.leaves, "values": rec.values, "next_word": random.getrandbits(32)}

    cases = []
    for i, (si, seed, sims, bs, pol) in enumerate([(0, 11, 16, 8, "random"), (0, 12, 24, 32, "immediate_value"),
                                                    (1, 13, 20, 4, "random"), (2, 14, 12, 1, "random"),
                                                    (3, 15, 32, 16, "immediate_value"), (5, 16, 16, 8, "random"),
                                                    (7, 17, 24, 5, "immediate_value"), (8, 18, 40, 32, "random"),
                                                    (9, 19, 24, 8, "random"), (13, 20, 16, 16, "immediate_value"),
                                                    (14, 21, 20, 6, "random"), (11, 22, 12, 4, "random")]):
        cases.append(run_chess(sts[si], seed, sims, bs, 1.4, pol, 3.0 if pol == "immediate_value" else 0.0,
                               vf.Value("random_rollout")))
    fx["chess_search"] = cases
    print(len(cases), "chess rollout searches")

    # ---- Connect4 with random-drawing value objects
    tagb = G.TagBackend(c4)

    def run_c4(st, seed, sims, bs, c, vname):
        val = G.RecordingValue(FV.VALUES[vname]())
        root = G.TState(st.board, st.turn, None)
        random.seed(seed)
        mv = mcts.get_move(root, val, pf.Policy("random"), tagb, sims, c, bs)
        order_ = [m[0] for m in list(c4.get_legal_moves(st))]
        return {"board": G.enc(st.board), "turn": st.turn, "seed": seed, "sims": sims, "bs": bs, "c": c,
                "value": vname, "move": mv[0], "root_na": [val.counts.get(col, 0) for col in order_],
                "order": order_, "leaves": val.leaves, "next_word": random.getrandbits(32)}

    cases = []
    init = c4.create_init_state()
    mids = G.random_positions(c4, 4, random.Random(91), 4, 26)
    for i, (st, sims, bs) in enumerate([(init, 100, 32), (init, 64, 1), (mids[0], 200, 8), (mids[1], 150, 32),
                                         (mids[2], 80, 5), (mids[3], 300, 64)]):
        cases.append(run_c4(st, 40 + i, sims, bs, 1.4, ("noisy", "shuffle")[i % 2]))
    fx["c4_hostvalue"] = cases
    print(len(cases), "c4 host-value searches")

    # ---- chess with random-drawing (and history-reading) value objects
    cases = []
    for i, (si, sims, bs, pol, vname) in enumerate([(0, 48, 16, "random", "noisy"), (1, 40, 8, "random", "history"),
                                                     (3, 64, 32, "immediate_value", "history"),
                                                     (6, 32, 4, "random", "shuffle"),
                                                     (14, 48, 12, "immediate_value", "history"),
                                                     (2, 24, 1, "random", "history")]):
        cases.append(run_chess(sts[si], 60 + i, sims, bs, 1.4, pol, 3.0 if pol == "immediate_value" else 0.0,
                               FV.VALUES[vname]()))
        cases[-1]["value"] = vname
    fx["chess_hostvalue"] = cases
    print(len(cases), "chess host-value searches")
    json.dump(fx, open(os.path.join(HERE, "fallback_get_move.json"), "w"))


if __name__ == "__main__":
    main()
