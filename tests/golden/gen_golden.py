#!/usr/bin/env python3
"""Generate the committed golden fixtures for Connect4 MCTS parity.

Runs ONLY in the build container (it needs /root/reference, which never travels to the
GPU box).  It drives the reference's own code, unmodified:

* ``engine/mcts/src/mcts.cpp`` + ``bindings_mcts.cpp`` compiled by ``oracle/Makefile`` (target
  ``ref``) into ``oracle/_ref/mcts*.so`` with the reference's flags (engine/mcts/setup.py:9);
* ``engine/games/connect4/c4_backend.py``, ``engine/value_functions.py`` (``random_rollout``,
  :35-45) and ``engine/policy_functions.py`` (``random``, :10-12), imported by file path.

Root visit counts are recovered through the plugin seams only: the root
state is a 3-field namedtuple ``(board, turn, tag)``; c4_backend.play_move builds children
with ``state._replace`` (c4_backend.py:23) so a tag set on the root's children is inherited
by every descendant, and a recording ``Value`` counts evaluated leaves per tag before
delegating to the reference ``Value.batch``.  Neither wrapper touches ``random``.

Output: small JSON files in this directory (data only: inputs and expected outputs).
Usage:  make -C oracle ref && python tests/golden/gen_golden.py
"""
from __future__ import annotations

import collections
import importlib.util
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = os.environ.get("ZC_REFERENCE", "/root/reference")


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    import glob
    so = glob.glob(os.path.join(REPO, "oracle", "_ref", "mcts*.so"))
    if not so:
        raise SystemExit("build the reference first: make -C oracle ref")
    mcts = _load("mcts", so[0])
    c4 = _load("ref_c4_backend", os.path.join(REF, "engine/games/connect4/c4_backend.py"))
    vf = _load("ref_value_functions", os.path.join(REF, "engine/value_functions.py"))
    pf = _load("ref_policy_functions", os.path.join(REF, "engine/policy_functions.py"))
    return mcts, c4, vf, pf


TState = collections.namedtuple("TState", ["board", "turn", "tag"])


class TagBackend:
    """Module-like proxy: play_move on an untagged (root) state tags the child with its column."""

    def __init__(self, c4):
        self.c4 = c4

    def play_move(self, state, move):
        child = self.c4.play_move(state, move)
        if getattr(state, "tag", "absent") is None:
            child = child._replace(tag=move[0])
        return child

    def __getattr__(self, name):
        return getattr(self.c4, name)


class RecordingValue:
    def __init__(self, inner):
        self.inner = inner
        self.counts = collections.Counter()
        self.leaves = 0

    def batch(self, states, **kw):
        for s in states:
            self.counts[s.tag] += 1
        self.leaves += len(states)
        return self.inner.batch(states, **kw)


def enc(board):
    return "".join("." if ch == " " else ch for row in board for ch in row)


def dec(s):
    return [[(" " if ch == "." else ch) for ch in s[r * 7:(r + 1) * 7]] for r in range(6)]


def consumed_since(seed, after_state, limit=2_000_000):
    r = random.Random(seed)
    n = 0
    while r.getstate() != after_state:
        r.getrandbits(32)
        n += 1
        if n > limit:
            raise RuntimeError("consumption not found")
    return n


def random_positions(c4, n, rng, min_ply=1, max_ply=38, allow_terminal=False):
    out = []
    while len(out) < n:
        st = c4.create_init_state()
        k = rng.randint(min_ply, max_ply)
        ok = True
        for _ in range(k):
            mv = sorted(c4.get_legal_moves(st))
            if not mv:
                ok = False
                break
            st = c4.play_move(st, rng.choice(mv))
            if c4.check_win(st) or c4.check_draw(st):
                if allow_terminal:
                    break
                ok = False
                break
        if ok or allow_terminal:
            out.append(st)
    return out


def main():
    mcts, c4, vf, pf = load_reference()
    t0 = time.time()
    meta = {"generator": "tests/golden/gen_golden.py", "python": sys.version.split()[0],
            "reference": "rishabhgoel0213/ZeroClone @ /root/reference (see SURVEY.md)"}

    # 1. CPython MT19937 known answers (random.seed(int) -> init_by_array; getrandbits; _randbelow)
    mt = {"meta": meta, "seeds": []}
    for seed in [0, 1, 7, 42, 12345, 2**32 + 7, 987654321987654321]:
        r = random.Random(seed)
        st = r.getstate()[1]
        entry = {"seed": seed, "state0_first8": list(st[:8]), "state0_last": st[623], "index0": st[624],
                 "getrandbits32": [r.getrandbits(32) for _ in range(16)]}
        r = random.Random(seed)
        entry["randbelow"] = {str(n): [r.randrange(n) for _ in range(24)] for n in [1, 2, 3, 4, 5, 6, 7, 20, 33, 50]}
        mt["seeds"].append(entry)
    r = random.Random(0)
    mt["seed0_state"] = list(r.getstate()[1])
    json.dump(mt, open(os.path.join(HERE, "mt19937_kat.json"), "w"))

    # 2. CPython set-iteration order of {(i,0) for legal i} per legal-column mask (c4_backend.py:49-50)
    order = {}
    for mask in range(128):
        s = {(i, 0) for i in range(7) if (mask >> i) & 1}
        order[mask] = [m[0] for m in list(s)]
    json.dump({"meta": meta, "order": order}, open(os.path.join(HERE, "c4_set_order.json"), "w"))

    # 3. Backend fixtures: legal move list (set order), check_win, check_draw, state_to_tensor planes
    prng = random.Random(2024)
    poss = random_positions(c4, 300, prng, 0, 42, allow_terminal=True)
    back = []
    for st in poss:
        t = c4.state_to_tensor(st)
        back.append({"board": enc(st.board), "turn": st.turn,
                     "legal": [m[0] for m in list(c4.get_legal_moves(st))],
                     "win": bool(c4.check_win(st)), "draw": bool(c4.check_draw(st)),
                     "cur": "".join("1" if v else "0" for v in t[0].ravel()),
                     "opp": "".join("1" if v else "0" for v in t[1].ravel())})
    json.dump({"meta": meta, "cases": back}, open(os.path.join(HERE, "c4_backend.json"), "w"))

    # 4. Rollout goldens: Value('random_rollout') (value_functions.py:35-45)
    val = vf.Value("random_rollout")
    rolls = []
    prng = random.Random(77)
    starts = [c4.create_init_state()] + random_positions(c4, 150, prng, 1, 41, allow_terminal=True)
    for i, st in enumerate(starts):
        seed = 1000 + i
        random.seed(seed)
        v = val(st, backend=c4)
        rolls.append({"board": enc(st.board), "turn": st.turn, "seed": seed, "value": v,
                      "consumed": consumed_since(seed, random.getstate())})
    json.dump({"meta": meta, "cases": rolls}, open(os.path.join(HERE, "c4_rollout.json"), "w"))

    # 5. get_move goldens: move + root Na per move (in the root's move-list order) + RNG words consumed
    policy = pf.Policy("random")
    tagb = TagBackend(c4)

    def run_get_move(st, seed, sims, bs, c):
        rec = RecordingValue(vf.Value("random_rollout"))
        root = TState(st.board, st.turn, None)
        random.seed(seed)
        mv = mcts.get_move(root, rec, policy, tagb, sims, c, bs)
        after = random.getstate()
        order_ = [m[0] for m in list(c4.get_legal_moves(st))]
        return {"board": enc(st.board), "turn": st.turn, "seed": seed, "sims": sims, "bs": bs, "c": c,
                "move": mv[0], "order": order_, "root_na": [rec.counts[col] for col in order_],
                "leaves": rec.leaves, "consumed": consumed_since(seed, after),
                "next_word": random.getrandbits(32)}

    cases = []
    init = c4.create_init_state()
    for seed in range(32):
        cases.append(run_get_move(init, seed, 100, 1, 1.4))
    for seed in range(32):
        cases.append(run_get_move(init, seed, 100, 32, 1.4))
    for seed in range(8):
        cases.append(run_get_move(init, seed, 800, 32, 1.4))
    prng = random.Random(99)
    mids = random_positions(c4, 24, prng, 2, 30)
    for i, st in enumerate(mids):
        cases.append(run_get_move(st, 500 + i, 100, 32, 1.4))
        cases.append(run_get_move(st, 600 + i, 200, 8, 1.4))
    for i, st in enumerate(mids[:6]):
        cases.append(run_get_move(st, 700 + i, 800, 32, 1.4))
    # edge cases: single sim, partial final flush, other c, near-full boards, already-won roots
    cases.append(run_get_move(init, 3, 1, 1, 1.4))
    cases.append(run_get_move(init, 4, 1, 32, 1.4))
    cases.append(run_get_move(init, 5, 7, 32, 1.4))
    cases.append(run_get_move(init, 6, 50, 32, 1.4))
    cases.append(run_get_move(init, 7, 333, 64, 1.4))
    cases.append(run_get_move(init, 8, 100, 32, 0.0))
    cases.append(run_get_move(init, 9, 100, 32, 2.5))
    cases.append(run_get_move(init, 10, 257, 100, 1.25))
    prng = random.Random(5)
    deep = random_positions(c4, 10, prng, 30, 40)
    for i, st in enumerate(deep):
        cases.append(run_get_move(st, 800 + i, 300, 32, 1.4))
    prng = random.Random(6)
    won = []
    while len(won) < 6:
        st = random_positions(c4, 1, prng, 7, 30, allow_terminal=True)[0]
        if c4.check_win(st) and c4.get_legal_moves(st):
            won.append(st)
    for i, st in enumerate(won):
        cases.append(run_get_move(st, 900 + i, 200, 32, 1.4))
    json.dump({"meta": meta, "cases": cases}, open(os.path.join(HERE, "c4_get_move.json"), "w"))

    # 6. Self-play: one global RNG stream across moves (random.seed once per game), 100 sims, bs 32
    games = []
    for seed in range(4):
        random.seed(seed)
        st = c4.create_init_state()
        moves = []
        value = vf.Value("random_rollout")
        while not (c4.check_win(st) or c4.check_draw(st)):
            mv = mcts.get_move(st, value, policy, c4, 100, 1.4, 32)
            moves.append(mv[0])
            st = c4.play_move(st, mv)
        result = (st.turn * 2 - 1) if c4.check_win(st) else 0   # engine.py:148-153
        games.append({"seed": seed, "sims": 100, "bs": 32, "c": 1.4, "moves": moves, "result": result,
                      "consumed": consumed_since(seed, random.getstate())})
    json.dump({"meta": meta, "games": games}, open(os.path.join(HERE, "c4_selfplay.json"), "w"))
    print(f"golden fixtures written in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
