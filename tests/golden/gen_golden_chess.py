#!/usr/bin/env python3
"""Golden fixtures for the chess rules (SURVEY.md §8c fixtures 5-8), from the reference.

Runs ONLY in the build container: imports the reference's chess backend compiled from its
own sources by oracle/Makefile (target `ref`: oracle/_ref/chess_backend*.so, flags of
engine/games/chess/setup.py) and records, as plain data:
  perft      node counts under the reference's rules (no castling / en passant generated,
             queen promotion, insufficient-material exit) for standard test FENs
  movelists  ordered get_legal_moves output with capture values, for positions reached by
             seeded random play from several FENs
  play       play_move results (board, turn, fifty counter, castling flags, history heads)
  terminal   check_win / check_draw, including the reference tests' five FENs
             (tests/test_cb.py:105-116), fifty-move and repetition histories
  tensors    state_to_tensor planes (packed bits)

Usage: make -C oracle ref && python tests/golden/gen_golden_chess.py
"""
import glob
import importlib.util
import json
import os
import random
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))

FENS = {
    "start": "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
    "kiwipete": "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1",
    "pos3": "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1",
    "pos4": "r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1",
    "pos5": "rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8",
    "promo": "8/P6k/8/8/8/8/6Kp/8 w - - 0 1",
}
PERFT = {"start": 5, "kiwipete": 3, "pos3": 4, "pos4": 3, "pos5": 3, "promo": 4}
TEST_CB = [
    ("rnb1kbnr/pppp1ppp/8/4p3/6Pq/5P2/PPPPP2P/RNBQKBNR w KQkq - 0 1", True, False),
    ("r1bqkbnr/ppp2Qpp/n2p4/4p3/2B1P3/8/PPPP1PPP/RNB1K1NR b KQkq - 0 1", True, False),
    ("7k/5Q2/6K1/8/8/8/8/8 b - - 0 1", False, True),
    ("8/8/8/8/8/8/2n5/2K4k w - - 0 1", False, True),
    ("8/8/8/1k6/8/8/4K3/5B2 w - - 0 1", False, True),
]


def load_ref():
    so = glob.glob(os.path.join(REPO, "oracle", "_ref", "chess_backend*.so"))
    if not so:
        raise SystemExit("build the reference first: make -C oracle ref")
    spec = importlib.util.spec_from_file_location("chess_backend", so[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def enc_hist(h):
    """Move history as one string: 'frfctrtc' + capture value digit per move (values are
    0,1,3,5,9), most recent first."""
    return "".join("%d%d%d%d%d" % (m[0][0], m[0][1], m[0][2], m[0][3], int(m[1])) for m in h)


def enc_state(s, hist=False):
    e = {"board": "".join(chr(x) if x else " " for x in s.board), "turn": int(s.turn),
         "fifty": int(s.fifty_move_rule_counter),
         "castle": int(s.w_ck) | int(s.w_cq) << 1 | int(s.b_ck) << 2 | int(s.b_cq) << 3,
         "nhw": len(s.hist_white), "nhb": len(s.hist_black)}
    if hist:
        e["hw"] = enc_hist(s.hist_white)
        e["hb"] = enc_hist(s.hist_black)
    else:
        e["hw_head"] = enc_hist(list(s.hist_white)[:1])
        e["hb_head"] = enc_hist(list(s.hist_black)[:1])
    return e


def enc_moves(ms):
    return [[int(m[0][0]), int(m[0][1]), int(m[0][2]), int(m[0][3]), float(m[1])] for m in ms]


def perft(cb, s, d):
    if d == 0:
        return 1
    ms = cb.get_legal_moves(s)
    if d == 1:
        return len(ms)
    return sum(perft(cb, cb.play_move(s, m), d - 1) for m in ms)


def random_walk(cb, s, rng, plies):
    out = []
    for _ in range(plies):
        ms = cb.get_legal_moves(s)
        if not ms:
            break
        s = cb.play_move(s, rng.choice(ms))
        out.append(s)
    return out


def main():
    cb = load_ref()
    t0 = time.time()
    meta = {"generator": "tests/golden/gen_golden_chess.py", "reference": "engine/games/chess (compiled by oracle/Makefile)"}

    per = []
    for name, fen in FENS.items():
        s = cb.state_from_fen(fen)
        per.append({"name": name, "fen": fen, "counts": [perft(cb, s, d) for d in range(1, PERFT[name] + 1)]})
        print(name, per[-1]["counts"], f"{time.time() - t0:.1f}s", flush=True)
    json.dump({"meta": meta, "perft": per}, open(os.path.join(HERE, "chess_perft.json"), "w"))

    rng = random.Random(2025)
    positions = []
    for name, fen in FENS.items():
        s0 = cb.state_from_fen(fen)
        positions.append(s0)
        for _ in range(12):
            positions += random_walk(cb, s0, rng, rng.randint(1, 60))[-3:]
    init = cb.create_init_state()
    for _ in range(40):
        positions += random_walk(cb, init, rng, rng.randint(20, 160))[-2:]
    mov, play, term, tens = [], [], [], []
    for s in positions:
        ms = cb.get_legal_moves(s)
        e = enc_state(s)
        mov.append({"state": e, "moves": enc_moves(ms)})
        if ms:
            m = rng.choice(ms)
            play.append({"state": e, "move": enc_moves([m])[0], "after": enc_state(cb.play_move(s, m))})
        term.append({"state": enc_state(s, True), "win": bool(cb.check_win(s)), "draw": bool(cb.check_draw(s))})
    for s in positions[::5]:
        t = np.asarray(cb.state_to_tensor(s), np.float32)
        tens.append({"state": enc_state(s), "shape": list(t.shape),
                     "bits": np.packbits((t.reshape(-1) != 0).astype(np.uint8)).tobytes().hex()})
    # the reference tests' FENs, the fifty-move rule and repetition histories
    for fen, w, d in TEST_CB:
        s = cb.state_from_fen(fen)
        term.append({"state": enc_state(s, True), "win": bool(cb.check_win(s)), "draw": bool(cb.check_draw(s)),
                     "expect": [w, d], "fen": fen})
    s = cb.create_init_state()
    bounce = [((7, 6, 5, 5), 0.0), ((0, 6, 2, 5), 0.0), ((5, 5, 7, 6), 0.0), ((2, 5, 0, 6), 0.0)]
    for k in range(16):
        s = cb.play_move(s, bounce[k % 4])
        term.append({"state": enc_state(s, True), "win": bool(cb.check_win(s)), "draw": bool(cb.check_draw(s)),
                     "note": f"knight bounce ply {k + 1}"})
    s = cb.state_from_fen("4k3/8/8/8/8/8/8/R3K3 w - - 47 1")
    for m in [((7, 0, 6, 0), 0.0), ((0, 4, 0, 3), 0.0), ((6, 0, 7, 0), 0.0), ((0, 3, 0, 4), 0.0)]:
        s = cb.play_move(s, m)
        term.append({"state": enc_state(s, True), "win": bool(cb.check_win(s)), "draw": bool(cb.check_draw(s)),
                     "note": "fifty-move counter"})
    # random games played to their end (the reference's terminal tests at every ply)
    for g in range(40):
        s = cb.create_init_state()
        prev = None
        for _ in range(600):
            if cb.check_win(s) or cb.check_draw(s):
                break
            ms = cb.get_legal_moves(s)
            prev = s
            s = cb.play_move(s, rng.choice(ms))
        for x in (prev, s):
            if x is not None:
                term.append({"state": enc_state(x, True), "win": bool(cb.check_win(x)), "draw": bool(cb.check_draw(x)),
                             "note": f"random game {g}"})
    json.dump({"meta": meta, "cases": mov}, open(os.path.join(HERE, "chess_movelists.json"), "w"))
    json.dump({"meta": meta, "cases": play}, open(os.path.join(HERE, "chess_play.json"), "w"))
    json.dump({"meta": meta, "cases": term}, open(os.path.join(HERE, "chess_terminal.json"), "w"))
    json.dump({"meta": meta, "cases": tens}, open(os.path.join(HERE, "chess_tensor.json"), "w"))
    print(len(mov), "positions", f"{time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
