"""Per-game outputs (move, MT words consumed, expansions) of two library builds on the same
2048 random roots of depth 0..39, at several sims / batch sizes; prints the games that differ.

    python tools/cmp_libs.py libA.so libB.so"""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json
sys.path.insert(0, %r)
import numpy as np, torch
from zeroclone_amd import _native
G, S, B = 2048, %d, %d
eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B)
rs = np.random.default_rng(7)
def has4(b):
    for sh in (1, 7, 6, 8):
        m = b & (b >> sh)
        if m & (m >> (2 * sh)):
            return True
    return False
roots = np.zeros(G, _native.C4_STATE_DTYPE)
depths = []
for i in range(G):
    while True:
        st, turn, ok = [0, 0], 0, True
        dep = int(rs.integers(0, 40))
        for _ in range(dep):
            occ = st[0] | st[1]
            cols = [c for c in range(7) if not (occ >> (7 * c + 5)) & 1]
            c = int(rs.choice(cols))
            st[turn] |= (occ + (1 << (7 * c))) & (0x3F << (7 * c))
            if has4(st[turn]):
                ok = False
                break
            turn ^= 1
        if ok:
            break
    roots[i]["stones"] = st
    roots[i]["turn"] = turn
    depths.append(dep)
eng.seed(0, list(range(G)))
mv, na, st = eng.c4_search(roots, S, 1.4, B)
print(json.dumps({"mv": mv.tolist(), "words": st["rng_words"].tolist(), "exp": st["expansions"].tolist(), "dep": depths}))
'''
def run(lib, S, B):
    env = dict(os.environ, ZC_LIB=os.path.join(ROOT, lib))
    out = subprocess.run([sys.executable, "-c", CHILD % (ROOT, S, B)], env=env, check=True, capture_output=True, text=True, timeout=300).stdout
    return json.loads(out.strip().splitlines()[-1])
for S, B in [(7, 7), (9, 3), (40, 8), (200, 8), (800, 32), (300, 64), (500, 63)]:
    a, b = run(sys.argv[1], S, B), run(sys.argv[2], S, B)
    bad = [i for i in range(len(a["mv"])) if (a["mv"][i], a["words"][i], a["exp"][i]) != (b["mv"][i], b["words"][i], b["exp"][i])]
    print(S, B, "differ:", len(bad), "of", len(a["mv"]))
    for i in bad[:12]:
        print("  game", i, "depth", a["dep"][i], "mv", a["mv"][i], b["mv"][i], "words", a["words"][i], b["words"][i], "exp", a["exp"][i], b["exp"][i])
