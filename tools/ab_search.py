#!/usr/bin/env python3
"""A/B timing of library variants on the C2 search (4096 games x 800 sims x bs 32).

    python tools/ab_search.py libA.so libB.so ...   (paths relative to the repo root)

Each round runs every variant in its own process (ZC_LIB=<path>), in turn, so that clock
and thermal drift hit all of them alike; prints the median search time per variant.
AB_ROOTS=mixed searches from mid-game roots (random depths 0..27, the steady-state mix of
self-play) instead of the empty board; AB_MODE=philox times the Philox rollout mode."""
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CHILD = r'''
import sys, time, zlib, torch
sys.path.insert(0, %r)
import numpy as np
from zeroclone_amd import _native
G, S, B = %d, 800, 32
eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B)
if %r == "philox":
    eng.c4_rollout_mode("philox", 12345)
roots = np.zeros(G, _native.C4_STATE_DTYPE)
if %r == "mixed":
    rs = np.random.default_rng(1234)
    def has4(b):
        for sh in (1, 7, 6, 8):
            m = b & (b >> sh)
            if m & (m >> (2 * sh)):
                return True
        return False
    for i in range(G):
        while True:
            st, turn, ok = [0, 0], 0, True
            for _ in range(int(rs.integers(0, 28))):
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
ts, h = [], 0
for r in range(9):
    eng.seed(0, list(range(r * G, (r + 1) * G)))
    t = time.perf_counter()
    out = eng.c4_search(roots, S, 1.4, B)
    ts.append(time.perf_counter() - t)
    for a in out:  # moves, root visit counts, per-game stats (incl. MT words consumed)
        h = zlib.crc32(np.ascontiguousarray(a).tobytes(), h)
ts = sorted(ts[2:])
print(ts[len(ts) // 2] * 1e3, h)
'''


def main():
    libs = sys.argv[1:]
    games = int(os.environ.get("AB_GAMES", "4096"))
    res = {lib: [] for lib in libs}
    hashes = {}
    for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
        for lib in libs:
            env = dict(os.environ, ZC_LIB=os.path.join(ROOT, lib))
            out = subprocess.run([sys.executable, "-c", CHILD % (ROOT, games, os.environ.get("AB_MODE", "exact"), os.environ.get("AB_ROOTS", "empty"))],
                                 env=env, check=True,
                                 capture_output=True, text=True, timeout=300).stdout
            ms, h = out.strip().splitlines()[-1].split()
            res[lib].append(float(ms))
            hashes.setdefault(lib, set()).add(h)
            print(rnd, lib, res[lib][-1], flush=True)
    ref = hashes[libs[0]]
    for lib in libs:
        same = "outputs identical" if hashes[lib] == ref and len(ref) == 1 else "OUTPUTS DIFFER"
        print(f"{lib}: median {statistics.median(res[lib]):.3f} ms  all {res[lib]}  {same}")


if __name__ == "__main__":
    main()
