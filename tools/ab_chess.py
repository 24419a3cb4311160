#!/usr/bin/env python3
"""A/B timing of library variants on the chess crude search (BASELINE C4: 1024 games x 400
sims x bs 32, crude_chess_score, immediate_value(3)), from the opening and from mixed roots
(each game a few random plies in), every variant in its own process (ZC_LIB=<path>), rounds
alternating.  Prints the median ms per move per variant and whether the outputs (moves, root
visit counts, per-game counters incl. MT words consumed) hash identically.

    python tools/ab_chess.py zeroclone_amd/libzeroclone_amd.so zeroclone_amd/libzc_variant.so"""
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CHILD = r'''
import sys, time, zlib
sys.path.insert(0, %r)
import numpy as np, torch
from zeroclone_amd import _native
import oracle
G, S, B = 1024, 400, 32
eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B)
rs = np.random.default_rng(5)
roots = []
for i in range(G):
    st = oracle.chess_init()
    for _ in range(int(rs.integers(0, 24)) if i %% 2 else 0):
        ms = oracle.chess_moves(st)
        if not ms:
            break
        nxt = oracle.chess_play(st, ms[int(rs.integers(0, len(ms)))])
        if oracle.chess_win(nxt) or oracle.chess_draw(nxt) or not oracle.chess_moves(nxt):
            break
        st = nxt
    r = np.zeros(1, _native.CHESS_STATE_DTYPE)
    r["board"][0] = np.frombuffer(bytes(st.board), np.uint8)
    r["turn"], r["fifty"], r["castle"] = st.turn, st.fifty, st.castle
    roots.append(r)
roots = torch.from_numpy(np.concatenate(roots).view(np.uint8).reshape(G, 72).copy()).cuda()
mv = torch.zeros(G, dtype=torch.int16, device="cuda")
na = torch.zeros((G, 256), dtype=torch.int32, device="cuda")
st = torch.zeros((G, 8), dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
eng.seed(0, list(range(G)))
ts, h = [], 0
for r in range(7):
    torch.cuda.synchronize()
    t = time.perf_counter()
    eng.chess_search_async(0, G, roots.data_ptr(), S, 1.4, B, 1, 3.0, mv.data_ptr(), na.data_ptr(), st.data_ptr(), s)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t)
    assert int(st[:, 5].abs().sum()) == 0
    for a in (mv, na, st):
        h = zlib.crc32(a.cpu().numpy().tobytes(), h)
ts = sorted(ts[2:])
print(ts[len(ts) // 2] * 1e3, h)
'''


def main():
    libs = sys.argv[1:]
    res = {lib: [] for lib in libs}
    hashes = {}
    for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
        for lib in libs:
            env = dict(os.environ, ZC_LIB=os.path.join(ROOT, lib))
            cp = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True,
                                timeout=300)
            if cp.returncode:
                sys.exit(f"{lib}: child failed ({cp.returncode})\n{cp.stderr[-3000:]}")
            out = cp.stdout
            ms, h = out.strip().splitlines()[-1].split()
            res[lib].append(float(ms))
            hashes.setdefault(lib, set()).add(h)
            print(rnd, lib, res[lib][-1], flush=True)
    ref = hashes[libs[0]]
    for lib in libs:
        same = "outputs identical" if hashes[lib] == ref and len(ref) == 1 else "OUTPUTS DIFFER"
        print(f"{lib}: median {statistics.median(res[lib]):.3f} ms per move  all {res[lib]}  {same}")


if __name__ == "__main__":
    main()
