#!/usr/bin/env python3
"""A/B timing of library variants on the driver line's chess crude figure (bench.py
chess_modes: a burned-in 1024-game pool, one pooled self-play launch of K x 1024 moves of
400 sims), every variant in its own process (ZC_LIB=<path>), rounds alternating.  Pooled
schedules are timing-dependent, so only rates are compared here; outputs are pinned by the
tests (tests/test_gpu_pools.py, tests/test_gpu_chess_selfplay.py).

    python tools/ab_chess_pooled.py zeroclone_amd/libzeroclone_amd.so zeroclone_amd/libzc_variant.so"""
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CHILD = r'''
import sys, time
sys.path.insert(0, %r)
import torch
from bench import chess_burned_pool
from zeroclone_amd import _native
dev = torch.device("cuda", 0)
pool, burn = chess_burned_pool(dev, 1024, 400, 32)
out = []
for K in (20, 20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    res = pool.run_pooled(K * 1024, 2 * K)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    out.append(int(pool.stats[:, 0].sum().item()) / dt)
    pool.take()
print(max(out), burn)
'''


def main():
    libs = sys.argv[1:]
    res = {lib: [] for lib in libs}
    for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
        for lib in libs:
            env = dict(os.environ, ZC_LIB=os.path.join(ROOT, lib))
            cp = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True,
                                timeout=400)
            if cp.returncode:
                sys.exit(f"{lib}: child failed ({cp.returncode})\n{cp.stderr[-3000:]}")
            rate, burn = cp.stdout.strip().splitlines()[-1].split()
            res[lib].append(float(rate))
            print(rnd, lib, f"{float(rate) / 1e6:.1f} M expansions/s (burn-in {burn} moves)", flush=True)
    for lib in libs:
        print(f"{lib}: median {statistics.median(res[lib]) / 1e6:.1f} M expansions/s  all "
              f"{[round(r / 1e6, 1) for r in res[lib]]}")


if __name__ == "__main__":
    main()
