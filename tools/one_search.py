#!/usr/bin/env python3
"""One C2-shaped search (4096 games x 800 sims x bs 32), repeated --reps times: a small
fixed workload for rocprofv3 kernel traces and PMC passes."""
import argparse
import os
import sys

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from zeroclone_amd import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=4096)
ap.add_argument("--sims", type=int, default=800)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--mode", default="exact", choices=["exact", "philox"])
a = ap.parse_args()
eng = _native.NativeEngine(max_games=a.games, max_sims=a.sims, max_batch=a.batch)
eng.c4_rollout_mode(a.mode, 7)
roots = np.zeros(a.games, _native.C4_STATE_DTYPE)
tot = 0
for r in range(a.reps):
    eng.seed(0, list(range(r * a.games, (r + 1) * a.games)))
    mv, na, st = eng.c4_search(roots, a.sims, 1.4, a.batch)
    tot += int(st["expansions"].sum())
    print(f"rep {r}: expansions {int(st['expansions'].sum())} depth_sum {int(st['depth_sum'].sum())}", flush=True)
print("total expansions", tot)
