#!/usr/bin/env python3
"""Spread of per-game work in one steady-state move (bench.py's workload): rollout blocks,
plies and expansions per game, as quantiles / mean — the tail a launch waits for."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay  # noqa: E402

torch.cuda.set_device(0)
sp = C4SelfPlay(4096, 800, c=1.4, batch_size=32, seed=0, device=0, record=True)
bench.burn_in(sp)
for _ in range(3):
    sp.step()
    st = sp.stats.cpu().numpy()
    for name, col in (("expansions", 0), ("depth_sum", 1), ("plies", 3), ("rng_words", 4), ("blocks", 6)):
        x = st[:, col].astype(np.float64)
        q = np.quantile(x, [0.5, 0.9, 0.99, 1.0])
        print(f"{name:11s} mean {x.mean():9.1f}  p50 {q[0]:9.1f}  p90 {q[1]:9.1f}  p99 {q[2]:9.1f}  max {q[3]:9.1f}"
              f"  max/mean {q[3] / max(x.mean(), 1e-9):.3f}", flush=True)
sp.close()

# per-game wall cycles of one stamped move (s_memtime, every phase of the search summed)
sp = C4SelfPlay(4096, 800, c=1.4, batch_size=32, seed=0, device=0, record=True)
bench.burn_in(sp)
sp.eng.phase_cycles(True)
roots = sp.roots.cpu().numpy().copy()
sp.step()
torch.cuda.synchronize()
pg = sp.eng.phase_cycles_games(4096).sum(axis=1).astype(np.float64)
sp.eng.phase_cycles(False)
empty = np.array([42 - bin(int(r[0]) | int(r[1])).count("1") for r in roots.view(np.uint64).reshape(-1, 3)[:, :2]])
q = np.quantile(pg, [0.1, 0.5, 0.9, 0.99, 1.0])
print("per-game cycles p10 %.0f p50 %.0f p90 %.0f p99 %.0f max %.0f  mean %.0f  max/mean %.3f" % (*q, pg.mean(), q[-1] / pg.mean()))
for lo, hi in ((0, 10), (10, 20), (20, 30), (30, 43)):
    sel = (empty >= lo) & (empty < hi)
    if sel.any():
        print(f"empty cells [{lo},{hi}): {sel.sum():5d} games, mean cycles {pg[sel].mean():.0f}, max {pg[sel].max():.0f}")
sp.close()
