#!/usr/bin/env python3
"""Spread of per-game work over one free-running self-play launch (bench.py's timed launch,
K moves per game): the launch ends with its slowest game, so max/mean of the per-game work
bounds what the tail costs.  Stats fields summed over the launch's K moves."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 60
torch.cuda.set_device(0)
sp = C4SelfPlay(4096, 800, c=1.4, batch_size=32, seed=0, device=0, record=True)
bench.burn_in(sp)
sp.run(8)
torch.cuda.synchronize()
for rep in range(2):
    sp.stats.zero_()
    sp.run(K)
    torch.cuda.synchronize()
    st = sp.stats.cpu().numpy()
    for name, col in (("expansions", 0), ("plies", 3), ("rng_words", 4), ("blocks", 6)):
        x = st[:, col].astype(np.float64)
        q = np.quantile(x, [0.01, 0.5, 0.99, 1.0])
        print(f"K={K} {name:11s} mean {x.mean():10.1f}  p1 {q[0]:10.1f}  p50 {q[1]:10.1f}  p99 {q[2]:10.1f}  max {q[3]:10.1f}"
              f"  max/mean {q[3] / max(x.mean(), 1e-9):.3f}", flush=True)
    # a proxy of per-game time: rollout blocks + expansions weighted by their measured costs
    w = st[:, 6] * 2700.0 + st[:, 0] * 1100.0
    print(f"K={K} weighted work max/mean {w.max() / w.mean():.3f}  p99/mean {np.quantile(w, 0.99) / w.mean():.3f}", flush=True)
sp.close()
