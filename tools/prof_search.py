#!/usr/bin/env python3
"""The bench's own workload for rocprofv3 passes: C4SelfPlay at 4096 games x 800 sims x bs 32,
burned in to steady state (every slot has finished a game and started another, as bench.py
does), then --steps x G timed moves in one pooled launch (--launch free: --steps moves per game) (c4_selfplay_kernel<false>, the
last launch of the trace; tools/summarize_profile.py --moves K reports it per move)."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=4096)
ap.add_argument("--sims", type=int, default=800)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--launch", choices=["pooled", "free"], default="pooled")
ap.add_argument("--no-burn-in", dest="burn_in", action="store_false")
ap.add_argument("--no-carry", dest="carry", action="store_false",
                help="pooled launches without carry-over (default: a carry warmup launch, then the timed carry "
                     "launch as the trace's last, undrained)")
a = ap.parse_args()
torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream(torch.device("cuda", 0)))
sp = C4SelfPlay(a.games, a.sims, c=1.4, batch_size=a.batch, seed=0, device=0, record=True)
burn = bench.burn_in(sp) if a.burn_in else 0
print(f"burn-in {burn} steps", flush=True)
r = bench.run_steps(sp, a.steps, warmup=2 if a.carry else 0, launch=a.launch, carry=a.carry, drain=False)
print(f"steps {a.steps}: {r['expansions'] / r['dt'] / 1e9:.4f} G expansions/s, "
      f"launch ms {r['launch_ms']:.3f} ({r['launch_ms'] / a.steps:.3f} per move), "
      f"depth {r['depth_sum'] / max(r['expansions'], 1):.3f}", flush=True)
import json  # noqa: E402
print(json.dumps({"expansions": r["expansions"], "depth_sum": r["depth_sum"], "moves": r["moves"],
                  "launch_ms": r["launch_ms"], "lib_sha256": bench.lib_sha()}), flush=True)
sp.close()
