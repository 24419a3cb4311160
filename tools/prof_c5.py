#!/usr/bin/env python3
"""C5 self-play moves (bench.puct_mode: chess PUCT, 1024 games x 1600 sims, policy + value
network) from a burned-in crude pool, for rocprofv3 --kernel-trace --stats: the kernel split
of the PUCT search with the network.  --steps moves (default 1)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=1)
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
crude, burn = bench.chess_burned_pool(dev)
print(f"burn-in {burn} moves", flush=True)
print(bench.puct_mode(crude, a.steps, dev), flush=True)
crude.close()
