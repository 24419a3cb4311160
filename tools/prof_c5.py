#!/usr/bin/env python3
"""C5 per GPU (chess PUCT self-play, 1024 games x 1600 sims, policy + value ResNet 128x8 fp16,
Dirichlet noise, temperature 1) from a burned-in crude pool, `--steps` eager steps — for
`rocprofv3 --kernel-trace --stats` (the kernel shares of the C5 step: tower + policy conv,
the policy Linear GEMM, puct select / backup, play, record).  Prints ms per step."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork  # noqa: E402
from zeroclone_amd.selfplay import ChessSelfPlay  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--graph", action="store_true", help="replay a captured step graph instead of eager steps")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    crude, burn = bench.chess_burned_pool(dev)
    torch.manual_seed(0)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork().eval(), dev)
    pool = ChessSelfPlay(1024, 1600, batch_size=32, seed=6, device=0, puct_net=net, temperature=1.0)
    pool.adopt(crude)
    crude.close()
    if a.graph:
        g = pool.capture_step()
        run = g.replay
    else:
        run = pool.step
    run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / a.steps
    pool.check()
    print(f"C5 step: {dt * 1e3:.1f} ms ({'graph' if a.graph else 'eager'}), burn-in {burn} moves", flush=True)
    pool.close()


if __name__ == "__main__":
    main()
