#!/usr/bin/env python3
"""Network-mode self-play pools as bench.py times them, `--steps` steps — for
`rocprofv3 --kernel-trace --stats` (the kernel shares of a step: tower, policy GEMM, the
search's select / backup, play, record) and for same-box A/Bs (tools/ab_c5.sh).

  c5      C5 per GPU: chess PUCT, 1024 games x 1600 sims, policy + value ResNet 128x8 fp16
  chess   C4: chess value network, 1024 games x 400 sims, ValueNetwork(128, 8)
  c2net   C2(iii): Connect4 value network, 4096 games x 800 sims, ValueNetwork(128, 8, 2)
  c2puct  C2 + PUCT: Connect4, 4096 x 800, policy (7 logits) + value ResNet
ZC_STREAMS=k (chess, c2net, c2puct) / ZC_PUCT_STREAMS=k (c5): the games in k parts on k streams.
Prints ms per step."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd import _native  # noqa: E402
from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork, ValueNetwork, for_inference  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay, ChessSelfPlay  # noqa: E402


def make_pool(mode, dev):
    torch.manual_seed(0)
    if mode in ("c5", "chess"):
        crude, burn = bench.chess_burned_pool(dev)
        if mode == "c5":
            net = MfmaPolicyValueNetwork(PolicyValueNetwork(head=os.environ.get("ZC_C5_HEAD", "conv")).eval(), dev)
            pool = ChessSelfPlay(1024, 1600, batch_size=32, seed=6, device=0, puct_net=net, temperature=1.0,
                                 puct_streams=int(os.environ.get("ZC_PUCT_STREAMS", "1")))
        else:
            model = for_inference(ValueNetwork(128, 8).eval(), dev, torch.float16)
            pool = ChessSelfPlay(1024, 400, batch_size=32, seed=4, device=0, net=model,
                                 policy=_native.ZC_POLICY_RANDOM, freedom=0.0,
                                 streams=int(os.environ.get("ZC_STREAMS", "1")))
        pool.adopt(crude)
        crude.close()
        return pool, burn
    src = C4SelfPlay(4096, 800, batch_size=32, seed=2024, device=0, record=True)
    burn = bench.burn_in(src)
    if mode == "c2net":
        model = for_inference(ValueNetwork(128, 8, in_planes=2).eval(), dev, torch.float16)
        pool = C4SelfPlay(4096, 800, batch_size=32, seed=7, device=0, net=model,
                          streams=int(os.environ.get("ZC_STREAMS", "1")))
    else:
        net = MfmaPolicyValueNetwork(PolicyValueNetwork(in_planes=2, board=(6, 7), n_logits=7).eval(), dev)
        pool = C4SelfPlay(4096, 800, batch_size=32, seed=7, device=0, puct_net=net, temperature=1.0,
                          streams=int(os.environ.get("ZC_STREAMS", "1")))
    pool.adopt(src)
    src.close()
    return pool, burn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="c5", choices=["c5", "chess", "c2net", "c2puct"])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--graph", action="store_true", help="replay a captured step graph instead of eager steps")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    pool, burn = make_pool(a.mode, dev)
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
    if hasattr(pool, "check"):
        pool.check()
    print(f"{a.mode} step: {dt * 1e3:.1f} ms ({'graph' if a.graph else 'eager'}), burn-in {burn}", flush=True)
    pool.close()


if __name__ == "__main__":
    main()
