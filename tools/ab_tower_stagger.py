#!/usr/bin/env python3
"""A/B of the fused tower's workgroup stagger (ZC_TOWER_STAGGER=cycles[,shift], net_conv.hip
TowerPolicy) in one process, settings alternating: ValueNetwork(128, 8) on 32768 8x8 boards
(the chess batch) and 131072 6x7 boards (Connect4).  Prints ms, TFLOP/s and whether the
outputs equal the unstaggered ones.

    python tools/ab_tower_stagger.py 0 6000 12000 12000,0"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, flops_per_position  # noqa: E402


def main():
    settings = sys.argv[1:] or ["0", "12000"]
    reps = int(os.environ.get("AB_REPS", "5"))
    for (planes, h, w, n) in [(17, 8, 8, 32768), (2, 6, 7, 131072)]:
        torch.manual_seed(0)
        net = MfmaValueNetwork(ValueNetwork(128, 8, in_planes=planes), "cuda")
        g = torch.Generator(device="cuda").manual_seed(1)
        x = (torch.rand(n, planes, h, w, device="cuda", generator=g) < 0.3).half()
        res = {k: [] for k in settings}
        ref = None
        same = {k: True for k in settings}
        for rnd in range(4):
            for k in settings:
                os.environ["ZC_TOWER_STAGGER"] = k
                a, v = net.tower(x, fused=True)
                torch.cuda.synchronize()
                if ref is None:
                    ref = a.clone()
                same[k] &= bool(torch.equal(a, ref))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    net.tower(x, fused=True)
                e1.record()
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) / reps)
        flop = flops_per_position(128, 8, 32, h, w) * n
        for k in settings:
            ms = statistics.median(res[k][1:])
            print(f"{h}x{w}x{n} stagger {k}: {ms:.3f} ms  {flop / ms / 1e9:.0f} TFLOP/s  all {[round(t, 3) for t in res[k]]}"
                  f"  {'identical' if same[k] else 'OUTPUTS DIFFER'}", flush=True)
    os.environ.pop("ZC_TOWER_STAGGER", None)


if __name__ == "__main__":
    main()
