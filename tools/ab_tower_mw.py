#!/usr/bin/env python3
"""The fused 16x16x32 tower with 2 M tiles per wave (the product) against 4 M tiles per wave
(tower_kernel MW = 4: each B fragment read from LDS feeds four MFMAs; each wave half the
pixels), alternating in one process (net switch tower_mw), on the chess 8x8 x 32768 and the
Connect4 6x7 x 131072 batches: ms per tower (HIP events, warm), TFLOP/s, bit-identity.

Round 6: no faster (profiles/r06_ab_tower_mw4.log, DESIGN.md Round 6 "The tower"); the MW = 4
kernel and its tower_mw switch were removed afterwards, so this runs only against that build."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native  # noqa: E402
from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, flops_per_position  # noqa: E402


def main():
    reps, rounds = 10, 5
    for (planes, h, w, n) in [(17, 8, 8, 32768), (2, 6, 7, 131072)]:
        torch.manual_seed(0)
        vnet = ValueNetwork(128, 8, in_planes=planes).eval()
        for m in vnet.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.1, 0.1)
                m.running_var.uniform_(0.5, 1.5)
        net = MfmaValueNetwork(vnet, "cuda")
        x = (torch.rand(n, planes, h, w, device="cuda") < 0.3).half()
        res, outs = {2: [], 4: []}, {}
        for _ in range(rounds):
            for mw in (2, 4):
                _native.net_switch("tower_mw", mw)
                a, v = net.tower(x)
                torch.cuda.synchronize()
                outs[mw] = a.clone()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    net.tower(x)
                e1.record()
                torch.cuda.synchronize()
                res[mw].append(e0.elapsed_time(e1) / reps)
        _native.net_switch("tower_mw", 0)
        flop = flops_per_position(128, 8, 32, h, w) * n
        print(json.dumps({"shape": f"{h}x{w}x{n}",
                          **{f"mw{k}": {"ms": round(statistics.median(v), 4),
                                        "tflops": round(flop / statistics.median(v) / 1e9, 1),
                                        "all_ms": [round(t, 4) for t in v]} for k, v in res.items()},
                          "identical": bool(torch.equal(outs[2], outs[4]))}), flush=True)


if __name__ == "__main__":
    main()
