#!/usr/bin/env python3
"""The value tower (ValueNetwork(128, 8)) fused into one launch (zc_net_tower_async) vs one
packed launch per layer, in one process, alternating: the chess C4 batch (32768 boards 8x8,
17 planes) and the Connect4 C2(iii) batch (131072 boards 6x7, 2 planes).  Prints ms per
tower, the tower's TFLOP/s (conv FLOPs of nets.flops_per_position minus nothing: the head is
not run) and whether the outputs are bit-identical."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, flops_per_position  # noqa: E402


def main():
    reps = int(os.environ.get("AB_REPS", "5"))
    out = {}
    for (planes, h, w, n) in [(17, 8, 8, 32768), (2, 6, 7, 131072)]:
        torch.manual_seed(0)
        net = MfmaValueNetwork(ValueNetwork(128, 8, in_planes=planes), "cuda")
        g = torch.Generator(device="cuda").manual_seed(1)
        x = (torch.rand(n, planes, h, w, device="cuda", generator=g) < 0.3).half()
        res = {True: [], False: []}
        outs = {}
        for rnd in range(3):
            for fused in (True, False):
                a, _ = net.tower(x, fused=fused)
                torch.cuda.synchronize()
                outs[fused] = a.clone()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    net.tower(x, fused=fused)
                e1.record()
                torch.cuda.synchronize()
                res[fused].append(e0.elapsed_time(e1) / reps)
        flop = flops_per_position(128, 8, 32, h, w) * n  # the stem on its 32 padded planes
        key = f"{h}x{w}x{n}"
        out[key] = {
            "fused_ms": statistics.median(res[True]), "layered_ms": statistics.median(res[False]),
            "fused_tflops": flop / statistics.median(res[True]) / 1e9,
            "layered_tflops": flop / statistics.median(res[False]) / 1e9,
            "identical": bool(torch.equal(outs[True], outs[False])),
        }
        print(key, json.dumps(out[key]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
