#!/usr/bin/env python3
"""The fused 16x16x32 tower on its two activation layouts, alternating in one process
(zc_debug_net_switch "tower_epi": 0 = padded 144-half rows, the batched b64 epilogue; 3 = the
swizzled 256-byte rows with the 16-byte epilogue): chess 8x8 x 32768 boards and Connect4 6x7 x
131072 boards, random-init ValueNetwork(128, 8).  Prints ms and TFLOP/s per form and whether
the outputs are bit-identical (they must be: the same operations in the same order)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, flops_per_position  # noqa: E402
from zeroclone_amd import _native  # noqa: E402


def main():
    reps = int(os.environ.get("AB_REPS", "10"))
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    forms = [int(x) for x in os.environ.get("AB_FORMS", "0,3").split(",")]
    out = {}
    for (planes, h, w, n) in [(17, 8, 8, 32768), (2, 6, 7, 131072)]:
        torch.manual_seed(0)
        net = MfmaValueNetwork(ValueNetwork(128, 8, in_planes=planes).eval(), "cuda")
        x = (torch.rand(n, planes, h, w, device="cuda") < 0.3).half()
        flop = flops_per_position(128, 8, 32, h, w) * n
        res, outs, vals = {f: [] for f in forms}, {}, {}
        for _ in range(rounds):
            for f in forms:
                _native.net_switch("tower_epi", f)
                a, v = net.tower(x)
                torch.cuda.synchronize()
                outs[f] = a.clone()
                vals[f] = net(x).clone()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    net.tower(x)
                e1.record()
                torch.cuda.synchronize()
                res[f].append(e0.elapsed_time(e1) / reps)
        _native.net_switch("tower_epi", 0)
        key = f"{h}x{w}x{n}"
        out[key] = {str(f): {"ms": round(statistics.median(res[f]), 4),
                             "tflops": round(flop / statistics.median(res[f]) / 1e9, 1),
                             "all_ms": [round(t, 4) for t in res[f]]} for f in forms}
        out[key]["identical"] = all(torch.equal(outs[f], outs[forms[0]]) and torch.equal(vals[f], vals[forms[0]])
                                    for f in forms)
        print(key, json.dumps(out[key]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
