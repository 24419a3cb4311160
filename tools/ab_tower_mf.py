#!/usr/bin/env python3
"""The fused tower's two MFMA forms, alternating in one process (ZC_TOWER_MF is read per
launch): the 32x32x16 form (default) and the 16x16x32 form, on the chess C4 batch (32768
boards 8x8, 17 planes) and the Connect4 C2(iii) batch (131072 boards 6x7, 2 planes).  Prints
ms per tower, TFLOP/s, and each form's error against a torch fp32 reference of the same folded
network on the same fp16 input (max abs over the output activation), plus max |MF16 - MF32|."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd.nets import FoldedValueNetwork, MfmaValueNetwork, ValueNetwork, flops_per_position  # noqa: E402
from zeroclone_amd import _native  # noqa: E402


def main():
    reps = int(os.environ.get("AB_REPS", "5"))
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    out = {}
    for (planes, h, w, n) in [(17, 8, 8, 32768), (2, 6, 7, 131072)]:
        torch.manual_seed(0)
        vnet = ValueNetwork(128, 8, in_planes=planes).eval()
        for m in vnet.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.1, 0.1)
                m.running_var.uniform_(0.5, 1.5)
        net = MfmaValueNetwork(vnet, "cuda")
        g = torch.Generator(device="cuda").manual_seed(1)
        x = (torch.rand(n, planes, h, w, device="cuda", generator=g) < 0.3).half()
        res = {"32": [], "16": [], "16e": []}
        outs = {}
        for _ in range(rounds):
            for mf in ("32", "16", "16e"):
                _native.net_switch("tower_mf", int(mf[:2]))
                _native.net_switch("tower_epi", 1 if mf.endswith("e") else 0)
                a, _ = net.tower(x)
                torch.cuda.synchronize()
                outs[mf] = a.clone()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    net.tower(x)
                e1.record()
                torch.cuda.synchronize()
                res[mf].append(e0.elapsed_time(e1) / reps)
        same = {}
        for mf in ("32", "16"):
            _native.net_switch("tower_mf", int(mf))
            layered, _ = net.tower(x, fused=False)
            torch.cuda.synchronize()
            same[mf] = bool(torch.equal(outs[mf], layered))
        _native.net_switch("tower_mf", 0)
        _native.net_switch("tower_epi", 0)
        # torch fp32 reference on 2048 boards (the folded network, NHWC-compared)
        k = 2048
        f = FoldedValueNetwork(vnet).float().cuda()
        with torch.no_grad():
            t = f.res(torch.relu(f.stem(x[:k].float())))      # [k, 128, h, w]
        ref = t.permute(0, 2, 3, 1).reshape(k, h * w, 128)
        flop = flops_per_position(128, 8, 32, h, w) * n
        key = f"{h}x{w}x{n}"
        out[key] = {
            "mf32_ms": statistics.median(res["32"]), "mf16_ms": statistics.median(res["16"]),
            "mf32_tflops": round(flop / statistics.median(res["32"]) / 1e9, 1),
            "mf16_tflops": round(flop / statistics.median(res["16"]) / 1e9, 1),
            "mf16e_ms": statistics.median(res["16e"]),
            "mf16e_tflops": round(flop / statistics.median(res["16e"]) / 1e9, 1),
            "mf16e_equals_mf16": bool(torch.equal(outs["16e"], outs["16"])),
            "all_ms": res,
            "fused_equals_layered": same,
            "max_abs_mf16_vs_mf32": float((outs["16"].float() - outs["32"].float()).abs().max()),
            "max_abs_mf32_vs_fp32": float((outs["32"][:k].float() - ref).abs().max()),
            "max_abs_mf16_vs_fp32": float((outs["16"][:k].float() - ref).abs().max()),
            "ref_max_abs": float(ref.abs().max()),
        }
        print(key, json.dumps(out[key]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
