#!/usr/bin/env python3
"""Practical MFMA ceiling on this box for the value tower's shapes: torch (hipBLASLt / MIOpen) on
(a) a large square fp16 GEMM, (b) the conv3x3's implicit GEMM as one explicit GEMM
([pixels x 1152] x [1152 x 128]) and (c) MIOpen's own conv2d (channels_last fp16), next to
this package's packed MFMA conv on the same layer.  TFLOP/s by HIP events, 20 reps."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native  # noqa: E402


def timed(f, flops, reps=20):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    return {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}


def main():
    out = {}
    x = torch.randn(8192, 8192, device="cuda").half()
    y = torch.randn(8192, 8192, device="cuda").half()
    out["gemm_8192^3"] = timed(lambda: torch.mm(x, y), 2.0 * 8192 ** 3)
    del x, y
    L = _native.lib()
    for (h, w, n) in [(8, 8, 32768), (6, 7, 131072)]:
        pix = n * h * w
        fl = 2.0 * pix * 128 * 1152
        A = torch.randn(pix, 1152, device="cuda").half()
        B = torch.randn(1152, 128, device="cuda").half()
        out[f"gemm_{pix}x1152x128"] = timed(lambda: torch.mm(A, B), fl)
        Bt = B.t().contiguous()
        out[f"gemm_{pix}x1152x128_bt"] = timed(lambda: torch.mm(A, Bt.t()), fl)
        del A, B, Bt
        xin = torch.randn(n, 128, h, w, device="cuda").half().to(memory_format=torch.channels_last)
        wc = (torch.randn(128, 128, 3, 3, device="cuda") * 0.05).half().to(memory_format=torch.channels_last)
        out[f"miopen_conv_{n}x{h}x{w}"] = timed(lambda: torch.nn.functional.conv2d(xin, wc, padding=1), fl)
        xn = torch.randn(n, h, w, 128, device="cuda").half()
        wt = (torch.randn(9, 128, 128, device="cuda") * 0.05).half()
        wp = torch.empty_like(wt)
        bias = torch.zeros(128, device="cuda")
        o = torch.empty_like(xn)
        _native.check(L.zc_net_conv3x3_pack_async(128, wt.data_ptr(), wp.data_ptr(), None))
        out[f"zc_packed_conv_{n}x{h}x{w}"] = timed(
            lambda: _native.check(L.zc_net_conv3x3_packed_async(n, h, w, 128, xn.data_ptr(), wp.data_ptr(),
                                                                bias.data_ptr(), None, o.data_ptr(), 1, None)), fl)
        del xin, wc, xn, wt, wp, o
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
