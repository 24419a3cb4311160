#!/usr/bin/env python3
"""Per-layer timing of the MFMA conv3x3 kernel (net_conv.hip) vs MIOpen on the same shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    L = _native.lib()
    out = {}
    for (h, w, n) in [(8, 8, 32768), (6, 7, 131072)]:
        for cin in (128, 32):
            x = torch.randn(n, h, w, cin, device="cuda").half()
            wt = (torch.randn(9, 128, cin, device="cuda") * 0.05).half()
            bias = torch.zeros(128, device="cuda")
            res = torch.randn(n, h, w, 128, device="cuda").half()
            o = torch.empty(n, h, w, 128, device="cuda", dtype=torch.float16)
            fl = 2.0 * n * h * w * 128 * 9 * cin
            for use_res in (False, True):
                ms = timeit(lambda: _native.check(L.zc_net_conv3x3_async(
                    n, h, w, cin, x.data_ptr(), wt.data_ptr(), bias.data_ptr(),
                    res.data_ptr() if use_res else None, o.data_ptr(), 1, None)))
                out[f"{h}x{w} cin{cin} res{int(use_res)}"] = {"ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1)}
            xn = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            wn = wt.reshape(3, 3, 128, cin).permute(2, 3, 0, 1).contiguous(memory_format=torch.channels_last)
            ms = timeit(lambda: torch.nn.functional.conv2d(xn, wn, padding=1))
            out[f"{h}x{w} cin{cin} miopen"] = {"ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
