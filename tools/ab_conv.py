#!/usr/bin/env python3
"""A/B of the conv3x3 implementations (ZC_CONV_IMPL = tile / half; stream2 / stream3 = the packed-weight
form at 2 / 3 waves per SIMD; argv picks them):
bit-identical outputs and per-layer time.  Runs each impl in a child process."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.path.join(sys.argv[1], ".."))
from zeroclone_amd import _native
L = _native.lib()
out = {}
g = torch.Generator(device="cuda").manual_seed(0)
for (h, w, n) in [(8, 8, 32768), (6, 7, 131072), (8, 8, 1000), (6, 7, 777)]:
    for cin in (128, 32):
        x = torch.randn(n, h, w, cin, device="cuda", generator=g).half()
        wt = (torch.randn(9, 128, cin, device="cuda", generator=g) * 0.05).half()
        bias = torch.randn(128, device="cuda", generator=g) * 0.1
        res = torch.randn(n, h, w, 128, device="cuda", generator=g).half()
        o = torch.empty(n, h, w, 128, device="cuda", dtype=torch.float16)
        fl = 2.0 * n * h * w * 128 * 9 * cin
        packed = os.environ.get("ZC_AB_PACKED") == "1"
        if packed:
            wp = torch.empty_like(wt)
            _native.check(L.zc_net_conv3x3_pack_async(cin, wt.data_ptr(), wp.data_ptr(), None))
        for use_res in (False, True):
            if packed:
                f = lambda: _native.check(L.zc_net_conv3x3_packed_async(n, h, w, cin, x.data_ptr(), wp.data_ptr(), bias.data_ptr(),
                                                                        res.data_ptr() if use_res else None, o.data_ptr(), 1, None))
            else:
                f = lambda: _native.check(L.zc_net_conv3x3_async(n, h, w, cin, x.data_ptr(), wt.data_ptr(), bias.data_ptr(),
                                                                 res.data_ptr() if use_res else None, o.data_ptr(), 1, None))
            f(); torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10): f()
            b.record(); torch.cuda.synchronize()
            ms = a.elapsed_time(b) / 10
            key = f"{h}x{w} n{n} cin{cin} res{int(use_res)}"
            out[key] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1), "sum": float(o.float().sum().item()),
                        "hash": int((o.view(torch.int16).to(torch.int64) * torch.arange(o.numel(), device="cuda").view(o.shape) % 1000003).sum().item())}
print(json.dumps(out))
'''
IMPLS = sys.argv[1:] or ["tile", "half"]
res = {}
for impl in IMPLS:
    if impl.startswith("stream"):  # packed weights: stream2 / stream3 = waves per SIMD
        env = dict(os.environ, ZC_AB_PACKED="1", ZC_CONV_WPE=impl[-1])
    else:
        env = dict(os.environ, ZC_CONV_IMPL=impl)
    r = subprocess.run([sys.executable, "-c", CHILD, HERE], env=env, capture_output=True, text=True, timeout=600)
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(r.returncode)
    res[impl] = json.loads(r.stdout.strip().splitlines()[-1])
base = IMPLS[0]
same = {i: all(res[i][k]["hash"] == res[base][k]["hash"] for k in res[base]) for i in IMPLS}
for k in res[base]:
    print(f"{k:30s}" + " | ".join(f"{i} {res[i][k]['ms']:7.4f} ms {res[i][k]['tflops']:6.1f} TF" for i in IMPLS))
print("bit-identical:", same)
