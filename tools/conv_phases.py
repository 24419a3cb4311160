#!/usr/bin/env python3
"""Where a conv3x3_stream_kernel wave's time goes (diagnostic build, -DZC_CONV_STAMP):
per wave s_memtime at start / tile staged / main loop done / end plus HW_ID and XCC_ID;
per SIMD, the fraction of its busy span in which at least one wave is in its MFMA loop.
Run with ZC_LIB pointing at the stamped library."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native  # noqa: E402

h, w, n, cin = 8, 8, 32768, 128
if len(sys.argv) > 1:
    h, w, n, cin = (int(v) for v in sys.argv[1:5])
L = _native.lib()
x = torch.randn(n, h, w, cin, device="cuda").half()
wt = (torch.randn(9, 128, cin, device="cuda") * 0.05).half()
wp = torch.empty_like(wt)
bias = torch.zeros(128, device="cuda")
o = torch.empty(n, h, w, 128, device="cuda", dtype=torch.float16)
_native.check(L.zc_net_conv3x3_pack_async(cin, wt.data_ptr(), wp.data_ptr(), None))
bph = 2 if h == 8 else 3
nwg = (n + bph - 1) // bph
for _ in range(3):
    _native.check(L.zc_net_conv3x3_packed_async(n, h, w, cin, x.data_ptr(), wp.data_ptr(), bias.data_ptr(), None,
                                                o.data_ptr(), 1, None))
torch.cuda.synchronize()
nw = nwg * 4
buf = np.zeros(nw * 6, dtype=np.uint64)
assert L.zc_debug_conv_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(nw * 6)) == 0
s = buf.reshape(nw, 6).astype(np.int64)
hw, xcc, t0, t1, t2, t3 = (s[:, i] for i in range(6))
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = (((xcc & 15) * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
out = {"shape": f"{n} boards {h}x{w} cin {cin}", "waves": int(nw),
       "prologue_cyc_mean": float((t1 - t0).mean()), "main_cyc_mean": float((t2 - t1).mean()),
       "epilogue_cyc_mean": float((t3 - t2).mean()), "lifetime_cyc_mean": float((t3 - t0).mean())}
fr, spans, conc = [], [], []
for k in np.unique(key):
    m = key == k
    a0, a1, a2, a3 = t0[m], t1[m], t2[m], t3[m]
    lo, hi = a0.min(), a3.max()
    ev = np.concatenate([np.stack([a1, np.ones_like(a1)], 1), np.stack([a2, -np.ones_like(a2)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    cur, last, covered = 0, lo, 0
    for t, d in ev:
        if cur > 0:
            covered += t - last
        cur += d
        last = t
    fr.append(covered / max(hi - lo, 1))
    spans.append(hi - lo)
    # waves resident at once (start..end), averaged over the span
    ev2 = np.concatenate([np.stack([a0, np.ones_like(a0)], 1), np.stack([a3, -np.ones_like(a3)], 1)])
    ev2 = ev2[np.lexsort((ev2[:, 1], ev2[:, 0]))]
    cur, last, acc = 0, lo, 0
    for t, d in ev2:
        acc += cur * (t - last)
        cur += d
        last = t
    conc.append(acc / max(hi - lo, 1))
out["simds"] = len(fr)
out["main_covered_frac_mean"] = float(np.mean(fr))
out["resident_waves_mean"] = float(np.mean(conc))
out["simd_span_cyc_mean"] = float(np.mean(spans))
out["waves_per_simd_mean"] = float(nw / len(fr))
print(json.dumps(out, indent=1))
