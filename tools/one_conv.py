#!/usr/bin/env python3
"""One conv3x3 layer shape, launched a few times (for rocprofv3 counter passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native  # noqa: E402

h, w, n, cin = 8, 8, 32768, 128
if len(sys.argv) > 1:
    h, w, n, cin = (int(v) for v in sys.argv[1:5])
L = _native.lib()
x = torch.randn(n, h, w, cin, device="cuda").half()
wt = (torch.randn(9, 128, cin, device="cuda") * 0.05).half()
bias = torch.zeros(128, device="cuda")
o = torch.empty(n, h, w, 128, device="cuda", dtype=torch.float16)
packed = os.environ.get("ZC_AB_PACKED") == "1"  # the streamed-weight form (ZC_CONV_WPE picks 2 / 3)
if packed:
    wp = torch.empty_like(wt)
    _native.check(L.zc_net_conv3x3_pack_async(cin, wt.data_ptr(), wp.data_ptr(), None))
for _ in range(3):
    if packed:
        _native.check(L.zc_net_conv3x3_packed_async(n, h, w, cin, x.data_ptr(), wp.data_ptr(), bias.data_ptr(), None,
                                                    o.data_ptr(), 1, None))
    else:
        _native.check(L.zc_net_conv3x3_async(n, h, w, cin, x.data_ptr(), wt.data_ptr(), bias.data_ptr(), None,
                                             o.data_ptr(), 1, None))
torch.cuda.synchronize()
