#!/usr/bin/env python3
"""The fused value tower (zc_net_tower_async, ValueNetwork(128, 8) random init) launched a few
times on one shape, for rocprofv3 counter passes: 8x8 x 32768 boards (default) or
`6 7 131072`; an optional fourth argument sets the number of launches (default 3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork  # noqa: E402

h, w, n = 8, 8, 32768
if len(sys.argv) > 1:
    h, w, n = (int(v) for v in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
planes = 17 if (h, w) == (8, 8) else 2
torch.manual_seed(0)
net = MfmaValueNetwork(ValueNetwork(128, 8, in_planes=planes), "cuda")
x = (torch.rand(n, planes, h, w, device="cuda") < 0.3).half()
for _ in range(reps):
    net.tower(x)
torch.cuda.synchronize()
