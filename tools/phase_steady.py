#!/usr/bin/env python3
"""Phase cycles (s_memtime stamps, ZC stamp build) of the search kernel in steady-state
self-play: burn-in as bench.py, then a few stamped moves; prints per-launch wall cycles of
every stamp slot summed over games / games (i.e. per game), and counters per bulk."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay  # noqa: E402

torch.cuda.set_device(0)
sp = C4SelfPlay(4096, 800, c=1.4, batch_size=32, seed=0, device=0, record=True)
bench.burn_in(sp)
tot = None
K = 4
for _ in range(K):
    sp.eng.phase_cycles(True)
    sp.step()
    torch.cuda.synchronize()
    ph = sp.eng.phase_cycles(False)
    tot = ph if tot is None else {k: tot[k] + ph[k] for k in ph}
G = 4096
print({k: round(v / K / G) for k, v in tot.items()}, flush=True)
print("sum", round(sum(tot.values()) / K / G))
sp.close()
