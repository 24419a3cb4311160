#!/usr/bin/env python3
"""Where the fused tower's wave time goes (diagnostic build -DZC_TOWER_STAMP=1, libzc_tst.so):
per wave, s_memtime cycles of the layers' MFMA loops, their epilogues and the barrier waits,
against the whole kernel, summed over all waves of 5 launches (8x8 x 32768 and 6x7 x 131072).

    ZC_LIB=$PWD/zeroclone_amd/libzc_tst.so python tools/tower_stamps.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native  # noqa: E402
from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork  # noqa: E402


def main():
    f = _native.lib().zc_debug_tower_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(4, np.uint64)
    for (planes, h, w, n) in [(17, 8, 8, 32768), (2, 6, 7, 131072)]:
        torch.manual_seed(0)
        net = MfmaValueNetwork(ValueNetwork(128, 8, in_planes=planes).eval(), "cuda")
        x = (torch.rand(n, planes, h, w, device="cuda") < 0.3).half()
        for _ in range(3):
            net.tower(x)
        torch.cuda.synchronize()
        assert f(buf.ctypes.data, 1) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            net.tower(x)
        e1.record()
        torch.cuda.synchronize()
        assert f(buf.ctypes.data, 1) == 0
        mf, ep, ba, tot = (float(v) for v in buf)
        print(json.dumps({"shape": f"{h}x{w}x{n}", "mfma_loop": round(mf / tot, 4), "epilogue": round(ep / tot, 4),
                          "barrier_wait": round(ba / tot, 4), "rest": round(1 - (mf + ep + ba) / tot, 4),
                          "cycles_per_wave_launch": round(tot / 5 / (n * h * w / 128 * 4), 1),
                          "mfma_loop_cycles_per_wave_launch": round(mf / 5 / (n * h * w / 128 * 4), 1),
                          "ms": round(e0.elapsed_time(e1) / 5, 4), "lib": os.path.basename(_native.lib()._name)}), flush=True)


if __name__ == "__main__":
    main()
