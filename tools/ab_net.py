#!/usr/bin/env python3
"""Whole-network A/B of conv variants: the value tower (ValueNetwork(128, 8), MFMA path) on
the chess C4 batch (32768 boards 8x8, 17 planes) and the Connect4 C2(iii) batch (131072
boards 6x7, 2 planes).  Each variant "lib[:wpe]" runs in its own process (ZC_LIB, ZC_CONV_WPE),
in turn over rounds; prints median ms per forward and whether the values are identical.

    python tools/ab_net.py lib_head.so:3 libzeroclone_amd.so:3 libzeroclone_amd.so:4"""
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CHILD = r'''
import sys, zlib, torch
sys.path.insert(0, %r)
from zeroclone_amd.nets import ValueNetwork, MfmaValueNetwork
out = []
for (planes, h, w, n) in [(17, 8, 8, 32768), (2, 6, 7, 131072)]:
    torch.manual_seed(0)
    net = MfmaValueNetwork(ValueNetwork(128, 8, in_planes=planes), "cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand(n, planes, h, w, device="cuda", generator=g) < 0.3).half()
    v = net(x); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5): v = net(x)
    b.record(); torch.cuda.synchronize()
    out.append("%%.3f" %% (a.elapsed_time(b) / 5))
    out.append(str(zlib.crc32(v.cpu().numpy().tobytes())))
print(" ".join(out))
'''


def main():
    variants = sys.argv[1:]
    res = {v: [] for v in variants}
    for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
        for v in variants:
            lib, _, wpe = v.partition(":")
            env = dict(os.environ, ZC_LIB=os.path.join(ROOT, "zeroclone_amd", lib), ZC_CONV_WPE=wpe or "3")
            o = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, check=True, capture_output=True,
                               text=True, timeout=300).stdout.strip().splitlines()[-1].split()
            res[v].append(o)
            print(rnd, v, o, flush=True)
    ref = res[variants[0]][0]
    for v in variants:
        chess = statistics.median(float(r[0]) for r in res[v])
        c4 = statistics.median(float(r[2]) for r in res[v])
        same = all(r[1] == ref[1] and r[3] == ref[3] for r in res[v])
        print(f"{v:28s} chess 8x8x32768 {chess:8.3f} ms   c4 6x7x131072 {c4:8.3f} ms   "
              f"{'values identical' if same else 'VALUES DIFFER'}")


if __name__ == "__main__":
    main()
