#!/usr/bin/env python3
"""C2(iii) measurement: Connect4 self-play search with a random-init value network.

4096 games x 800 sims, batch 32: every flush evaluates 4096*32 leaves with the fp16
ValueNetwork (folded BN, channels-last) between the select and backup kernels; one move is
captured in a HIP graph and replayed.  Reports expansions/s and the network's TFLOP/s."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native
from zeroclone_amd.nets import ValueNetwork, flops_per_position, for_inference
from zeroclone_amd.valued import C4ValuedSearch, NetValue


def _nchw_forward(m, x):
    x = torch.relu(m.stem(x.contiguous()))
    x = m.res(x)
    return torch.tanh(m.fc(x.mean(dim=(2, 3))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--find", action="store_true", help="MIOpen exhaustive kernel search (cudnn.benchmark)")
    ap.add_argument("--nchw", action="store_true")
    ap.add_argument("--net-only", action="store_true")
    ap.add_argument("--mfma", action="store_true", help="this package's MFMA conv kernels instead of MIOpen")
    ap.add_argument("--planes", type=int, default=2)
    ap.add_argument("--hw", default="6x7")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.find
    torch.manual_seed(0)
    H, W = (int(v) for v in a.hw.split("x"))
    net = ValueNetwork(a.channels, a.blocks, in_planes=a.planes).eval()
    model = for_inference(net, "cuda", torch.float16, backend="mfma" if a.mfma else "torch")
    if a.nchw:
        model = model.to(memory_format=torch.contiguous_format)
        model.forward = lambda x, m=model: _nchw_forward(m, x)
    eng = _native.NativeEngine(max_games=a.games, max_sims=a.sims, max_batch=a.bs)
    eng.seed(0, list(range(a.games)))
    vs = C4ValuedSearch(eng, a.games, a.bs, leaves=False)
    value = NetValue(model) if not a.mfma else (lambda leaves, planes, counts: model(planes))
    roots = torch.zeros((a.games, 3), dtype=torch.int64, device="cuda")
    L = a.games * a.bs
    # network alone
    x = (torch.rand(L, a.planes, H, W, device="cuda") < 0.3).half()
    with torch.no_grad():
        for _ in range(2):
            model(x)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            model(x)
        torch.cuda.synchronize()
        net_ms = (time.perf_counter() - t) / 5 * 1e3
    fl = flops_per_position(a.channels, a.blocks, a.planes, H, W)
    out = {"net_ms_per_flush": round(net_ms, 3), "positions_per_flush": L,
           "net_tflops": round(fl * L / net_ms / 1e9, 1), "flops_per_position": fl}
    if a.net_only:
        print(json.dumps(out))
        return
    if a.no_graph:
        run = lambda: vs.enqueue(roots, a.sims, 1.4, value)
    else:
        g = vs.capture(roots, a.sims, 1.4, value)
        run = g.replay
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.steps):
        t = time.perf_counter()
        run()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    st = vs.stats.cpu()
    exp = int(st[:, 0].sum())
    ms = sorted(ts)[len(ts) // 2] * 1e3
    flushes = (a.sims + a.bs - 1) // a.bs
    out.update({"ms_per_move": round(ms, 1), "expansions": exp, "exp_per_s": round(exp / ms * 1e3),
                "net_share": round(net_ms * flushes / ms, 3), "graph": not a.no_graph})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
