#!/usr/bin/env python3
"""Chess search throughput (BASELINE configs C4: 1024 games x 400 sims, value-only network).

  crude : configs/crude_chess.yaml search (crude_chess_score in the kernel, immediate_value)
  net   : configs/chess_value.yaml search — ValueNetwork(128, 8) random init, fp16, between the
          select and backup kernels of every flush; one move captured in a HIP graph."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native  # noqa: E402
from zeroclone_amd.nets import ValueNetwork, flops_per_position, for_inference  # noqa: E402
from zeroclone_amd.valued import ChessValuedSearch, NetValue  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=1024)
    ap.add_argument("--sims", type=int, default=400)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--mode", default="crude,net")
    a = ap.parse_args()
    G, S, B = a.games, a.sims, a.bs
    eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B)
    eng.seed(0, list(range(G)))
    root = _native.chess_init()
    roots = torch.from_numpy(np.array([root] * G, _native.CHESS_STATE_DTYPE).view(np.uint8).reshape(G, 72).copy()).cuda()
    out = {}
    if "crude" in a.mode:
        mv = torch.zeros(G, dtype=torch.int16, device="cuda")
        na = torch.zeros((G, 256), dtype=torch.int32, device="cuda")
        st = torch.zeros((G, 8), dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        run = lambda: eng.chess_search_async(0, G, roots.data_ptr(), S, 1.4, B, 1, 3.0, mv.data_ptr(),  # noqa: E731
                                             na.data_ptr(), st.data_ptr(), s)
        run()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.steps
        exp = int(st[:, 0].sum())
        assert int(st[:, 5].abs().sum()) == 0
        out["crude"] = {"ms_per_move": round(dt * 1e3, 2), "exp_per_s": round(exp / dt), "expansions": exp,
                        "mean_depth": round(float(st[:, 1].sum()) / max(exp, 1), 3)}
    if "net" in a.mode:
        torch.manual_seed(0)
        model = for_inference(ValueNetwork(128, 8).eval(), "cuda", torch.float16)
        vs = ChessValuedSearch(eng, G, B, leaves=False)
        g = vs.capture(roots, S, 1.4, NetValue(model))
        g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.steps
        exp = int(vs.stats[:, 0].sum())
        x = torch.zeros(G * B, 17, 8, 8, dtype=torch.float16, device="cuda")
        with torch.no_grad():
            model(x)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                model(x)
            torch.cuda.synchronize()
            net_ms = (time.perf_counter() - t) / 3 * 1e3
        fl = flops_per_position(128, 8, 17, 8, 8) * G * B
        flushes = (S + B - 1) // B
        out["net"] = {"ms_per_move": round(dt * 1e3, 1), "exp_per_s": round(exp / dt), "expansions": exp,
                      "net_ms_per_flush": round(net_ms, 2), "net_tflops": round(fl / net_ms / 1e9, 1),
                      "net_share": round(net_ms * flushes / (dt * 1e3), 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
