#!/usr/bin/env python3
"""Where the pooled launch's fixed cost goes: the bench's workload
(4096 burned-in games x 800 sims x bs 32), pooled launches of K x 4096 moves with the
launch-timeline stamps on (zc_debug_c4_launch_stamps: per wave s_memrealtime at its start, at
its last move's start and at its end, 100 MHz).  Per launch: the event time, the span of the
stamps, and the wave-time lost at the two ends — the ramp (start_w - first start) and the tail
(last end - end_w) — as mean per-wave milliseconds, i.e. the launch time the chip spends only
partly busy; plus the tail's shape (how long after the budget ran out the last waves ended)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd import _native  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=str, default="20,60")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--carry", type=int, default=1, help="carry launches (warmup launch carries moves in)")
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream(torch.device("cuda", 0)))
    G = 4096
    sp = C4SelfPlay(G, 800, c=1.4, batch_size=32, seed=0, device=0, record=True)
    burn = bench.burn_in(sp)
    buf = torch.zeros((G, 4), dtype=torch.int64, device="cuda")
    _native.check(_native.lib().zc_debug_c4_launch_stamps(sp.eng._h, buf.data_ptr()))
    out = {"burn_in_steps": burn, "clock": "s_memrealtime, 100 MHz", "launches": []}
    for k in [int(x) for x in a.steps.split(",")] * a.reps:
        if a.carry:   # the timed launch's stamps, before the drain's launch overwrites them
            sp.run_pooled(a.warmup * G, 2 * a.warmup, carry=True)
            torch.cuda.synchronize()
            buf.zero_()
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            sp.run_pooled(k * G, 2 * k, kernel_done=ev[1], carry=True)
            torch.cuda.synchronize()
            r = {"launch_ms": ev[0].elapsed_time(ev[1]), "expansions": int(sp.stats[:, 0].sum())}
            ts = buf.cpu().numpy().astype(np.float64) / 1e5   # ms
            sp.drain()
        else:
            buf.zero_()
            r = bench.run_steps(sp, k, warmup=a.warmup, launch="pooled", carry=False)
            ts = buf.cpu().numpy().astype(np.float64) / 1e5   # ms
        start, last, end = ts[:, 0], ts[:, 1], ts[:, 2]
        moves = (buf[:, 3].cpu().numpy() & 0xFFFFFFFF).astype(np.float64)  # (high word: where the wave ran)
        t0, t1 = start.min(), end.max()
        budget_out = last.max()   # the last ticket was taken then (a wave's last move started)
        rec = {"steps": k, "carry": a.carry, "launch_ms": round(r["launch_ms"], 3), "per_step_ms": round(r["launch_ms"] / k, 4),
               "stamp_span_ms": round(t1 - t0, 3),
               "ramp_ms_mean": round(float((start - t0).mean()), 4),
               "tail_ms_mean": round(float((t1 - end).mean()), 4),
               "first_wave_end_ms": round(float(end.min() - t0), 3),
               "last_ticket_ms": round(float(budget_out - t0), 3),
               "after_last_ticket_ms": round(float(t1 - budget_out), 3),
               "end_p10_p50_p90_ms": [round(float(np.percentile(end - t0, q)), 3) for q in (10, 50, 90)],
               "last_move_ms_p50_p90_max": [round(float(np.percentile(end - last, q)), 3) for q in (50, 90, 100)],
               "moves_min_mean_max": [int(moves.min()), round(float(moves.mean()), 2), int(moves.max())],
               "expansions": r["expansions"]}
        rec["lost_ms"] = round(rec["ramp_ms_mean"] + rec["tail_ms_mean"], 4)
        rec["lost_frac"] = round(rec["lost_ms"] / max(rec["stamp_span_ms"], 1e-9), 4)
        out["launches"].append(rec)
        print(json.dumps(rec), flush=True)
    _native.check(_native.lib().zc_debug_c4_launch_stamps(sp.eng._h, None))
    out["lib_sha256"] = bench.lib_sha()
    print(json.dumps(out), flush=True)
    sp.close()


if __name__ == "__main__":
    main()
