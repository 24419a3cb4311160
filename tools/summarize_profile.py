#!/usr/bin/env python3
"""Summarise rocprofv3 outputs under gpurun_out/ into a small JSON for profiles/.

  --stats   gpurun_out/prof/run_kernel_stats.csv     (rocprofv3 --kernel-trace --stats)
  --trace   gpurun_out/prof/run_kernel_trace.csv     (same pass: per-launch durations)
  --fetch   gpurun_out/hbm/fetch_counter_collection.csv  (--pmc FETCH_SIZE, own pass)
  --write   gpurun_out/hbm/write_counter_collection.csv  (--pmc WRITE_SIZE, own pass)
  --pmc     gpurun_out/pmc/pmc_counter_collection.csv    (SQ counters + GRBM_GUI_ACTIVE, own pass)

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB;
gfx950's FETCH_SIZE under-reports a wide streaming read by exactly 2x, so the read side is
doubled (an upper bound for this kernel's narrower gathers); WRITE_SIZE is taken as is.

Issue roofline (the search kernel is a per-game serial chain, not an HBM stream): a SIMD
issues a wave64 VALU instruction over 2 cycles (32 lanes per cycle, MI355X_MICROARCH.md
"A wave (64 lanes) ... issues each VALU instruction over 2 cycles"; one wave alone sustains
one per 4) and the CU's one scalar unit one SALU instruction per cycle.  With
the dispatch's cycles C = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs),
  valu_util = 2 * sum(SQ_INSTS_VALU) / (1024 SIMDs * C)
  salu_util = sum(SQ_INSTS_SALU) / (256 CUs * C)
  issue_any = sum(SQ_ACTIVE_INST_ANY) / sum(SQ_WAVE_CYCLES)   (share of a wave's cycles issuing)
and the binding unit is the busier of VALU and SALU.  Only the last --last launches of the
kernel are used (the driver's burn-in steps come first).
"""
import argparse
import collections
import csv
import hashlib
import json
import os

KERNEL = "c4_selfplay_kernel<false>"  # the product kernel (K self-play moves per launch)
N_CU, N_SIMD, N_XCD = 256, 1024, 8


def rows_of(path, kernel):
    return [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]


def per_dispatch(path, kernel, last):
    """{dispatch id: {counter: value summed over the dispatch's rows}} of the last `last` launches."""
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows_of(path, kernel):
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(d)[-last:] if last else sorted(d)
    return [d[i] for i in ids]


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--pmc")
    ap.add_argument("--kernel", default=KERNEL)
    ap.add_argument("--last", type=int, default=1, help="launches to average (0 = all)")
    ap.add_argument("--moves", type=int, default=1, help="moves per launch: bytes and times are reported per move")
    ap.add_argument("--note", default="")
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zeroclone_amd",
                                                  "libzeroclone_amd.so"),
                    help="the library the profiled run loaded: its sha256 stamps the summary (bench.py marks "
                         "the summary stale when the loaded library differs)")
    ap.add_argument("--extra-json", default=None, help="a JSON line (e.g. tools/prof_walk.py's output) to embed")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out = {"kernel": a.kernel, "launches_used": a.last or "all", "moves_per_launch": a.moves}
    if a.lib and os.path.exists(a.lib):
        out["lib_sha256"] = hashlib.sha256(open(a.lib, "rb").read()).hexdigest()
        out["lib_mtime"] = os.path.getmtime(a.lib)
    if a.extra_json:
        with open(a.extra_json) as fh:
            lines = [ln for ln in fh.read().splitlines() if ln.startswith("{")]
        out["run"] = json.loads(lines[-1])
        if out["run"].get("lib_sha256"):   # the GPU run's own stamp wins over the local file's
            out["lib_sha256"] = out["run"]["lib_sha256"]
    if a.note:
        out["note"] = a.note
    if a.stats:
        for r in csv.DictReader(open(a.stats)):
            if a.kernel in r["Name"]:
                out["rocprof_stats"] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                        "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                                        "percent_of_gpu_time": float(r["Percentage"])}
    if a.trace:
        durs = [(int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
        durs = [d for _, d in sorted(durs)]
        sel = durs[-a.last:] if a.last else durs
        out["trace_last_avg_ns"] = mean(sel)
        out["trace_last_avg_ns_per_move"] = mean(sel) / a.moves
    if a.fetch and a.write:
        f = mean([d["FETCH_SIZE"] for d in per_dispatch(a.fetch, a.kernel, a.last)])
        w = mean([d["WRITE_SIZE"] for d in per_dispatch(a.write, a.kernel, a.last)])
        f, w = f / a.moves, w / a.moves
        out["hbm"] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
                      "bytes_per_launch": (2 * f + w) * 1024.0,
                      "bytes_per_launch_uncorrected": (f + w) * 1024.0,
                      "per": "move",
                      "correction": "read side x2 (gfx950 FETCH_SIZE half-count), KiB -> B"}
    if a.pmc:
        ds = per_dispatch(a.pmc, a.kernel, a.last)
        agg = {k: mean([d[k] for d in ds]) for k in ds[0]} if ds else {}
        n = agg.get("SQ_WAVES", 0) or 1
        out["sq_per_wave"] = {k: v / n for k, v in sorted(agg.items()) if k.startswith("SQ_") and k != "SQ_WAVES"}
        out["sq_waves"] = agg.get("SQ_WAVES")
        if "GRBM_GUI_ACTIVE" in agg:
            cyc = agg["GRBM_GUI_ACTIVE"] / N_XCD
            iss = {"cycles_per_launch": cyc}
            if "SQ_INSTS_VALU" in agg:
                iss["valu_util"] = 2.0 * agg["SQ_INSTS_VALU"] / (N_SIMD * cyc)
            if "SQ_INSTS_SALU" in agg:
                iss["salu_util"] = agg["SQ_INSTS_SALU"] / (N_CU * cyc)
            if "SQ_INSTS_LDS" in agg:
                iss["lds_instr_per_simd_cycle"] = agg["SQ_INSTS_LDS"] / (N_SIMD * cyc)
            if "SQ_ACTIVE_INST_ANY" in agg and agg.get("SQ_WAVE_CYCLES"):
                iss["issue_any"] = agg["SQ_ACTIVE_INST_ANY"] / agg["SQ_WAVE_CYCLES"]
            if "SQ_WAIT_ANY" in agg and agg.get("SQ_WAVE_CYCLES"):
                iss["wait_any"] = agg["SQ_WAIT_ANY"] / agg["SQ_WAVE_CYCLES"]
            units = {k: iss[k] for k in ("valu_util", "salu_util") if k in iss}
            if units:
                b = max(units, key=units.get)
                iss["bound_unit"] = b.split("_")[0]
                iss["frac"] = units[b]
            if out.get("trace_last_avg_ns"):   # the same launch(es), timed in the --stats pass
                iss["clock_ghz"] = cyc / out["trace_last_avg_ns"]
            out["issue"] = iss
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
