#!/usr/bin/env python3
"""Summarise rocprofv3 outputs under gpurun_out/ into a small JSON for profiles/.

  --stats   gpurun_out/prof/run_kernel_stats.csv     (rocprofv3 --kernel-trace --stats)
  --fetch   gpurun_out/hbm/fetch_counter_collection.csv  (--pmc FETCH_SIZE, own pass)
  --write   gpurun_out/hbm/write_counter_collection.csv  (--pmc WRITE_SIZE, own pass)
  --pmc     gpurun_out/pmc/pmc_counter_collection.csv    (SQ counters, own pass)

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB;
gfx950's FETCH_SIZE under-reports a wide streaming read by exactly 2x, so the read side is
doubled (an upper bound for this kernel's narrower gathers); WRITE_SIZE is taken as is.
"""
import argparse
import collections
import csv
import json

KERNEL = "c4_search_kernel<false, false>"  # the product kernel (not the stamped diagnostic build)


def per_launch(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(vals) / len(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--pmc")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out = {"kernel": KERNEL}
    if a.stats:
        for r in csv.DictReader(open(a.stats)):
            if KERNEL in r["Name"]:
                out["rocprof_stats"] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                        "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                                        "percent_of_gpu_time": float(r["Percentage"])}
    if a.fetch and a.write:
        f = per_launch(a.fetch, "FETCH_SIZE")
        w = per_launch(a.write, "WRITE_SIZE")
        out["hbm"] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
                      "bytes_per_launch": (2 * f + w) * 1024.0,
                      "bytes_per_launch_uncorrected": (f + w) * 1024.0,
                      "correction": "read side x2 (gfx950 FETCH_SIZE half-count), KiB -> B"}
    if a.pmc:
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(a.pmc)):
            if KERNEL in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n = agg.get("SQ_WAVES", 0) or 1
        out["sq_per_wave"] = {k: v / n for k, v in sorted(agg.items()) if k != "SQ_WAVES"}
        out["sq_waves"] = agg.get("SQ_WAVES")
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
