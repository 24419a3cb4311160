#!/usr/bin/env python3
"""profiles/<tag>_chess_crude_pmc.json from tools/gpu_check.sh's cprof / cpmc stages (the chess
crude search, tools/bench_chess.py --mode crude: 1024 games x 400 sims x bs 32 from the
opening, one move per launch): rocprof stats, per-wave counters per move (warm launches),
issue utilisation, stamped with the library's sha256.

    python tools/summarize_chess_pmc.py gpurun_out profiles/r04_chess_crude_pmc.json"""
import collections
import csv
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    root, out_path = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(f"{root}/cpmc/pmc_counter_collection.csv")):
        if "chess_search_kernel" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = sorted(per, key=int)[1:]   # warm launches
    c = {k: sum(per[i][k] for i in ids) / len(ids) for k in per[ids[0]]}
    ms = sum(dur[i] for i in ids) / len(ids) / 1e6
    w, C = c["SQ_WAVES"], c["GRBM_GUI_ACTIVE"] / 8
    stats = [r for r in csv.DictReader(open(f"{root}/cprof/run_kernel_stats.csv")) if "chess_search_kernel" in r["Name"]][0]
    sims = 400
    lib = os.path.join(HERE, "..", "zeroclone_amd", "libzeroclone_amd.so")
    out = {"kernel": "chess_search_kernel (crude_chess_score in the kernel, immediate_value(3))",
           "workload": "tools/bench_chess.py --mode crude: 1024 games x 400 sims x bs 32 from the opening, one move per launch",
           "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
           "rocprof_stats": {"calls": int(stats["Calls"]), "avg_ms": float(stats["AverageNs"]) / 1e6,
                             "min_ms": float(stats["MinNs"]) / 1e6},
           "counter_pass_warm_ms": round(ms, 4), "clock_ghz": round(C / (ms * 1e-3) / 1e9, 3),
           "per_wave_per_move": {"SQ_INSTS_VALU": round(c["SQ_INSTS_VALU"] / w), "SQ_INSTS_SALU": round(c["SQ_INSTS_SALU"] / w),
                                 "SQ_INSTS_LDS": round(c["SQ_INSTS_LDS"] / w), "wave_cycles": round(c["SQ_WAVE_CYCLES"] / w * 4)},
           "waves_per_game": round(w / 1024, 3),
           "per_simulation": {"instructions_all_waves": round((c["SQ_INSTS_VALU"] + c["SQ_INSTS_SALU"] + c["SQ_INSTS_LDS"])
                                                              / 1024 / sims),
                              "wave_cycles_per_wave": round(c["SQ_WAVE_CYCLES"] / w * 4 / sims),
                              "wall_cycles": round(C / sims)},
           "issue": {"valu_util": round(2 * c["SQ_INSTS_VALU"] / (1024 * C), 3), "salu_util": round(c["SQ_INSTS_SALU"] / (256 * C), 3),
                     "issue_any": round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
                     "wait_any": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)},
           "note": ("1024 games on 1024 SIMDs: round 5 runs each game as a workgroup of two waves (leader + helper, "
                    "chess_search.hip Helper), so SQ_WAVES = 2048 and the per-wave figures average the two roles; "
                    "per simulation: all instructions of a game's waves, a wave's own cycles, and the launch's wall "
                    "cycles per simulation. SQ_WAVE_CYCLES counts quad-cycles (x4). Counter pass: tools/gpu_check.sh "
                    "cpmc; stats: cprof.")}
    with open(out_path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out)[:600])


if __name__ == "__main__":
    main()
