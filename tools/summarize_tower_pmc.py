#!/usr/bin/env python3
"""profiles/rNN_tower_pmc.json from tools/pmc_tower.sh's two counter passes over the fused
tower (tower_kernel, tools/one_tower.py: ValueNetwork(128, 8) on 8x8 x 32768 boards):
per-launch counters (summed over XCDs), rocprof durations, held clock and MFMA busy, as
tools/summarize_conv_pmc.py does for one layer.  Usage: summarize_tower_pmc.py gpurun_out OUT.json"""
import csv
import statistics
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd.nets import flops_per_position  # noqa: E402

N, H, W = 32768, 8, 8
# the MFMA work of the tower: the stem on its 32 padded planes and 16 conv3x3 128 -> 128 (the
# head is not in this kernel)
FLOPS = 2.0 * 9 * H * W * 128 * (32 + 16 * 128) * N
LAYER_FLOPS = 2.0 * N * H * W * 128 * 9 * 128  # one 128 -> 128 layer (tools/one_conv.py's shape)


def load(root, tag):
    """Per-dispatch counters and durations of one counter pass, the first (cold) launch
    dropped when the pass has more than one."""
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    with open(f"{root}/pmc_tower/{tag}_counter_collection.csv") as fh:
        for r in csv.DictReader(fh):
            if "tower_kernel" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = sorted(per, key=int)
    if len(ids) > 1:
        per.pop(ids[0])
        dur.pop(ids[0])
    return per, dur


def trace_ms(root):
    """Warm launch durations (the first dropped) of the kernel-trace-only pass, if present."""
    path = f"{root}/pmc_tower/t_kernel_trace.csv"
    if not os.path.exists(path):
        return None
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(path))
         if "tower_kernel" in r["Kernel_Name"]]
    return [x / 1e6 for x in d[1:]] if len(d) > 1 else [x / 1e6 for x in d]


def lib_sha():
    import hashlib
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zeroclone_amd", "libzeroclone_amd.so")
    with open(lib, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def main():
    root, out = sys.argv[1], sys.argv[2]
    c, durs = {}, []
    for tag in ("a", "b"):
        per, dur = load(root, tag)
        for d in per.values():
            for k, v in d.items():
                c.setdefault(k, []).append(v)
        durs += list(dur.values())
    cnt = {k: sum(v) / len(v) for k, v in c.items()}
    ms_pmc = sum(durs) / len(durs) / 1e6          # warm launches under counter collection
    clock = cnt["GRBM_GUI_ACTIVE"] / 8 / (ms_pmc * 1e-3) / 1e9
    busy = cnt["SQ_VALU_MFMA_BUSY_CYCLES"] / (cnt["GRBM_GUI_ACTIVE"] / 8 * 1024)
    tr = trace_ms(root)
    ms = statistics.median(tr) if tr else ms_pmc  # warm launches, kernel trace only
    tf = FLOPS / (ms * 1e-3) / 1e12
    res = {"shape": "fused tower (zc_net_tower_async): stem 32 -> 128 + 8 residual blocks (16 conv3x3 128 -> 128), "
                    "8x8 boards, 32768 boards (tools/one_tower.py)",
           "duration_source": ("median of the kernel-trace-only pass's warm launches (tools/pmc_tower.sh pass t)"
                               if tr else "mean of the counter passes' warm launches"),
           "trace_ms": [round(x, 4) for x in tr] if tr else None,
           "counter_pass_avg_ms": round(ms_pmc, 4),
           "kernel": f"tower_kernel<8, 8, 2, 32, 4, 2, 1, {os.environ.get('ZC_TOWER_MF', '16')}> "
                     f"({'16x16x32' if os.environ.get('ZC_TOWER_MF', '16') == '16' else '32x32x16'} MFMA form)",
           "lib_sha256": lib_sha(), "flops_per_launch": FLOPS, "rocprof_avg_ms": round(ms, 4),
           "counter_launches_used": len(durs), "tflops": round(tf, 1),
           "per_128ch_layer_equivalent_ms": round(ms * LAYER_FLOPS / FLOPS, 4),
           "clock_ghz_grbm": round(clock, 3), "mfma_busy_frac": round(busy, 3),
           "frac_of_2p5PF_nominal": round(tf / 2500, 3),
           "counters": {k: round(v) for k, v in sorted(cnt.items())},
           "note": ("GRBM_GUI_ACTIVE is summed over 8 XCDs: clock = GRBM_GUI_ACTIVE/8/duration; MFMA busy = "
                    "SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs).  Counter passes: tools/pmc_tower.sh.  "
                    "The layer-by-layer form of the same layer: profiles/r02_conv_pmc.json (1,030 TFLOP/s).")}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in ("rocprof_avg_ms", "tflops", "clock_ghz_grbm", "mfma_busy_frac")}))


if __name__ == "__main__":
    main()
