#!/usr/bin/env python3
"""profiles/rNN_conv_pmc.json from tools/pmc_conv.sh's two counter passes per form (half /
stream): per-launch counters (summed over XCDs), rocprof durations, held clock and MFMA busy.
Usage: summarize_conv_pmc.py gpurun_out OUT.json"""
import csv
import json
import sys
from collections import defaultdict

FORMS = {"half": ("conv3x3_half_kernel", "staged half form (zc_net_conv3x3_async)"),
         "stream": ("conv3x3_stream_kernel", "packed streamed-weight form (zc_net_conv3x3_packed_async, 3 waves/SIMD)")}
FLOPS = 2.0 * 32768 * 64 * 128 * 9 * 128  # tools/one_conv.py: 8x8 boards, 32768 boards, 128 -> 128


def load(root, form, tag, key):
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    with open(f"{root}/pmc_{form}/{tag}_counter_collection.csv") as fh:
        for r in csv.DictReader(fh):
            if key in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, dur


def main():
    root, out = sys.argv[1], sys.argv[2]
    res = {"shape": "conv3x3 8x8 boards, 32768 boards, cin 128 -> 128, no residual, ReLU (tools/one_conv.py)",
           "flops_per_launch": FLOPS}
    for form, (key, desc) in FORMS.items():
        c, durs = {}, []
        for tag in ("a", "b"):
            per, dur = load(root, form, tag, key)
            for d in per.values():
                for k, v in d.items():
                    c.setdefault(k, []).append(v)
            durs += list(dur.values())
        cnt = {k: sum(v) / len(v) for k, v in c.items()}
        ms = sum(durs) / len(durs) / 1e6
        clock = cnt["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9
        busy = cnt["SQ_VALU_MFMA_BUSY_CYCLES"] / (cnt["GRBM_GUI_ACTIVE"] / 8 * 1024)
        res[form] = {"kernel": desc, "rocprof_avg_ms": round(ms, 4), "calls": len(durs),
                     "tflops": round(FLOPS / (ms * 1e-3) / 1e12, 1), "clock_ghz_grbm": round(clock, 3),
                     "mfma_busy_frac": round(busy, 3),
                     "frac_of_2p5PF_nominal": round(FLOPS / (ms * 1e-3) / 2.5e15, 3),
                     "counters": {k: round(v) for k, v in sorted(cnt.items())}}
    res["note"] = ("GRBM_GUI_ACTIVE is summed over 8 XCDs: clock = GRBM_GUI_ACTIVE/8/duration; MFMA busy = "
                   "SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs) (32 busy cycles per "
                   "v_mfma_f32_32x32x16_f16).  Counter passes: tools/pmc_conv.sh.  Practical ceiling on these "
                   "boxes: profiles/r02_gemm_ceiling.json (hipBLASLt fp16 8192^3: 1161 TFLOP/s).")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({f: {k: res[f][k] for k in ("rocprof_avg_ms", "tflops", "clock_ghz_grbm", "mfma_busy_frac")}
                      for f in FORMS}))


if __name__ == "__main__":
    main()
