#!/bin/bash
# C5 step A/B: the select kernel writing NCHW planes + the separate planes_to_nhwc launch
# (ZC_PUCT_NHWC=0) against the NHWC planes written directly (the product); same library,
# alternating processes, graph replays (tools/prof_c5.py).
set -u
cd "$(dirname "$0")/.."
for r in 1 2 3; do
  for v in 0 1; do
    echo -n "nhwc=$v round $r: "
    ZC_PUCT_NHWC=$v ZC_PUCT_STREAMS=4 timeout -k 10 240 python3 tools/prof_c5.py --mode c5 --steps 3 --graph 2>&1 | grep "step:" || exit 1
  done
done
