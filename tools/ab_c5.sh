#!/bin/bash
# Same-box A/B of the C5 step (tools/prof_c5.py, graph replays) between two libraries,
# alternating processes: tools/ab_c5.sh A.so B.so [rounds]
set -u
A=$1; B=$2; R=${3:-2}
for r in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    echo -n "$(basename "$L") round $r: "
    ZC_LIB="$L" timeout -k 10 240 python3 tools/prof_c5.py --mode ${MODE:-c5} --steps 3 --graph 2>&1 | grep "step:" || exit $?
  done
done
