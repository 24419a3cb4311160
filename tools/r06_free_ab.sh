#!/bin/bash
# Same-box A/B of library variants on the lockstep schedule (the free run: every game exactly
# K moves per launch, tools/prof_search.py --launch free), alternating processes.
set -u
cd "$(dirname "$0")/.."
for rnd in 1 2 3; do
  for l in ${LIBS:-lib_nolag.so libzeroclone_amd.so}; do
    echo "== round $rnd $l"
    ZC_LIB=$PWD/zeroclone_amd/$l timeout -k 10 200 python tools/prof_search.py --launch free --steps ${AB_STEPS:-20} 2>&1 | grep "G expansions" || exit 1
  done
done
