#!/bin/bash
# A/B of tower variants (ZC_LIB copies of the library), same box, alternating processes:
#   bash tools/ab_tower_libs.sh libzeroclone_amd.so libzc_variant.so ...
set -e
mkdir -p gpurun_out
for rnd in 1 2 3; do
  for l in "$@"; do
    echo "== round $rnd $l" >> gpurun_out/abt.log
    ZC_LIB=$PWD/zeroclone_amd/$l AB_REPS=5 timeout -k 10 300 python tools/ab_tower.py >> gpurun_out/abt.log 2>&1
  done
done
