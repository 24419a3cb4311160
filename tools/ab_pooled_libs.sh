#!/bin/bash
# Same-box A/B of library variants on the pooled headline launch (tools/prof_search.py:
# 4096 burned-in games, one launch of K x 4096 moves), alternating processes:
#   bash tools/ab_pooled_libs.sh libA.so libB.so ...   (paths relative to zeroclone_amd/)
set -e
for rnd in 1 2 3; do
  for l in "$@"; do
    echo "== round $rnd $l"
    ZC_LIB=$PWD/zeroclone_amd/$l timeout -k 10 200 python tools/prof_search.py --steps ${AB_STEPS:-20} 2>&1 | grep "G expansions"
  done
done
