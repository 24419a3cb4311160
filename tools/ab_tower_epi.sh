#!/bin/bash
# Same-box A/B of the fused tower's epilogue forms (ZC_TOWER_EPI, net_conv.hip tower_epi),
# alternating processes; tools/ab_tower.py also checks fused == layered bit for bit.
#   bash tools/ab_tower_epi.sh [forms...]   (default: 2 0)
set -e
forms=${*:-2 0}
for rnd in 1 2 3; do
  for epi in $forms; do
    echo "== round $rnd ZC_TOWER_EPI=$epi"
    ZC_TOWER_EPI=$epi AB_REPS=5 timeout -k 10 200 python tools/ab_tower.py | grep -v "^{"
  done
done
