set -e
for rnd in 1 2 3; do
  for epi in 2 0; do
    echo "== round $rnd ZC_TOWER_EPI=$epi"
    ZC_TOWER_EPI=$epi AB_REPS=5 timeout -k 10 200 python tools/ab_tower.py | grep -v "^{"
  done
done
