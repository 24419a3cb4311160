#!/bin/bash
# Summarise a profile pass (tools/gpu_check.sh sprof shbm spmc wprof whbm wpmc, then
# tools/pmc_tower.sh) into profiles/<tag>_*.json, each stamped with the library's sha256:
#   bash tools/final_profiles.sh r04        (run here, after gpurun merged gpurun_out/)
set -e
cd "$(dirname "$0")/.."
tag=${1:?tag}
G=gpurun_out
grep '^{' $G/sprof.log | tail -1 > $G/sprof_run.json
grep '^{' $G/wprof.log | tail -1 > $G/wprof_run.json
python tools/summarize_profile.py --stats $G/sprof/run_kernel_stats.csv --trace $G/sprof/run_kernel_trace.csv \
  --fetch $G/shbm/fetch_counter_collection.csv --write $G/shbm/write_counter_collection.csv \
  --pmc $G/spmc/pmc_counter_collection.csv --moves 60 --extra-json $G/sprof_run.json \
  --note "bench workload: 4096 burned-in games x 800 sims x bs 32, one pooled launch of 60 x 4096 moves (tools/prof_search.py --steps 60); per-move figures" \
  --out profiles/${tag}_c4_search_summary.json
python tools/summarize_profile.py --kernel "c4_walk_kernel<2>" --last 3 --stats $G/wprof/run_kernel_stats.csv \
  --trace $G/wprof/run_kernel_trace.csv --fetch $G/whbm/fetch_counter_collection.csv \
  --write $G/whbm/write_counter_collection.csv --pmc $G/wpmc/pmc_counter_collection.csv \
  --extra-json $G/wprof_run.json \
  --note "walk-only replay kernel (tools/prof_walk.py): the lockstep search of 4096 burned-in games x 800 sims x bs 32 with the recorded rollout values in place of the rollouts; identical tree (checked)" \
  --out profiles/${tag}_walk_summary.json
if [ -d $G/pmc_tower ]; then
  python tools/summarize_tower_pmc.py $G profiles/${tag}_tower_pmc.json
fi
