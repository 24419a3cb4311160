#!/bin/bash
# Runs ON THE GPU BOX after tools/gpu_check.sh's sprof/spmc/shbm stages: summarises the three
# rocprofv3 passes into profiles/$1 (what bench.py's roofline reads) and a copy under gpurun_out/.
set -e
cd "$(dirname "$0")/.."
python tools/summarize_profile.py --stats gpurun_out/sprof/run_kernel_stats.csv --trace gpurun_out/sprof/run_kernel_trace.csv \
  --fetch gpurun_out/shbm/fetch_counter_collection.csv --write gpurun_out/shbm/write_counter_collection.csv \
  --pmc gpurun_out/spmc/pmc_counter_collection.csv --last 1 --moves 60 --note "$2" --out "profiles/$1"
cp "profiles/$1" "gpurun_out/$1"
