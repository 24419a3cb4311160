#!/bin/bash
# Pace balancing A/B: the free run (prof_search --launch free) and the bench's own lockstep
# line (reference_schedule, after the pooled window) per library, alternating processes.
set -u
cd "$(dirname "$0")/.."
for rnd in 1 2; do
  for l in ${LIBS}; do
    ZC_LIB=$PWD/zeroclone_amd/$l timeout -k 10 200 python tools/prof_search.py --launch free --steps 20 2>&1 | grep "G expansions" | sed "s/^/$l free: /" || exit 1
    ZC_LIB=$PWD/zeroclone_amd/$l timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --net-steps 0 > gpurun_out/bench_lag.log 2>&1 || exit 1
    grep '^{' gpurun_out/bench_lag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l bench', round(d['value']/1e9,4), 'lockstep', round(d['extra']['reference_schedule']['value']/1e9,4))"
  done
done
