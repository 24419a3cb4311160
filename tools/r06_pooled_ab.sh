#!/bin/bash
# Same-box A/B of library variants on the pooled headline launch (K x 4096 moves after burn-in,
# tools/prof_search.py), alternating processes, then the driver's bench command on the product
# library (no CPU baseline, no network modes).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rnd in 1 2 3; do
  for l in ${LIBS:-lib_base.so libzeroclone_amd.so}; do
    echo "== round $rnd $l"
    ZC_LIB=$PWD/zeroclone_amd/$l timeout -k 10 200 python tools/prof_search.py --steps ${AB_STEPS:-20} 2>&1 | grep "G expansions" || exit 1
  done
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --net-steps 0 > gpurun_out/bench_quick.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_quick.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value']/1e9, d['ms_per_step'], d['extra']['reference_schedule']['value']/1e9, d['roofline']['frac'])"
