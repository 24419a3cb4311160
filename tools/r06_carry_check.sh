#!/bin/bash
# Carried pooled moves: the parity tests, then the driver's bench command with and without
# carry-over (and K = 60) on the same box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_selfplay_run.py tests/test_gpu_headline.py -x -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/carry_tests.log 2>&1 || { tail -30 gpurun_out/carry_tests.log; exit 1; }
tail -3 gpurun_out/carry_tests.log
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --no-carry" "--steps 60 --warmup 5" "--steps 60 --warmup 5 --no-carry"; do
  timeout -k 10 400 python bench.py $args --no-cpu-baseline --net-steps 0 > gpurun_out/bench_carry.log 2>&1 || { tail -20 gpurun_out/bench_carry.log; exit 1; }
  grep '^{' gpurun_out/bench_carry.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['extra']; print('$args', d['value']/1e9, d['ms_per_step'], x['selfplay_launch_ms'], x['moves'], (x.get('launch_pooled_no_carry') or {}).get('value',0)/1e9, x['reference_schedule']['value']/1e9)"
done
