#!/bin/bash
# The tower layouts: exactness tests, then the A/B timing (tools/ab_tower_swz.py).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_net.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_net.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python tools/ab_tower_swz.py > gpurun_out/ab_tower_swz.log 2>&1; rc=$?; grep -v '^{' gpurun_out/ab_tower_swz.log | tail -4; exit $rc
