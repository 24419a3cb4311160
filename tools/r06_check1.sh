#!/bin/bash
# round-6 check of the Connect4 search variants (runs on the GPU box): smoke, the Connect4
# parity tests, per-game output equality of the variants, lockstep A/B and the walk replay.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS=${LIBS:-"lib_base.so lib_plan2a.so lib_plan2b.so libzeroclone_amd.so"}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke fail; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_c4.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_c4.log; [ $rc -le 1 ] || exit $rc
first=$(echo $LIBS | cut -d' ' -f1)
for l in $LIBS; do
  [ $l = $first ] && continue
  timeout -k 10 400 python tools/cmp_libs.py zeroclone_amd/$first zeroclone_amd/$l > gpurun_out/cmp_$l.log 2>&1; rc=$?; echo "cmp $l rc=$rc"; tail -3 gpurun_out/cmp_$l.log; [ $rc -le 1 ] || exit $rc
done
AB_ROOTS=mixed AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 600 python tools/ab_search.py $(for l in $LIBS; do echo zeroclone_amd/$l; done) > gpurun_out/ab.log 2>&1; rc=$?; tail -6 gpurun_out/ab.log; [ $rc -le 1 ] || exit $rc
for l in $LIBS; do ZC_LIB=$PWD/zeroclone_amd/$l timeout -k 10 300 python tools/prof_walk.py --reps 5 > gpurun_out/walk_$l.log 2>&1 || exit $?; grep '^{' gpurun_out/walk_$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l', 'walk', d['walk_ms'], 'search', d['search_ms'], d['walk_ms_all'])"; done
