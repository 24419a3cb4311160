#!/bin/bash
# C5 (chess PUCT) after the deferred parallel expansion: the PUCT parity tests, then the C5
# step A/B against the previous library (tools/ab_c5.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_puct.py tests/test_gpu_pools.py::test_c5_chess_puct_pool_matches_puct_ref tests/test_gpu_fullshape.py::test_c5_chess_puct_full_shape -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_c5.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_c5.log; [ $rc -eq 0 ] || exit $rc
ZC_PUCT_STREAMS=4 bash tools/ab_c5.sh zeroclone_amd/lib_c5base.so zeroclone_amd/libzeroclone_amd.so 2 2>&1 | tee gpurun_out/ab_c5.log
