#!/bin/bash
# Chess generator change: the chess parity tests, then the crude search A/B (per move, outputs
# hashed) and the pooled crude figure, base library vs product.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_chess.py tests/test_gpu_chess_search.py tests/test_gpu_chess_rollouts.py \
  tests/test_gpu_chess_selfplay.py tests/test_gpu_api_chess.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/chess_tests.log 2>&1 || { tail -30 gpurun_out/chess_tests.log; exit 1; }
tail -2 gpurun_out/chess_tests.log
timeout -k 10 400 python tools/ab_chess.py ${LIBS:-zeroclone_amd/lib_chbase.so zeroclone_amd/libzeroclone_amd.so} 2>&1 | tail -6 || exit 1
timeout -k 10 400 python tools/ab_chess_pooled.py ${LIBS:-zeroclone_amd/lib_chbase.so zeroclone_amd/libzeroclone_amd.so} 2>&1 | tail -6
