#!/bin/bash
# tools/tower_stamps.py over the diagnostic builds of tools/tower_diag_libs.sh (args: the k's)
set -e
mkdir -p gpurun_out
for k in "${@:-0 1 2 3}"; do
  ZC_LIB=$PWD/zeroclone_amd/libzc_td$k.so timeout -k 10 200 python tools/tower_stamps.py >> gpurun_out/tower_diag.log 2>&1
done
