#!/bin/bash
# Two-tap weight prefetch (ZC_TOWER_PF2, libzc_pf2.so / libzc_pf2st.so from tools/tower_var_libs.sh):
# stamps, wall-time A/B against the product library, and the net tests on the variant.
set -e
mkdir -p gpurun_out
ZC_LIB=$PWD/zeroclone_amd/libzc_pf2st.so timeout -k 10 200 python tools/tower_stamps.py > gpurun_out/pf2_stamps.log 2>&1
rm -f gpurun_out/abt.log
timeout -k 10 400 bash tools/ab_tower_libs.sh libzeroclone_amd.so libzc_pf2.so
ZC_LIB=$PWD/zeroclone_amd/libzc_pf2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_net.py > gpurun_out/pf2_nettests.log 2>&1
