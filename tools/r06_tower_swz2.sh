#!/bin/bash
# The swizzled tower layout with single-buffered B operands (tower_epi 3, tower_mfma16_swz1):
# A/B against the padded product layout (tools/ab_tower_swz.py: ms, TFLOP/s, bit-identity) and
# the LDS counters of both (tools/one_tower.py under rocprofv3, ZC_TOWER_EPI read at load), all on
# the variant library zeroclone_amd/libzc_swz2.so (the patch tools/experiments/tower_swizzled_single_b.patch).
set -e
export ZC_LIB=$PWD/zeroclone_amd/libzc_swz2.so
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_tower_swz.py > gpurun_out/ab_swz2.log 2>&1
for e in 0 3; do
  ZC_TOWER_EPI=$e timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/swz2_pmc$e -o b \
    --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT \
    -- python3 tools/one_tower.py > gpurun_out/swz2_pmc$e.log 2>&1
  ZC_TOWER_EPI=$e timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/swz2_pmc$e -o a \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS \
    -- python3 tools/one_tower.py >> gpurun_out/swz2_pmc$e.log 2>&1
done
