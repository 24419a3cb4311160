# Two rocprofv3 counter passes over the fused tower (tools/one_tower.py), one per counter
# group, and a kernel-trace-only pass of 12 launches (durations without counter collection),
# for tools/summarize_tower_pmc.py.  Run on the GPU box from the repo root.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_tower -o a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS -- python3 tools/one_tower.py > gpurun_out/pmc_tower_a.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_tower -o b --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT -- python3 tools/one_tower.py > gpurun_out/pmc_tower_b.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_tower -o t -- python3 tools/one_tower.py 8 8 32768 12 > gpurun_out/pmc_tower_t.log 2>&1
