# L2 / vector-L1 counters of the fused tower (tools/one_tower.py, 8x8 x 32768): where its
# weight fragments come from.  Run on the GPU box from the repo root.
set -e
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_tower_l2 -o c --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -- python3 tools/one_tower.py > gpurun_out/pmc_tower_c.log 2>&1
