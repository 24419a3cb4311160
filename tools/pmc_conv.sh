set -e
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
for mode in half stream; do
  if [ $mode = stream ]; then export ZC_AB_PACKED=1 ZC_CONV_WPE=3; else unset ZC_AB_PACKED ZC_CONV_WPE; fi
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$mode -o a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS -- python3 tools/one_conv.py > gpurun_out/pmc_${mode}_a.log 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$mode -o b --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT -- python3 tools/one_conv.py > gpurun_out/pmc_${mode}_b.log 2>&1
done
