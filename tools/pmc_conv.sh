#!/bin/bash
export TMPDIR=/tmp
C=${1:-tcn_fwd_c64}
i=0
mkdir -p gpurun_out/pmc_$C
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set -d gpurun_out/pmc_$C/p$i -o p --output-format csv -- python3 tools/bench_conv.py 3 $C > gpurun_out/pmc_$C/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -3 gpurun_out/pmc_$C/p$i.log; }
done
