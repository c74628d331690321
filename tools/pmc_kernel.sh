#!/bin/bash
# Generic PMC passes (one counter set per rocprofv3 run) over a micro-benchmark command, then the per-dispatch
# means of one kernel -> profiles/pmc_<tag>.json.
#   bash tools/pmc_kernel.sh <tag> <kernel-name substring> <script.py> [args...]
# e.g. bash tools/pmc_kernel.sh gconv_wgrad3_c64 gconv_wgrad3_kernel tools/bench_gframe.py 3 64->64
export TMPDIR=/tmp
TAG=$1; KERN=$2; shift 2
D=gpurun_out/pmc_$TAG
mkdir -p $D
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  mkdir -p $D/p$i
  timeout -s KILL 90 rocprofv3 --pmc $set -d $D/p$i -o p --output-format csv -- python3 "$@" > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -3 $D/p$i.log; exit 1; }
done
python3 tools/pmc_json.py $D "$KERN" profiles/pmc_$TAG.json
