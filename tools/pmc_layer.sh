#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) over tools/bench_layer.py: the fused layer kernel's counters,
# BatchNorm (layer_fused_kernel<3, false>, pass 2 of the two-pass form) and LayerNorm (<3, true>, the whole
# layer) -> profiles/pmc_layer_fused.json, profiles/pmc_layer_fused_ln.json
export TMPDIR=/tmp
for norm in BatchNorm LayerNorm; do
  D=gpurun_out/pmc_layer_$norm
  mkdir -p $D
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    mkdir -p $D/p$i
    timeout -s KILL 90 rocprofv3 --pmc $set -d $D/p$i -o p --output-format csv -- python3 tools/bench_layer.py 3 $norm > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -3 $D/p$i.log; exit 1; }
  done
done
python3 tools/pmc_json.py gpurun_out/pmc_layer_BatchNorm "layer_fused_kernel<3, false, false>" profiles/pmc_layer_fused.json
python3 tools/pmc_json.py gpurun_out/pmc_layer_LayerNorm "layer_fused_kernel<3, true, false>" profiles/pmc_layer_fused_ln.json
