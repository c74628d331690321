#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) over tools/bench_layer.py: the LayerNorm one-kernel layer
# (layer_fused_kernel<3>, the north_star layer's inference forward) -> profiles/pmc_layer_fused_ln.json;
# with STGCN_LIB pointing at another build (e.g. -DSTGCN_FUSED_DBG=16: y stores dropped), TAG names the output.
export TMPDIR=/tmp
TAG=${TAG:-layer_fused_ln}
D=gpurun_out/pmc_$TAG
mkdir -p $D
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  mkdir -p $D/p$i
  timeout -s KILL 90 rocprofv3 --pmc $set -d $D/p$i -o p --output-format csv -- python3 tools/bench_layer.py 3 LayerNorm > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -3 $D/p$i.log; exit 1; }
done
python3 tools/pmc_json.py $D "layer_fused_kernel<3>" profiles/pmc_$TAG.json
