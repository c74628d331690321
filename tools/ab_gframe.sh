#!/bin/bash
# frame-kernel timing ablations at C = 64 (tools builds lib_d1..lib_d4, -DGCF_DBG / -DGWF_DBG): full kernels, no
# compute, no barrier, no DMA, no stores; tools/bench_gframe.py 64->64 per build
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in lib lib_d1 lib_d2 lib_d3 lib_d4; do
  STGCN_LIB=$PWD/realtime-st-gcn_amd/$v/libstgcn_amd.so timeout -k 10 120 python tools/bench_gframe.py 20 "64->64" > gpurun_out/abg_$v.json 2> gpurun_out/abg_$v.err || { tail -3 gpurun_out/abg_$v.err; exit 1; }
  echo "$v: $(cat gpurun_out/abg_$v.json)"
done
