#!/bin/bash
# Interleaved A/B/... of library builds on ONE box: tools/bench_conv.py cases against every lib dir given.
#   LIBS="lib lib_a lib_b" CASES="gconv_fwd_c64 gconv_fwd_c256" bash tools/ab_libs.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=${LIBS:-"lib lib_alt"}
for rep in 1 2; do
  for v in $LIBS; do
    for c in $CASES; do
      STGCN_LIB=$PWD/realtime-st-gcn_amd/$v/libstgcn_amd.so timeout -k 10 120 python tools/bench_conv.py 30 $c > gpurun_out/abc.txt 2>&1 || { cat gpurun_out/abc.txt; exit 1; }
      grep -v "amdgpu.ids\|gcn_tile\|^$" gpurun_out/abc.txt | sed "s/^/$v $rep /"
    done
  done
done
