#!/bin/bash
# A/B of two library builds on ONE box (lib = A, lib_alt = B), interleaved: conv kernel micro-benchmarks
# (tools/bench_conv.py) for the cases given (default: the temporal convs of the step).
export TMPDIR=/tmp
mkdir -p gpurun_out
CASES=${CASES:-"tcn_fwd_c64 tcn_fwd_c128 tcn_fwd_c256 tcn_dgrad_c128 tcn_dgrad_c256 tcn_fwd_s2_c128 tcn_dgrad_s2_c128"}
for rep in 1 2; do
  for v in lib lib_alt; do
    for c in $CASES; do
      STGCN_LIB=$PWD/realtime-st-gcn_amd/$v/libstgcn_amd.so timeout -k 10 120 python tools/bench_conv.py 30 $c > gpurun_out/abc.txt 2>&1 || { cat gpurun_out/abc.txt; exit 1; }
      echo "$v $rep $(grep -v amdgpu.ids gpurun_out/abc.txt | head -1)"
    done
  done
done
