#!/bin/bash
# A/B of two library builds on ONE box (lib = A, lib_alt = B), interleaved: bench_layer's fused kernel time.
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in lib lib_alt; do
    STGCN_LIB=$PWD/realtime-st-gcn_amd/$v/libstgcn_amd.so timeout -k 10 120 python tools/bench_layer.py 30 > gpurun_out/ab_$v.json 2>&1 || exit 1
    echo "$v rep $rep: $(tail -1 gpurun_out/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["fused_kernel_ms"], d["fused_fwd_ms"], d["unfused_fwd_ms"])')"
  done
done
