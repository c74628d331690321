#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 3 29 61 93 125 13 45 77 109; do
  STGCN_FUSED_DBG=$d timeout -k 10 120 python tools/bench_layer.py 20 > gpurun_out/layer_dbg$d.json 2>&1 || exit 1
  echo "dbg $d: $(tail -1 gpurun_out/layer_dbg$d.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["fused_kernel_ms"])')"
done
