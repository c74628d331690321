#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r02j.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_r02j.log
[ $rc -eq 0 ] || exit $rc
for d in 0 1 2 3; do
  STGCN_FUSED_DBG=$d timeout -k 10 120 python tools/bench_layer.py 20 > gpurun_out/layer_dbg$d.json 2>&1 || exit 1
  echo "dbg $d: $(tail -1 gpurun_out/layer_dbg$d.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["fused_kernel_ms"], d["fused_fwd_ms"], d["unfused_fwd_ms"])')"
done
