#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r02e.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/gpu_tests_r02e.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_layer.py 20 > gpurun_out/layer_r02e.json 2>&1
rc=$?; echo "layer rc=$rc"; cat gpurun_out/layer_r02e.json | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_layer -o layer --output-format csv -- python3 tools/bench_layer.py 10 > gpurun_out/prof_layer.log 2>&1
echo "prof rc=$?"
