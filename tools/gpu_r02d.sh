#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_gconv.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r02d.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/gpu_tests_r02d.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r02d.json 2> gpurun_out/bench_r02d.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_r02d.json; tail -3 gpurun_out/bench_r02d.err
exit $rc
