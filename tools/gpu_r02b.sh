#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_rt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r02b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_r02b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/bench_r02b.json 2> gpurun_out/bench_r02b.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_r02b.json; tail -3 gpurun_out/bench_r02b.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_configs.py --frames 2000 --steps 20 > gpurun_out/configs_r02b.json 2> gpurun_out/configs_r02b.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs_r02b.json; tail -3 gpurun_out/configs_r02b.err
exit $rc
