#!/bin/bash
# GPU box script: tests, stage debug, short bench.  Stops on any crash-like exit status.
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
ok $rc || exit $rc
timeout -k 10 120 python tools/debug_layer.py 256 256 1 BatchNorm > gpurun_out/debug.log 2>&1
rc=$?; echo "debug rc=$rc"; cat gpurun_out/debug.log | tail -8
ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
