#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 --output-format csv -- python3 tools/bench_configs.py --only 3 --frames 200 > gpurun_out/prof_c3.log 2>&1
echo "c3 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python3 tools/bench_configs.py --only 5 --steps 3 --warmup 2 > gpurun_out/prof_c5.log 2>&1
echo "c5 rc=$?"
