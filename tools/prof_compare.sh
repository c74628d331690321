#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_halo -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_halo.log 2>&1 || exit $?
export STGCN_NO_HALO=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nohalo -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_nohalo.log 2>&1
