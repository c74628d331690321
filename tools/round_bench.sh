#!/bin/bash
# Round-closing numbers (run on the GPU box): full GPU suite, smoke, the official bench line (config 2, CPU
# baseline, layer rooflines), config 4, graph-mode step, configs 3/5/f1, rocprofv3 kernel summary of the default
# (single-stream) step.  Output in gpurun_out/; copy what is judged into profiles/.   bash tools/round_bench.sh r03
export TMPDIR=/tmp
TAG=${1:-r04}
mkdir -p gpurun_out
STGCN_TEST_REPORT=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
echo "bench: $(cut -c1-200 gpurun_out/bench_$TAG.json)"
timeout -k 10 300 python bench.py --config 4 --steps 120 --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
timeout -k 10 300 python bench.py --graph --steps 120 --no-cpu-baseline --no-layer-roofline > gpurun_out/bench_graph_$TAG.json 2> gpurun_out/bench_graph_$TAG.err || exit $?
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs_$TAG.json 2> gpurun_out/configs_$TAG.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-layer-roofline --kernel-steps 0 > gpurun_out/prof_$TAG.log 2>&1
echo "prof rc=$?"
