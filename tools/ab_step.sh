#!/bin/bash
# Interleaved whole-step A/B of library builds on ONE box (config-2 bench line, no CPU baseline / layer roofline):
#   LIBS="lib lib_alt" REPS=3 bash tools/ab_step.sh [extra bench.py args]
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=${LIBS:-"lib lib_alt"}
for rep in $(seq 1 ${REPS:-3}); do
  for v in $LIBS; do
    STGCN_LIB=$PWD/realtime-st-gcn_amd/$v/libstgcn_amd.so timeout -k 10 180 python bench.py --steps 150 --no-cpu-baseline \
      --no-layer-roofline --kernel-steps 0 "$@" > gpurun_out/ab_step.json 2> gpurun_out/ab_step.err || { tail -5 gpurun_out/ab_step.err; exit 1; }
    echo "$v rep $rep: $(tail -1 gpurun_out/ab_step.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
