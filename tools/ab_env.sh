#!/bin/bash
# Interleaved A/B of bench.py variants on ONE box: each argument is "NAME:ENV=VAL,ENV2=VAL:extra bench flags"
# (empty env / flags allowed), run REPS times in turn; prints ms/step per run.  Example:
#   bash tools/ab_env.sh "plan::" "noplan:STGCN_PREP_PLAN=0:" "graph::--graph"
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-3}
STEPS=${STEPS:-100}
for rep in $(seq $REPS); do
  for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; flags=${rest#*:}
    out=gpurun_out/ab_$name.json
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python bench.py --steps $STEPS --warmup 10 --no-cpu-baseline --no-layer-roofline --kernel-steps 0 $flags > $out 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; exit 1; }
    echo "$name rep $rep: $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])' $out)"
  done
done
