#!/bin/bash
# A/B of an env switch on ONE box, interleaved full-step bench runs: tools/ab_env.sh VAR "A B" [steps]
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=$1; VALS=$2; STEPS=${3:-100}
for rep in ${REPS:-1 2 3}; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps $STEPS --warmup 10 --no-cpu-baseline > gpurun_out/ab_env_$v.json 2>/dev/null || exit 1
    echo "$VAR=$v rep $rep: $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' gpurun_out/ab_env_$v.json)"
  done
done
