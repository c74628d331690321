#!/bin/bash
# A/B of an environment switch on ONE box, interleaved: bench_conv cases with and without it.
# usage: ENVSET="STGCN_GCONV_SCATTER=1" CASES="gconv_fwd_c64 ..." bash tools/ab_env.sh
export TMPDIR=/tmp
for rep in 1 2; do
  for mode in base env; do
    for c in $CASES; do
      if [ $mode = env ]; then out=$(env $ENVSET timeout -k 10 120 python tools/bench_conv.py 30 $c 2>&1 | grep -v amdgpu.ids)
      else out=$(timeout -k 10 120 python tools/bench_conv.py 30 $c 2>&1 | grep -v amdgpu.ids); fi
      echo "$mode $rep $out"
    done
  done
done
