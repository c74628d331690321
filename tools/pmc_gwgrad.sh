#!/bin/bash
# PMC passes (tools/pmc_kernel.sh) of gconv_wgrad3 at the four config-2 shapes it serves -> profiles/pmc_gconv_wgrad3_<shape>.json
set -e
for c in "64to64 gconv_fwd_c64" "128to128 gconv_fwd_c128" "256to256 gconv_fwd_c256" "128to256 gconv_fwd_128to256"; do
  set -- $c
  bash tools/pmc_kernel.sh gconv_wgrad3_$1 gconv_wgrad3_kernel tools/bench_conv.py 3 $2
done
