#!/bin/bash
# PMC passes (tools/pmc_kernel.sh) of gconv_wgrad3 at the four config-2 shapes it serves -> profiles/pmc_gconv_wgrad3_<shape>.json
# (256 -> 256 runs the wide plan, gconv_wgrad3w_kernel)
set -e
for c in "64to64 gconv_fwd_c64 gconv_wgrad3_kernel" "128to128 gconv_fwd_c128 gconv_wgrad3_kernel" \
         "256to256 gconv_fwd_c256 gconv_wgrad3w_kernel" "128to256 gconv_fwd_128to256 gconv_wgrad3_kernel"; do
  set -- $c
  bash tools/pmc_kernel.sh gconv_wgrad3_$1 $3 tools/bench_conv.py 3 $2
done
