# conv_wide diagnostic variants (STGCN_WIDE_DBG bits: 1 contiguous B fragments, 2 no helper work)
mkdir -p gpurun_out
for m in ${MODES:-0 1 2 3}; do echo "mode $m"; for c in ${CASES:-tcn_fwd_c128 tcn_fwd_c256 tcn_dgrad_c128 tcn_dgrad_c256}; do STGCN_WIDE_DBG=$m timeout -k 10 60 python tools/bench_conv.py 20 $c > gpurun_out/wd1.log 2>&1; rc=$?; grep tcn gpurun_out/wd1.log; [ $rc -eq 0 ] || exit $rc; done; done
