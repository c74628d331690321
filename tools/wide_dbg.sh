mkdir -p gpurun_out
for m in 0 1 2 4 6 7; do echo "mode $m"; STGCN_WIDE_DBG=$m timeout -k 10 60 python tools/bench_conv.py 20 tcn_fwd_c128 2>&1 | grep tcn; STGCN_WIDE_DBG=$m timeout -k 10 60 python tools/bench_conv.py 20 tcn_fwd_c256 2>&1 | grep tcn || exit 1; done
