#!/bin/bash
# PMC of tools/store_pattern (three store shapes of the same 61.44 MB): WRITE_SIZE and the write-request counters per
# dispatch, then its own timing.  Output: gpurun_out/pmc_store/
export TMPDIR=/tmp
D=gpurun_out/pmc_store
mkdir -p $D
timeout -k 10 60 ./tools/store_pattern > $D/timing.txt 2>&1 || exit $?
i=0
for set in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  mkdir -p $D/p$i
  timeout -s KILL 60 rocprofv3 --pmc $set -d $D/p$i -o p --output-format csv -- ./tools/store_pattern > $D/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
cat $D/timing.txt
