#!/bin/bash
# Random-read calibration (scripts/randread.hip): loads/s and fabric requests
# per 16-B random load, independent vs dependent, MALL-resident vs not.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/scripts/randread
O=$GRAFT_REPO_ROOT/gpurun_out/randread
mkdir -p $O
for cfg in "2048 0 8" "2048 0 4" "2048 0 2" "2048 1 8" "128 0 8" "128 1 8" "16 0 8" "2048 0 8 256 4" "2048 0 8 256 64" "128 0 8 256 64"; do
  timeout -k 10 60 $R $cfg | tee -a $O/sweep.jsonl
done
for cfg in "2048 0 8" "128 0 8" "2048 0 8 256 64"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum -d $O/pmc_$tag -o run --output-format csv -- $R $cfg > $O/pmc_$tag.log 2>&1
done
find $O -name "*counter_collection.csv" | head
