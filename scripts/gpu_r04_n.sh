#!/bin/bash
# Round 4 A/B: 6 keys per MPH bucket with more spare slots (GM_MPH_SLACK=16: keys/16)
# bucket words in L2 against a fuller Bloom filter (5 places without overflow;
# 6 and 8 spill into the overflow region on this set).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_n
mkdir -p $O
run() {  # run <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config c2 --steps 8 --warmup 2 --no-cpu --no-host-io --no-update \
    > $O/b_$lab.log 2>&1 || { tail -5 $O/b_$lab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$lab.log').read().strip().splitlines()[-1]); print('c2 $lab', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'kernel ms', 'parity', d.get('parity_sample',{}).get('ok'))" | tee -a $O/lambda6.txt
}
for rep in 1 2; do
  run base GM_X=0
  run lam6s16 GM_MPH_LAMBDA=6 GM_MPH_SLACK=16
  run lam5s16 GM_MPH_LAMBDA=5 GM_MPH_SLACK=16
done
