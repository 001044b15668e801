#!/bin/bash
# Round 4 A/B: load factor of the open-addressing tables (GM_HOT_LOAD_PCT, default 25) with the 6-key MPH buckets
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_p
mkdir -p $O
run() {  # run <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config c2 --steps 8 --warmup 2 --no-cpu --no-host-io --no-update \
    > $O/b_$lab.log 2>&1 || { tail -5 $O/b_$lab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$lab.log').read().strip().splitlines()[-1]); print('c2 $lab', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'kernel ms', 'parity', d.get('parity_sample',{}).get('ok'))" | tee -a $O/hotload.txt
}
for rep in 1 2; do
  run base GM_X=0
  run load30 GM_HOT_LOAD_PCT=30
  run load20 GM_HOT_LOAD_PCT=20
done
