#!/bin/bash
# Round 4 re-check of chain nodes with the 6-key MPH tables: C2 with chains
# (GM_CHAIN=1; built by default only past 256 MiB of tables) and C3 without.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_u
mkdir -p $O
run() {  # run <cfg> <label> <env...>
  local cfg=$1 lab=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cfg --steps 6 --warmup 2 --no-cpu --no-host-io --no-update \
    > $O/b_${cfg}_$lab.log 2>&1 || { tail -5 $O/b_${cfg}_$lab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_${cfg}_$lab.log').read().strip().splitlines()[-1]); print('$cfg $lab', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'kernel ms', 'parity', d.get('parity_sample',{}).get('ok'))" | tee -a $O/chain.txt
}
for rep in 1 2; do
  run c2 base GM_X=0
  run c2 chain GM_CHAIN=1
done
for rep in 1 2; do
  run c3 base GM_X=0
  run c3 nochain GM_CHAIN=0
done
