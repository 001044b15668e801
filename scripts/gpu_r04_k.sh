#!/bin/bash
# Round 4 A/B: the large tables' home-slot probes as plain nt loads
# (GM_HOT_POLICY=3: evict-first in the XCD L2, Infinity Cache still used) --
# the one load policy scripts/gpu_r04_e.sh did not try.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_k
mkdir -p $O
IMG=/dev/shm/gm_c3_$$.img
trap 'rm -f $IMG' EXIT
run() {  # run <cfg> <label> <env...>
  local cfg=$1 lab=$2; shift 2
  local extra=""; [ $cfg = c3 ] && extra="--index-cache $IMG"
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cfg $extra --steps 8 --warmup 2 --no-cpu --no-host-io --no-update \
    > $O/b_${cfg}_$lab.log 2>&1 || { tail -5 $O/b_${cfg}_$lab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_${cfg}_$lab.log').read().strip().splitlines()[-1]); print('$cfg $lab', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'kernel ms', 'parity', d.get('parity_sample',{}).get('ok'))" | tee -a $O/policy_nt.txt
}
for cfg in c2 c3; do
  for rep in 1 2; do
    run $cfg base GM_X=0
    run $cfg big_nt GM_L1_BYPASS=0x38 GM_HOT_POLICY=3
    run $cfg t45_nt GM_L1_BYPASS=0x30 GM_HOT_POLICY=3
    run $cfg t3_nt GM_L1_BYPASS=0x08 GM_HOT_POLICY=3
  done
done
