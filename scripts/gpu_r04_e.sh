#!/bin/bash
# Round 4 A/B: cache policies -- the compact staging list stored sc1
# (GM_STAGE_SC1), and the large tables' probes as sc0 sc1 / sc1 nt loads
# (GM_L1_BYPASS table mask + GM_HOT_POLICY) -- on C2 and C3, same box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_e
mkdir -p $O
IMG=/dev/shm/gm_c3_$$.img
trap 'rm -f $IMG' EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "compact_staging or submit_wait or edge_cases or random_sets" > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
GM_STAGE_SC1=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "compact_staging or submit_wait" > $O/pytest_sc1.log 2>&1
rc=$?; tail -n 3 $O/pytest_sc1.log; [ $rc -ne 0 ] && exit $rc
run() {  # run <cfg> <label> <env...>
  local cfg=$1 lab=$2; shift 2
  local extra=""; [ $cfg = c3 ] && extra="--index-cache $IMG"
  env "$@" timeout -k 10 300 python3 -u bench.py --config $cfg $extra --steps 8 --warmup 2 --no-cpu --no-parity --no-host-io --no-update \
    > $O/b_${cfg}_$lab.log 2>&1 || { tail -5 $O/b_${cfg}_$lab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_${cfg}_$lab.log').read().strip().splitlines()[-1]); print('$cfg $lab', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'kernel ms')" | tee -a $O/policy_ab.txt
}
for cfg in c2 c3; do
  for rep in 1 2; do
    run $cfg base GM_X=0
    run $cfg stage_sc1 GM_STAGE_SC1=1
    run $cfg big_sys GM_L1_BYPASS=0x38 GM_HOT_POLICY=2
    run $cfg big_sc1nt GM_L1_BYPASS=0x38 GM_HOT_POLICY=4
    run $cfg t45_sys GM_L1_BYPASS=0x30 GM_HOT_POLICY=2
  done
done
