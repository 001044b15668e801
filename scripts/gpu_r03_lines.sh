#!/bin/bash
# Bench lines of the other configs on one GPU (round 3): C1, C3 and C5 with the
# replicated plan (the unsharded 100M-filter index), each under its own time
# limit, copied to gpurun_out/profiles/$TAG/bench_<config>.json.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r03}
P=gpurun_out/profiles/$TAG
mkdir -p $P
for cfg in ${CONFIGS:-c1 c3 c5}; do
  lim=300; [ $cfg = c5 ] && lim=900
  timeout -k 10 $lim python3 -u bench.py --config $cfg ${BENCH_ARGS:-} > gpurun_out/bench_$cfg.log 2>&1
  rc=$?
  tail -n 1 gpurun_out/bench_$cfg.log > $P/bench_$cfg.json
  echo "[$cfg] rc=$rc $(python3 -c "import json; d=json.load(open('$P/bench_$cfg.json')); print(round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', 'frac', round(d.get('roofline',{}).get('frac',0),3), 'parity', d.get('parity_sample',{}).get('ok'))" 2>&1)"
  [ $rc -ne 0 ] && { tail -n 5 gpurun_out/bench_$cfg.log; exit $rc; }
done
exit 0
