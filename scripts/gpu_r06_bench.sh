#!/bin/bash
# Round 6 final bench lines on the final library (its PMC traffic files are in
# profiles/): CONFIGS in order -> profiles/$TAG/bench_<cfg>.json.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06_final}
P=gpurun_out/profiles/$TAG
mkdir -p $P
for cfg in ${CONFIGS:-c2 c1 c3 c4}; do
  extra=""
  [ $cfg = c3 ] && extra="--index-cache /dev/shm/gm_c3_$$.img"
  [ $cfg = c4 ] && extra="--steps 10 --warmup 3"
  timeout -k 10 900 python3 -u bench.py --config $cfg $extra > gpurun_out/bench_$cfg.log 2>&1 || { tail -5 gpurun_out/bench_$cfg.log; rm -f /dev/shm/gm_c3_$$.img; exit 1; }
  tail -n 1 gpurun_out/bench_$cfg.log > $P/bench_$cfg.json
  python3 -c "import json; d=json.load(open('$P/bench_$cfg.json')); r=d.get('roofline',{}); print('$cfg', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms/step', round(r.get('kernel_ms',0),4), 'kernel ms', 'frac', round(r.get('frac',0),3), 'traffic', r.get('traffic'), 'lines', r.get('lines_per_topic'), 'parity', d.get('parity_sample',{}).get('ok'))"
done
rm -f /dev/shm/gm_c3_$$.img
