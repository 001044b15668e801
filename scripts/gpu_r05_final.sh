#!/bin/bash
# Round 5 final measurement on the final library: rocprofv3 stats + PMC of C2
# and C3 (traffic.json / traffic_c3.json for this library), the bench lines of
# C2 (default, with CPU baseline and parity), C1, C3 and C4 -> profiles/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05_final}
P=gpurun_out/profiles/$TAG
mkdir -p $P
for cfg in c2 c3; do
  if [ $cfg = c2 ]; then extra=""; out=profiles/traffic.json; else extra="--index-cache /dev/shm/gm_c3_$$.img"; out=profiles/traffic_c3.json; fi
  CONFIG=$cfg PROF_TAG=_$cfg BENCH_ARGS="$extra" bash scripts/profile.sh || exit $?
  python3 scripts/traffic.py gpurun_out/prof_$cfg --config $cfg --out $out > gpurun_out/traffic_$cfg.log 2>&1 || { cat gpurun_out/traffic_$cfg.log; exit 1; }
  cp $out $P/
  cp gpurun_out/prof_$cfg/stats/run_kernel_stats.csv $P/kernel_stats_$cfg.csv
  for f in gpurun_out/prof_$cfg/*.log; do cp "$f" $P/${cfg}_$(basename $f); done
  python3 scripts/pmc_summary.py gpurun_out/prof_$cfg > $P/pmc_per_launch_$cfg.json
done
for cfg in c2 c1 c3 c4; do
  extra=""; [ $cfg = c3 ] && extra="--index-cache /dev/shm/gm_c3_$$.img"
  [ $cfg = c4 ] && extra="--steps 10 --warmup 3"
  timeout -k 10 600 python3 -u bench.py --config $cfg $extra > gpurun_out/bench_$cfg.log 2>&1 || { tail -5 gpurun_out/bench_$cfg.log; exit 1; }
  tail -n 1 gpurun_out/bench_$cfg.log > $P/bench_$cfg.json
  python3 -c "import json; d=json.load(open('$P/bench_$cfg.json')); r=d.get('roofline',{}); print('$cfg', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms/step', round(r.get('kernel_ms',0),4), 'kernel ms', 'frac', round(r.get('frac',0),3), 'traffic', r.get('traffic'), 'lines', r.get('lines_per_topic'), 'parity', d.get('parity_sample',{}).get('ok'))"
done
rm -f /dev/shm/gm_c3_$$.img
