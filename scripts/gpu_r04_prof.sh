#!/bin/bash
# Round 4 measurement: rocprofv3 stats + PMC passes of C2 and C3 (C3 from an
# index image cached in /tmp after the first pass), traffic_<config>.json from
# them, then the bench lines of C2 and C3 on this library, and the 2-rank
# rehearsals (replicated build-once, prefix, C4).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r04_v1}
P=gpurun_out/profiles/$TAG
mkdir -p $P
df -h /tmp /dev/shm > $P/box_disk.txt 2>&1
free -g >> $P/box_disk.txt 2>&1
for cfg in ${CONFIGS:-c2 c3}; do
  if [ $cfg = c2 ]; then extra=""; out=profiles/traffic.json; else extra="--index-cache /tmp/gm_$cfg.img"; out=profiles/traffic_$cfg.json; fi
  CONFIG=$cfg PROF_TAG=_$cfg BENCH_ARGS="$extra" bash scripts/profile.sh || exit $?
  python3 scripts/traffic.py gpurun_out/prof_$cfg --config $cfg --out $out > gpurun_out/traffic_$cfg.log 2>&1 || { cat gpurun_out/traffic_$cfg.log; exit 1; }
  cp $out $P/
  cp gpurun_out/prof_$cfg/stats/run_kernel_stats.csv $P/kernel_stats_$cfg.csv
  python3 scripts/pmc_summary.py gpurun_out/prof_$cfg > $P/pmc_per_launch_$cfg.json
  lim=600
  timeout -k 10 $lim python3 -u bench.py --config $cfg $extra > gpurun_out/bench_$cfg.log 2>&1 || { tail -5 gpurun_out/bench_$cfg.log; exit 1; }
  tail -n 1 gpurun_out/bench_$cfg.log > $P/bench_$cfg.json
  python3 -c "import json; d=json.load(open('$P/bench_$cfg.json')); r=d['roofline']; print('$cfg', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel ms', 'frac', round(r['frac'],3), 'traffic', r['traffic'], 'lines/topic', r.get('lines_per_topic'), 'parity', d.get('parity_sample',{}).get('ok'))"
done
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_bench.py > $P/pytest_bench.log 2>&1
rc=$?
tail -n 12 $P/pytest_bench.log
exit $rc
