#!/bin/bash
# Round 6: PMC profiles of C1 (k_match_fused, 1M topics) and C4 (k_fanout_copy)
# on the final library, then their traffic files and bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
P=gpurun_out/profiles/r06_final4
mkdir -p $P
CONFIG=c1 TOPICS=1000000 PROF_TAG=_c1 bash scripts/profile.sh || exit 1
python3 scripts/traffic.py gpurun_out/prof_c1 --config c1 --topics 1000000 --out profiles/traffic_c1.json > gpurun_out/traffic_c1.log 2>&1 || { cat gpurun_out/traffic_c1.log; exit 1; }
CONFIG=c4 TOPICS=1000 PROF_TAG=_c4 bash scripts/profile.sh || exit 1
python3 scripts/traffic.py gpurun_out/prof_c4 --config c4 --kernel k_fanout_copy --topics 1000 --out profiles/traffic_c4.json > gpurun_out/traffic_c4.log 2>&1 || { cat gpurun_out/traffic_c4.log; exit 1; }
for c in c1 c4; do
  cp profiles/traffic_$c.json $P/
  cp gpurun_out/prof_$c/stats/run_kernel_stats.csv $P/kernel_stats_$c.csv
  for f in gpurun_out/prof_$c/*.log; do cp "$f" $P/${c}_$(basename $f); done
done
for c in c1 c4; do
  extra=""; [ $c = c4 ] && extra="--steps 10 --warmup 3"
  timeout -k 10 600 python3 -u bench.py --config $c $extra > gpurun_out/bench_$c.log 2>&1 || { tail -5 gpurun_out/bench_$c.log; exit 1; }
  tail -n 1 gpurun_out/bench_$c.log > $P/bench_$c.json
  python3 -c "import json; d=json.load(open('$P/bench_$c.json')); r=d['roofline']; print('$c', d['value'], r['frac'], r.get('traffic'), r.get('traffic_source'))"
done
