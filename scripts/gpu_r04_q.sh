#!/bin/bash
# The prefix and hash plans at 100M topics per rank (10M filters, world 1) on
# the shipped library, with oracle samples.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/${QTAG:-r04_q}
mkdir -p $O
for plan in prefix hash; do
  timeout -k 10 400 python3 -u bench.py --config c5 --plan $plan --filters 10000000 --topics 100000000 --steps 3 --warmup 1 --no-cpu > $O/bench_c5_${plan}_100m.log 2>&1 || { tail -20 $O/bench_c5_${plan}_100m.log; exit 1; }
  tail -n 1 $O/bench_c5_${plan}_100m.log > $O/bench_c5_${plan}_100m.json
  python3 -c "import json; d=json.load(open('$O/bench_c5_${plan}_100m.json')); print('$plan', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', 'parity', d.get('parity_sample',{}).get('ok'))"
done
