#!/bin/bash
# Round 4: the whole GPU suite on the final library, then the prefix and hash
# plans' device steps at 100M topics per rank (one GPU, world 1: the permute /
# unpermute and merge launches at full batch size) with the oracle sample.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_g
mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for plan in prefix hash; do
  timeout -k 10 400 python3 -u bench.py --config c5 --plan $plan --filters 10000000 --topics 100000000 --steps 3 --warmup 1 --no-cpu > $O/bench_c5_${plan}_100m.log 2>&1 || { tail -20 $O/bench_c5_${plan}_100m.log; exit 1; }
  tail -n 1 $O/bench_c5_${plan}_100m.log > $O/bench_c5_${plan}_100m.json
  python3 -c "import json; d=json.load(open('$O/bench_c5_${plan}_100m.json')); print('$plan', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', 'parity', d.get('parity_sample',{}).get('ok'), d.get('detail',{}).get('device_exchange'))"
done
