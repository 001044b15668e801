#!/bin/bash
# Round-end check of bench.py exactly as the driver runs it (N=1, defaults),
# then the prefix / hash plans at 100M topics per rank.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_r
mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -n 1 $O/bench_default.log > $O/bench_default.json
python3 -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print('default', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', r['kernel_ms'], r['kernel_ms_median'], r['frac'], r['traffic'], r.get('l2_hit_rate'), d['parity_sample']['ok'], d['cpu_baseline']['value'])"
bash scripts/gpu_r04_q.sh
