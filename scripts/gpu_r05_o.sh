#!/bin/bash
# Round 5, GPU call o: the C5 lines on the shipped library -- replicated (100M
# filters) and the prefix plan at world 1 (10M filters), both with parity samples.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_o
mkdir -p $O
GM_INDEX_STATS=1 timeout -k 10 700 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu --no-host-io \
  > $O/bench_c5.log 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
tail -n 1 $O/bench_c5.log > $O/bench_c5.json
timeout -k 10 400 python3 -u bench.py --config c5 --plan prefix --filters 10000000 --steps 10 --warmup 2 --no-cpu \
  > $O/bench_c5_prefix_10m.log 2>&1 || { tail -20 $O/bench_c5_prefix_10m.log; exit 1; }
tail -n 1 $O/bench_c5_prefix_10m.log > $O/bench_c5_prefix_10m.json
python3 -c "
import json
for f in ('bench_c5', 'bench_c5_prefix_10m'):
    d = json.load(open('gpurun_out/r05_o/%s.json' % f))
    print(f, round(d['value'] / 1e9, 3), 'G/s', round(d['ms_per_step'], 3), 'ms', (d.get('detail') or {}).get('index_build_s'), d.get('parity_sample', {}).get('ok'))
"
