#!/bin/bash
# Round 5, GPU call l: the index build after the parallel trie / sweep / fills
# -- C5 (100M filters) and C3 (10M) bench lines with the build's phase times
# (GM_INDEX_STATS) and their parity samples.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r05_l}
mkdir -p $O
GM_INDEX_STATS=1 timeout -k 10 900 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu --no-host-io \
  > $O/bench_c5.log 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
tail -n 1 $O/bench_c5.log > $O/bench_c5.json
grep "gm_index\] [a-z]" $O/bench_c5.err | head -20
GM_INDEX_STATS=1 timeout -k 10 400 python3 -u bench.py --config c3 --steps 10 --warmup 2 --no-host-io \
  > $O/bench_c3.log 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
tail -n 1 $O/bench_c3.log > $O/bench_c3.json
export O
python3 -c "
import json, os
for c in ('c5', 'c3'):
    d = json.load(open(os.environ['O'] + '/bench_%s.json' % c))
    print(c, round(d['value'] / 1e9, 3), 'G/s', round(d['ms_per_step'], 3), 'ms', 'build_s', d['detail'].get('index_build_s'), 'compile_s', d['detail'].get('index_compile_s'), 'rss', d['detail'].get('host_peak_rss_gb'), 'parity', d.get('parity_sample', {}).get('ok'), 'upd', d['detail'].get('index_update'))
"
