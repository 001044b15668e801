#!/bin/bash
# Round 5, GPU call f: the C5 line (100M filters, replicated, 100M topics) with
# the index_update detail (the first update downloads the 38 GB lazy mirror)
# and the subscriber-update detail at 100M filters (--subs-update: a second
# 100M-filter index built with one subscriber per filter).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_f
mkdir -p $O
timeout -k 10 1100 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu --no-host-io --subs-update \
  > $O/bench_c5.log 2>&1
rc=$?
tail -c 400 $O/bench_c5.log
python3 -c "
import json
d = json.loads(open('gpurun_out/r05_f/bench_c5.log').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value'] / 1e9, d.get('parity_sample'))
print({k: v for k, v in d['detail'].items() if k.startswith(('subs', 'index_update', 'index_build', 'host_peak'))})
"
exit $rc
