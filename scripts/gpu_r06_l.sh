#!/bin/bash
# Round 6, GPU call l: the whole GPU suite after the concurrent small host
# calls (staging and device wait outside the context lock), then a C2 line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_l
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --config c2 --no-cpu > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -n 1 $O/bench_c2.log > $O/bench_c2.json
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r06_l/bench_c2.json')); de=d['detail']
print('c2', round(d['value']/1e9,3), 'host_io', round(de['host_io_topics_per_s']/1e9,3))
print('small single', json.dumps(de.get('small_calls_single_device')))
m=de['multi_device']; print('small multi', json.dumps(m.get('small_calls')))
PY
