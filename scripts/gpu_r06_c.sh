#!/bin/bash
# Round 6, GPU call c: the bench's two-rank test on the new library, then a C2 bench line (multi-device block, link roofline).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bench.py::test_bench_two_ranks_c2 -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python3 -u bench.py --config c2 > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -n 1 $O/bench_c2.log > $O/bench_c2.json
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r06_c/bench_c2.json'))
r=d['roofline']; de=d['detail']
print('c2', round(d['value']/1e9,3),'G/s', round(d['ms_per_step'],3),'ms/step kernel', round(r['kernel_ms'],3), 'frac', round(r['frac'],3))
print('host_io', round(de['host_io_topics_per_s']/1e9,3), 'link', json.dumps(de['host_io_link']))
print('update', json.dumps(de['index_update']))
print('multi', json.dumps(de['multi_device']))
PY
