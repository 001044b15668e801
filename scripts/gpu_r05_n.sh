#!/bin/bash
# Round 5, GPU call n: the staged lazy-mirror download -- image / update /
# multi-device tests, then the C5 line (its first update downloads the 38 GB mirror).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r05_n}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_image.py tests/test_gpu_updates.py tests/test_gpu_multi.py -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
GM_INDEX_STATS=1 timeout -k 10 700 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu --no-host-io \
  > $O/bench_c5.log 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
tail -n 1 $O/bench_c5.log > $O/bench_c5.json
python3 -c "
import json
d = json.load(open('gpurun_out/${TAG:-r05_n}/bench_c5.json'))
print(round(d['value'] / 1e9, 3), d['ms_per_step'], d['detail'].get('index_build_s'), d['detail'].get('index_update'), d.get('parity_sample', {}).get('ok'))
"
