#!/bin/bash
# Round 6, GPU call y: fan-out tests and the C4 line after the clamp went
# behind a flag (only small host fan-outs clamp to the device's total).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${OUT:-r06_y}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "fanout or c4" \
  tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_scale.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2; do
  timeout -k 10 600 python3 -u bench.py --config c4 --steps 10 --warmup 3 > $O/bench_c4_$k.log 2>&1 || { tail -5 $O/bench_c4_$k.log; exit 1; }
  tail -n 1 $O/bench_c4_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value']/1e9, d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
