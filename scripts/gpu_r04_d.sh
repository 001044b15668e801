#!/bin/bash
# Round 4: the split tile scan's sums mode (GM_SCAN_SUMS): parity suite, then a
# same-box C1 A/B (GM_SCAN_SUMS=0 / default), 400 timed steps each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py > $O/pytest.log 2>&1
rc=$?
tail -n 5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1 0 1; do
  export GM_SCAN_SUMS=$v
  timeout -k 10 300 python3 -u bench.py --config c1 --steps 400 --warmup 40 --no-cpu --no-parity --no-host-io --no-update \
    > $O/bench_c1_s$v.log 2>&1 || { tail -5 $O/bench_c1_s$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_c1_s$v.log').read().strip().splitlines()[-1]); print('c1 sums=$v', round(d['ms_per_step'],4), 'ms/step', round(d['roofline']['kernel_ms'],4), 'kernel ms', round(d['value']/1e9,3), 'G/s')" | tee -a $O/sums_ab.txt
done
