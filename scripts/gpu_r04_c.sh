#!/bin/bash
# Round 4, GPU call c: the level-0 round from registers (IX_D0): parity suite
# (parity, updates, images), then a same-box A/B GM_D0=0 / default on C2 and C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_updates.py tests/test_gpu_image.py > $O/pytest.log 2>&1
rc=$?
tail -n 5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for cfg in c2 c3; do
  for v in 0 1 0 1; do
    export GM_D0=$v
    timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu --no-parity --no-host-io --no-update \
      > $O/bench_${cfg}_d0$v.log 2>&1 || { tail -5 $O/bench_${cfg}_d0$v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_d0$v.log').read().strip().splitlines()[-1]); print('$cfg d0=$v', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'kernel ms', round(d['value']/1e9,3), 'G/s', 'probes/topic', round(d['detail']['probes_per_topic'],3), 'nnz', d['detail']['nnz_per_step'])" | tee -a $O/d0_ab.txt
  done
done
