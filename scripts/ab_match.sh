#!/bin/bash
# A/B of k_match variants at C2 on the GPU box: parity tests once, then the
# bench per variant (GM_MATCH_MAIN), each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -n 15 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for v in ${VARIANTS:-split splitw8 split2}; do
  GM_MATCH_MAIN=$v timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_$v.log 2>&1
  rc=$?; echo "MAIN=$v rc=$rc"; tail -n 1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']/1e9, 'Gtopics/s kernel_ms', d['roofline']['kernel_ms'], 'listed', d['detail']['overflow_rows'])" || tail -n 5 gpurun_out/ab_$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
