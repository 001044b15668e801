#!/bin/bash
# A/B of k_match_fast variants at C2 on the GPU box: parity tests once, then the
# bench per variant (GM_MATCH_CH), each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -n 15 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
for ch in ${CHS:-1 2}; do
  GM_MATCH_CH=$ch timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_ch$ch.log 2>&1
  rc=$?; echo "CH=$ch rc=$rc"; tail -n 2 gpurun_out/ab_ch$ch.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
done
exit 0
