#!/bin/bash
# Update-path tests and latency (round 3): the GPU update tests, then
# scripts/update_c23.py for C2 and C3 with phase times.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${TAG:-r03u}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_updates.py tests/test_gpu_mirror.py -v -m gpu --timeout 500 \
  --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest.log | tail -n 20
[ $rc -ne 0 ] && exit $rc
GM_UPDATE_TIMING=1 timeout -k 10 600 python3 -u scripts/update_c23.py c2 c3 > $OUT/update.jsonl 2> $OUT/update_phases.txt
rc=$?; cat $OUT/update.jsonl; tail -n 12 $OUT/update_phases.txt
exit $rc
