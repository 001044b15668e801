#!/bin/bash
# Patch update with exact capacity checks: update tests, then update perf with phase timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02i
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_updates.py \
  > gpurun_out/r02i/updates.txt 2>&1 || { tail -40 gpurun_out/r02i/updates.txt; exit 1; }
tail -3 gpurun_out/r02i/updates.txt
GM_UPDATE_TIMING=1 timeout -k 10 600 python3 -u scripts/update_perf.py 100 1000 10000 > gpurun_out/r02i/update_perf.jsonl 2> gpurun_out/r02i/update_perf.err \
  || { tail -20 gpurun_out/r02i/update_perf.err; exit 1; }
grep gm_update gpurun_out/r02i/update_perf.err || true
cat gpurun_out/r02i/update_perf.jsonl
