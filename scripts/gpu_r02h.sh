#!/bin/bash
# In-place (patch) index update: the update tests, the parity suite (rh_mask
# view change), then update latency / match time patch vs overlay vs flat at C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02h
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_updates.py \
  > gpurun_out/r02h/updates.txt 2>&1 || { tail -40 gpurun_out/r02h/updates.txt; exit 1; }
tail -3 gpurun_out/r02h/updates.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mirror.py \
  > gpurun_out/r02h/parity.txt 2>&1 || { tail -40 gpurun_out/r02h/parity.txt; exit 1; }
tail -3 gpurun_out/r02h/parity.txt
timeout -k 10 600 python3 -u scripts/update_perf.py 100 1000 10000 > gpurun_out/r02h/update_perf.jsonl 2> gpurun_out/r02h/update_perf.err \
  || { tail -20 gpurun_out/r02h/update_perf.err; exit 1; }
cat gpurun_out/r02h/update_perf.jsonl
