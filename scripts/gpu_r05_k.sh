#!/bin/bash
# Round 5, GPU call k: the spare blob (a freed snapshot's device tables reused
# by the next update) -- update / image / multi-device tests, then ten C5
# updates in a row (one-pass and unfused alternating).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_k
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_updates.py tests/test_gpu_image.py tests/test_gpu_multi.py -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
GM_UPDATE_TIMING=1 timeout -k 10 900 python3 -u scripts/update_c23.py --ab c5 > $O/update_ab.jsonl 2> $O/update_ab.err \
  || { tail -20 $O/update_ab.err; exit 1; }
cat $O/update_ab.jsonl
