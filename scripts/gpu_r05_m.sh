#!/bin/bash
# Round 5, GPU call m: the chunked prefix step (world 8 in lock step, chunked
# and unchunked) and the rest of the sharded tests.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_m
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 600 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
