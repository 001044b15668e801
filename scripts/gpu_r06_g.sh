#!/bin/bash
# Round 6, GPU call g: the sharded index behind the C ABI, the multi-device
# tests, and the bench's two-rank test (N>1 multi-device block in a child).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_g
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_multi.py tests/test_gpu_bench.py::test_bench_two_ranks_c2 \
  -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
