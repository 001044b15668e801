#!/bin/bash
# Round 6, GPU call z: emqx_gm_match_fanout (a publish window in one device
# round trip) -- parity and multi-device tests, then the A/B against the two calls.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${OUT:-r06_z}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_multi.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 -u scripts/publish_window_ab.py --reps 2 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
cat $O/ab.log
