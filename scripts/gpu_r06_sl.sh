#!/bin/bash
# Round 6: the one-launch looped scan for small fan-outs -- parity, multi-device,
# then the publish-window probe and both small-path A/Bs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${OUT:-r06_sl}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_multi.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -u scripts/publish_window_probe.py 200 1024 > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
tail -1 $O/probe.log
timeout -k 10 400 python3 -u scripts/publish_window_ab.py --reps 2 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 400 python3 -u scripts/small_fanout_ab.py --reps 2 > $O/fanout_ab.log 2>&1 || { tail -5 $O/fanout_ab.log; exit 1; }
cat $O/fanout_ab.log
