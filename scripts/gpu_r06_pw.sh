#!/bin/bash
# Round 6: a device timeline of one caller's publish windows (emqx_gm_match_fanout).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${OUT:-r06_pw}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/publish_window_probe.py 200 1024 > $O/plain.log 2>&1 || { tail -5 $O/plain.log; exit 1; }
tail -1 $O/plain.log
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/publish_window_probe.py 200 1024 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
grep "publish windows" $O/trace.log
