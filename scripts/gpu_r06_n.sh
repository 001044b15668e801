#!/bin/bash
# Round 6, GPU call n: a device timeline of one caller's small host calls.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${OUT:-r06_n}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/small_call_probe.py 200 1024 > $O/plain.log 2>&1 || { tail -5 $O/plain.log; exit 1; }
tail -1 $O/plain.log
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/small_call_probe.py 200 1024 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
grep "calls of" $O/trace.log
ls $O/trace
