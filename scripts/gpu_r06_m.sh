#!/bin/bash
# Round 6, GPU call m: small host calls, concurrent path vs the serial one.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_m
mkdir -p $O
timeout -k 10 600 python3 -u scripts/small_calls_ab.py --devices 0 > $O/small_calls_ab.log 2>&1 || { tail -20 $O/small_calls_ab.log; exit 1; }
cat $O/small_calls_ab.log | grep devices
