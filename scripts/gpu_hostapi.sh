#!/bin/bash
# Host-side HIP API time per match call (C1 by default): a runtime + kernel trace of the
# bench, then the API calls of one call in order with their durations (scripts/hostapi.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/hostapi
mkdir -p $O
timeout -s KILL 300 rocprofv3 --hip-runtime-trace --kernel-trace -d $O/tr -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-parity --no-host-io --no-update ${BENCH_ARGS:---config c1} > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 scripts/hostapi.py $O/tr | tee $O/hostapi.txt
