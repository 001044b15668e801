#!/bin/bash
# C2 per-call timeline: kernel + memory-copy trace of 5 timed calls, then the idle gap
# between one call's last kernel and the next call's first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/gaps
mkdir -p $O
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tr -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-parity --no-host-io --no-update ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
python3 scripts/gaps.py $O/tr | tee $O/gaps.txt
