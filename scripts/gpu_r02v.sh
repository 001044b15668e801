#!/bin/bash
# Paired exact probe: parity suite, then A/B at C2 and C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02v
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_updates.py > gpurun_out/r02v/parity.txt 2>&1 || { tail -30 gpurun_out/r02v/parity.txt; exit 1; }
tail -2 gpurun_out/r02v/parity.txt
BENCH_ARGS="--no-host-io" bash scripts/ab_env.sh - GM_PAIR_PROBE=0 - GM_PAIR_PROBE=0 2>&1 | tee gpurun_out/r02v/ab_c2.txt || exit 1
BENCH_ARGS="--config c3 --no-host-io" bash scripts/ab_env.sh - GM_PAIR_PROBE=0 2>&1 | tee gpurun_out/r02v/ab_c3.txt
