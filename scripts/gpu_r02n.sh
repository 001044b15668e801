#!/bin/bash
# L2 working-set A/B at C2: depth-1/2 hot-table load (t2 = 7 MB at 0.30) and the
# depth-3 exact-edge filter density.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02n
BENCH_ARGS="--no-host-io" bash scripts/ab_env.sh - GM_HOT_LOAD_PCT_UPPER=50 GM_HOT_LOAD_PCT_UPPER=60 GM_EFILT_DIV=4 GM_EFILT_DIV=8 GM_EFILT_DIV=1 - GM_HOT_LOAD_PCT_UPPER=60,GM_EFILT_DIV=4 2>&1 | tee gpurun_out/r02n/ab.txt
