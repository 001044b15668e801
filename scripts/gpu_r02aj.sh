#!/bin/bash
# Depth-1/2 table load A/B at C2 (t2 = 8.5 MB at the default 0.25).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02aj
BENCH_ARGS="--no-host-io --no-update" bash scripts/ab_env.sh - GM_HOT_LOAD_PCT_UPPER=15 GM_HOT_LOAD_PCT_UPPER=20 GM_HOT_LOAD_PCT_UPPER=35 - GM_HOT_LOAD_PCT_UPPER=15 2>&1 | tee gpurun_out/r02aj/ab.txt
