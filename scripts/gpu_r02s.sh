#!/bin/bash
# C3 A/B: edge-filter L2 budget and table load (10M mixed filters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02s
BENCH_ARGS="--config c3 --no-host-io" bash scripts/ab_env.sh - GM_EFILT_MAX_KB=4096 GM_HOT_LOAD_PCT=30 GM_HOT_LOAD_PCT=20 2>&1 | tee gpurun_out/r02s/ab.txt
