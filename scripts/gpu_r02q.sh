#!/bin/bash
# Hot-table load A/B at C2 with the 4-8 bit/key exact-edge filter.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02q
BENCH_ARGS="--no-host-io" bash scripts/ab_env.sh GM_HOT_LOAD_PCT=25 GM_HOT_LOAD_PCT=20 GM_HOT_LOAD_PCT=15 GM_HOT_LOAD_PCT=10 GM_HOT_LOAD_PCT=20,GM_HOT_LOAD_PCT_UPPER=30 GM_HOT_LOAD_PCT=20 2>&1 | tee gpurun_out/r02q/ab2.txt
