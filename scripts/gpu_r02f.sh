#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02f
bash scripts/ab_env.sh - GM_HOT_LOAD_PCT_UPPER=80 GM_HOT_LOAD_PCT=55 GM_HOT_LOAD_PCT=30 GM_EFILT_ALL=1 2>&1 | tee gpurun_out/r02f/ab.txt || exit $?
bash scripts/gpu_full.sh r02_v1
