#!/bin/bash
# Exact-edge filter density sweep at C2 (bits per key ~ 32/DIV..64/DIV), and filters on every table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02p
BENCH_ARGS="--no-host-io" bash scripts/ab_env.sh GM_EFILT_DIV=8 GM_EFILT_DIV=16 GM_EFILT_DIV=32 GM_EFILT_DIV=64 GM_EFILT_ALL=1,GM_EFILT_DIV=8 GM_EFILT_ALL=1,GM_EFILT_DIV=16 GM_EFILT_ALL=1,GM_EFILT_DIV=32 GM_NO_EDGE_FILTER=1 GM_EFILT_DIV=8 2>&1 | tee gpurun_out/r02p/ab.txt
