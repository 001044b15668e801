#!/bin/bash
# CW_CAP A/B: 236 (default build) vs 192 (emqx_amd/libemqx_gpu_match_cap192.so), C2 then C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02j
L192=EMQX_GM_LIB=$PWD/emqx_amd/libemqx_gpu_match_cap192.so
BENCH_ARGS="--no-host-io" bash scripts/ab_env.sh - $L192 - $L192 2>&1 | tee gpurun_out/r02j/c2.txt || exit $?
BENCH_ARGS="--config c3 --no-host-io" bash scripts/ab_env.sh - $L192 2>&1 | tee gpurun_out/r02j/c3.txt || exit $?
