#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02e
bash scripts/ab_env.sh GM_NT=1 GM_MATCH_MAIN=fused,GM_NT=1 GM_MATCH_MAIN=fused GM_NT=1 GM_MATCH_MAIN=fused,GM_NT=1 2>&1 | tee gpurun_out/r02e/ab.txt || exit $?
LAT_MODE=device timeout -k 10 300 python3 -u scripts/host_latency.py 1000000 10000000 100000000 2>&1 | tee gpurun_out/r02e/lat_dev.jsonl || exit $?
timeout -k 10 300 python3 -u scripts/host_latency.py 2>&1 | tee gpurun_out/r02e/lat_both.jsonl || exit $?
GM_MATCH_MAIN=fused GM_NT=1 timeout -k 10 900 python3 -u -m pytest tests -v -s -m gpu -k "parity or sharded or scale" --timeout 600 --timeout-method thread > gpurun_out/r02e/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r02e/pytest.log | tail -15; exit $rc
