#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02d
bash scripts/ab_env.sh - GM_NT=1 - GM_NT=1 2>&1 | tee gpurun_out/r02d/ab.txt || exit $?
timeout -k 10 400 python3 -u scripts/host_latency.py > gpurun_out/r02d/latency.jsonl 2> gpurun_out/r02d/latency.err || { tail -5 gpurun_out/r02d/latency.err; exit 1; }
cat gpurun_out/r02d/latency.jsonl
timeout -k 10 600 python3 -u -m pytest tests -v -s -m gpu -k "host_path or sharded or fanout or parity" --timeout 300 --timeout-method thread > gpurun_out/r02d/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r02d/pytest.log | tail -15; exit $rc
