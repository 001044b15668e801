#!/bin/bash
# One GPU call: optional probe, A/B of env knobs at C2 (scripts/ab_env.sh), the
# kernel stats of the default build, then the -m gpu suite.
# usage: gpu_ab.sh <tag> "<ab specs>" [pytest -k filter|-]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; SPECS=$2; K=${3:-}
mkdir -p gpurun_out/$TAG
if [ -n "${PROBE:-}" ]; then timeout -k 10 300 python3 scripts/probe_torch_hip.py 2>&1 | tee gpurun_out/$TAG/probe.txt; fi
if [ -n "$SPECS" ]; then bash scripts/ab_env.sh $SPECS 2>&1 | tee gpurun_out/$TAG/ab.txt || exit $?; fi
if [ -n "${KSTATS:-}" ]; then bash scripts/kstats.sh $TAG --steps 3 --warmup 1 --no-cpu --no-parity 2>&1 | tee gpurun_out/$TAG/kstats.txt || exit $?; fi
if [ "$K" != "-" ]; then
  timeout -k 10 1100 python3 -u -m pytest tests -v -s -m gpu ${K:+-k "$K"} --timeout 900 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
  rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/$TAG/pytest.log | tail -15; exit $rc
fi
