#!/bin/bash
# Round measurement on the GPU box: rocprofv3 stats + PMC passes of the C2
# bench, traffic.json from the PMC passes, then the full bench line (CPU
# baseline + PCIe-inclusive rate).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash scripts/profile.sh || exit $?
python3 scripts/traffic.py gpurun_out/prof > gpurun_out/traffic.log 2>&1 || { cat gpurun_out/traffic.log; exit 1; }
cp profiles/traffic.json gpurun_out/traffic.json
timeout -k 10 600 python -u bench.py --host-io > gpurun_out/bench_full.log 2>&1 || { tail -5 gpurun_out/bench_full.log; exit 1; }
tail -n 1 gpurun_out/bench_full.log
