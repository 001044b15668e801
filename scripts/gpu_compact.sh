#!/bin/bash
# Compact staging (GM_STAGE_COMPACT): parity, then C2 / C3 A/B and a kernel-stats pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/compact
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -q -m gpu --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/ab_env.sh - GM_STAGE_COMPACT=0 - GM_STAGE_COMPACT=0 2>&1 | tee $O/ab_c2.txt || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-host-io --no-update > $O/stats.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/compact/stats/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3))
PY
