#!/bin/bash
# Where the prefix plan's 100M-topic step goes at world 1: rocprofv3 kernel
# stats of bench.py --plan prefix (1M filters so the build is short).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out/r04_h
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --config c5 --plan prefix --filters 1000000 --topics 100000000 --steps 3 --warmup 1 --no-cpu --no-parity > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log | tail -n 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04_h/kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):5d} calls  {r["Name"][:110]}')
PY
