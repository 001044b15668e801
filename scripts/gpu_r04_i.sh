#!/bin/bash
# Round 4: the prefix plan's new copy kernel (k_gather_segs) and torch-side
# split sizes: the sharded/bench tests, then the 100M-topic prefix step
# profiled again (profiles/r04_i).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_i}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_bench.py -x -v --timeout 400 --timeout-method thread -k "permute or prefix or c5" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --config c5 --plan prefix --filters 1000000 --topics 100000000 --steps 3 --warmup 1 --no-cpu > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log | tail -n 1 > $O/bench_prefix_1m_100m.json
cat $O/bench_prefix_1m_100m.json | cut -c1-600
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
O=$O python3 - <<'PY'
import csv, os
rows = list(csv.DictReader(open(os.environ["O"] + "/kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):5d} calls  {r["Name"][:100]}')
PY
