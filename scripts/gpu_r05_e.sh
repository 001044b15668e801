#!/bin/bash
# Round 5, GPU call e: the prefix plan after the world-1 aliasing and the
# wave-aggregated shard counts: its tests, then the C5 prefix step at world 1
# (1M filters, 100M topics) and its rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out/r05_e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_sharded.py -k "route or prefix or permute" \
  tests/test_gpu_bench.py::test_bench_c5_prefix_one_gpu_device_path \
  tests/test_gpu_bench.py::test_bench_two_ranks_c5_prefix > $O/pytest.log 2>&1
rc=$?
tail -n 8 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py --config c5 --plan prefix --gpus 1 --filters 1000000 --topics 100000000 \
  --steps 5 --warmup 1 --no-cpu > $O/bench_prefix.log 2>&1 || { tail -5 $O/bench_prefix.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench_prefix.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py \
  --config c5 --plan prefix --gpus 1 --filters 1000000 --topics 100000000 --steps 3 --warmup 1 --no-cpu --no-parity \
  > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats_prefix.csv
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/r05_e/kernel_stats_prefix.csv")))[:10]:
    print(f'{float(r["AverageNs"])/1e6:8.3f} ms x{r["Calls"]:>4}  {r["Name"][:100]}')
PY
