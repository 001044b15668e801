#!/bin/bash
# Round 5, GPU call c: the sharded / routing tests (SWAR device route, world-1
# aliasing), the spec-ids split-scan test, the two-rank C5 rehearsal (per-rank
# RSS); then the C5 prefix step at world 1 (1M filters, 100M topics) with a
# rocprofv3 kernel-stats pass, as profiles/r04_l measured it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out/r05_c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_sharded.py \
  tests/test_gpu_parity.py::test_no_speculative_ids_split_scan \
  tests/test_gpu_bench.py::test_bench_two_ranks_c5_replicated \
  tests/test_gpu_bench.py::test_bench_c5_prefix_one_gpu_device_path > $O/pytest.log 2>&1
rc=$?
tail -n 12 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py --config c5 --plan prefix --gpus 1 --filters 1000000 --topics 100000000 \
  --steps 3 --warmup 1 --no-cpu > $O/bench_prefix.log 2>&1 || { tail -5 $O/bench_prefix.log; exit 1; }
tail -c 700 $O/bench_prefix.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --config c5 --plan prefix \
  --gpus 1 --filters 1000000 --topics 100000000 --steps 3 --warmup 1 --no-cpu --no-parity > $O/prof.log 2>&1 \
  || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats_prefix.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05_c/kernel_stats_prefix.csv")))
for r in rows[:14]:
    print(f'{float(r["AverageNs"])/1e6:8.3f} ms x{r["Calls"]:>4}  {r["Name"][:90]}')
PY
