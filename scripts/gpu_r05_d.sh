#!/bin/bash
# Round 5, GPU call d: rocprofv3 kernel stats of the C5 prefix step at world 1
# (1M filters, 100M topics), then a C3 bench line (10M filters) carrying the
# subscriber-update (O(delta)) and host-io details.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out/r05_d
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py \
  --config c5 --plan prefix --gpus 1 --filters 1000000 --topics 100000000 --steps 3 --warmup 1 --no-cpu --no-parity \
  > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats_prefix.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05_d/kernel_stats_prefix.csv")))
for r in rows[:16]:
    print(f'{float(r["AverageNs"])/1e6:8.3f} ms x{r["Calls"]:>4}  {r["Name"][:100]}')
PY
timeout -k 10 900 python3 -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu > $O/bench_c3.log 2>&1 \
  || { tail -5 $O/bench_c3.log; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/r05_d/bench_c3.log').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value'] / 1e9, d['parity_sample']['ok'])
print({k: v for k, v in d['detail'].items() if k.startswith(('host_io', 'subs', 'index_update'))})
"
