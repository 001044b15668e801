#!/bin/bash
# Experiment: index memory type (GM_INDEX_MEM) vs match-kernel time and L2/EA traffic.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/mem
for m in ${MODES:-default aux0 aux2 aux1 aux17 aux3}; do
  if [ "$m" = default ]; then unset EMQX_GM_LIB; else export EMQX_GM_LIB=$PWD/emqx_amd/libemqx_gpu_match_$m.so; fi
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu --topics 20000000 > gpurun_out/mem/b_$m.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/mem/b_$m.log; exit 1; }
  tail -n 1 gpurun_out/mem/b_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value']/1e9, 'Gtopics/s kernel_ms', d['roofline']['kernel_ms'])"
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/mem/p_$m -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --topics 20000000 > gpurun_out/mem/p_$m.log 2>&1 || { echo "pmc $m failed"; tail -5 gpurun_out/mem/p_$m.log; exit 1; }
  python3 - "$m" <<'PY'
import csv, glob, sys, collections
m = sys.argv[1]
f = glob.glob(f"gpurun_out/mem/p_{m}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    if "k_walk" not in k and "k_tokenize" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(m, k[-30:], {c: round(v / n[(k, c)] / 20e6, 3) for c, v in d.items()}, "(per topic)")
PY
done
