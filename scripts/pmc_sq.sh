#!/bin/bash
# One SQ-counter pass (<= 8 SQ_ counters) over a short C2 bench; per-kernel
# averages per launch.  usage: pmc_sq.sh <tag> [counters...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; shift
C=${*:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM}
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc/$tag -o run --output-format csv -- python3 bench.py --topics 20000000 --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc/$tag.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc/$tag.log; exit 1; }
python3 - "$tag" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/pmc/{tag}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    if not any(x in k for x in ("k_walk", "k_tokenize", "k_assemble")): continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    w = d.get("SQ_WAVES", 0) / max(1, n[(k, "SQ_WAVES")])
    print(k[-28:], {c: round(v / n[(k, c)] / max(w, 1), 1) for c, v in d.items()}, "(per wave)")
PY
