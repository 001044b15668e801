#!/bin/bash
# Per-kernel device time of a bench configuration (rocprofv3 --kernel-trace
# --stats), printed as "kernel calls avg_ms".  usage: kstats.sh <tag> <bench args...>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/ks
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ks/$tag -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/ks/$tag.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/ks/$tag.log; exit 1; }
python3 - "$tag" <<'PY'
import csv, glob, sys, json
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/ks/{tag}/*kernel_stats.csv")[0]
print("==", tag)
for r in csv.DictReader(open(f)):
    print(f"  {r['Name'].split('(')[0][-36:]:36s} {r['Calls']:>4s} {float(r['AverageNs'])/1e6:9.3f} ms")
try:
    line = [l for l in open(f"gpurun_out/ks/{tag}.log") if l.startswith('{"metric"')][-1]
    d = json.loads(line)
    print("  value", round(d["value"] / 1e9, 3), "G/s; kernel_ms", round(d["roofline"]["kernel_ms"], 3))
except Exception as e:
    print("  (no bench line)", e)
PY
