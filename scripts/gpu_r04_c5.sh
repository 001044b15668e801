#!/bin/bash
# Round 4: C5 (100M mixed filters, replicated index on one GPU).  The first
# bench run compiles the index (host RSS of the build in its line) and writes
# its image to /dev/shm; the rocprofv3 stats + PMC passes import it; then the
# bench line again from the image.  traffic_c5.json from the PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r04_v1}
P=gpurun_out/profiles/$TAG
mkdir -p $P
IMG=/dev/shm/gm_c5_$$.img
trap 'rm -f $IMG' EXIT
timeout -k 10 900 python3 -u bench.py --config c5 --index-cache $IMG --steps 5 --warmup 2 > gpurun_out/bench_c5_build.log 2>&1 || { tail -5 gpurun_out/bench_c5_build.log; exit 1; }
tail -n 1 gpurun_out/bench_c5_build.log > $P/bench_c5_build.json
ls -la $IMG
CONFIG=c5 PROF_TAG=_c5 BENCH_ARGS="--index-cache $IMG" bash scripts/profile.sh || exit $?
python3 scripts/traffic.py gpurun_out/prof_c5 --config c5 --out profiles/traffic_c5.json > gpurun_out/traffic_c5.log 2>&1 || { cat gpurun_out/traffic_c5.log; exit 1; }
cp profiles/traffic_c5.json $P/
cp gpurun_out/prof_c5/stats/run_kernel_stats.csv $P/kernel_stats_c5.csv
python3 scripts/pmc_summary.py gpurun_out/prof_c5 > $P/pmc_per_launch_c5.json
timeout -k 10 600 python3 -u bench.py --config c5 --index-cache $IMG > gpurun_out/bench_c5.log 2>&1 || { tail -5 gpurun_out/bench_c5.log; exit 1; }
tail -n 1 gpurun_out/bench_c5.log > $P/bench_c5.json
python3 -c "import json; d=json.load(open('$P/bench_c5.json')); r=d['roofline']; b=json.load(open('$P/bench_c5_build.json'))['detail']; print('c5', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel ms frac', round(r['frac'],3), 'traffic', r['traffic'], 'lines', r.get('lines_per_topic'), 'parity', d.get('parity_sample',{}).get('ok'), 'build_s', round(b['index_build_s'],1), 'rss_gb', round(b['host_peak_rss_gb'],1))"
