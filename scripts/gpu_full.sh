#!/bin/bash
# Round measurement on the GPU box: rocprofv3 stats + PMC passes of the C2
# bench, traffic.json from the PMC passes, then the full bench line (CPU
# baseline, parity sample, PCIe-inclusive rate) and the C4 line; everything
# judged is collected under gpurun_out/profiles/<tag>/ (only gpurun_out/ comes
# back from the box; copy it to profiles/ there).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-r02}
P=gpurun_out/profiles/$TAG
mkdir -p gpurun_out profiles $P
bash scripts/profile.sh || exit $?
python3 scripts/traffic.py gpurun_out/prof > gpurun_out/traffic.log 2>&1 || { cat gpurun_out/traffic.log; exit 1; }
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -5 gpurun_out/bench_full.log; exit 1; }
tail -n 1 gpurun_out/bench_full.log
timeout -k 10 300 python3 -u bench.py --config c4 --steps 10 --warmup 3 > gpurun_out/bench_c4.log 2>&1 || { tail -5 gpurun_out/bench_c4.log; exit 1; }
tail -n 1 gpurun_out/bench_c4.log
cp gpurun_out/prof/stats/run_kernel_stats.csv $P/kernel_stats.csv
for f in gpurun_out/prof/*.log; do cp "$f" $P/; done
python3 scripts/pmc_summary.py gpurun_out/prof > $P/pmc_per_launch.json
cp profiles/traffic.json $P/traffic.json
tail -n 1 gpurun_out/bench_full.log > $P/bench.json
tail -n 1 gpurun_out/bench_c4.log > $P/bench_c4.json
