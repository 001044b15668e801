#!/bin/bash
# Full bench lines for C3 and C1 under the current defaults + C3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02t
mkdir -p $O
timeout -k 10 700 python3 -u bench.py --config c3 --steps 5 --warmup 2 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
tail -n 1 $O/c3.json | cut -c1-400
bash scripts/kstats.sh r02t_c3 --config c3 --steps 3 --warmup 1 --no-cpu --no-parity --no-host-io > $O/c3_kstats.txt 2>&1 || { tail -5 $O/c3_kstats.txt; exit 1; }
tail -12 $O/c3_kstats.txt
timeout -k 10 300 python3 -u bench.py --config c1 --steps 20 --warmup 5 > $O/c1.json 2> $O/c1.err || { tail -5 $O/c1.err; exit 1; }
tail -n 1 $O/c1.json | cut -c1-400
