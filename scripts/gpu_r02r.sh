#!/bin/bash
# C3 and C5 (one 12.5M-filter shard) bench lines + C3 kernel stats, and the
# host latency table, under the current defaults.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 700 python3 -u bench.py --config c3 --steps 5 --warmup 2 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
tail -n 1 $O/c3.json
bash scripts/kstats.sh r02r_c3 --config c3 --steps 3 --warmup 1 --no-cpu --no-parity --no-host-io > $O/c3_kstats.txt 2>&1 || { tail -5 $O/c3_kstats.txt; exit 1; }
cat $O/c3_kstats.txt | tail -12
timeout -k 10 900 python3 -u bench.py --config c5 --filters 12500000 --steps 5 --warmup 2 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
tail -n 1 $O/c5.json
timeout -k 10 600 python3 -u scripts/host_latency.py > $O/latency.jsonl 2> $O/latency.err || { tail -5 $O/latency.err; exit 1; }
cat $O/latency.jsonl
