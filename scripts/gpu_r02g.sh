#!/bin/bash
# C3 and C5 (one shard = 1/8 of 100M filters) on one GPU with kernel stats, and
# a hot-table load-factor A/B at C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02g
bash scripts/ab_env.sh - GM_HOT_LOAD_PCT=30 GM_HOT_LOAD_PCT=25 GM_HOT_LOAD_PCT=35 GM_HOT_LOAD_PCT=30 2>&1 | tee gpurun_out/r02g/ab.txt || exit $?
timeout -k 10 600 python3 -u bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/r02g/c3.json 2> gpurun_out/r02g/c3.err || { tail -5 gpurun_out/r02g/c3.err; exit 1; }
tail -n 1 gpurun_out/r02g/c3.json
bash scripts/kstats.sh r02g_c3 --config c3 --steps 3 --warmup 1 --no-cpu --no-parity --no-host-io | tee gpurun_out/r02g/c3_kstats.txt || exit $?
timeout -k 10 900 python3 -u bench.py --config c5 --filters 12500000 --steps 5 --warmup 2 > gpurun_out/r02g/c5.json 2> gpurun_out/r02g/c5.err || { tail -5 gpurun_out/r02g/c5.err; exit 1; }
tail -n 1 gpurun_out/r02g/c5.json
