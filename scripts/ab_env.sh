#!/bin/bash
# A/B of environment knobs at C2: one bench per argument ("-" = no knob,
# otherwise VAR=VALUE[,VAR=VALUE]), each under its own time limit.
# usage: ab_env.sh - GM_NO_EDGE_FILTER=1 ...   (BENCH_ARGS adds bench options)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
i=0
for spec in "$@"; do
  i=$((i + 1))
  envs=()
  [ "$spec" != "-" ] && IFS=',' read -r -a envs <<< "$spec"
  env "${envs[@]}" timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-parity ${BENCH_ARGS:-} > gpurun_out/ab/ab_$i.log 2>&1
  rc=$?
  echo "[$spec] rc=$rc $(tail -n 1 gpurun_out/ab/ab_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9, 3), 'Gtopics/s kernel_ms', round(d['roofline']['kernel_ms'], 3), 'probes', round(d['detail']['probes_per_topic'], 3), 'listed', d['detail']['overflow_rows'])" 2>&1)"
  [ $rc -ne 0 ] && { tail -n 5 gpurun_out/ab/ab_$i.log; exit $rc; }
done
exit 0
