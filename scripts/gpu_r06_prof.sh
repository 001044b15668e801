#!/bin/bash
# Round 6 final profiles on the final library: rocprofv3 --kernel-trace --stats
# and the PMC passes (scripts/profile.sh) of one config, then its traffic file
# (scripts/traffic.py: the library's hash stamped, so bench.py reports it as
# roofline.traffic) -> profiles/$TAG.  CONFIGS: the configs, in order.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06_final}
P=gpurun_out/profiles/$TAG
mkdir -p $P
for cfg in ${CONFIGS:-c2 c3}; do
  case $cfg in
    c2) extra=""; out=profiles/traffic.json ;;
    *) extra="--index-cache /dev/shm/gm_${cfg}_$$.img"; out=profiles/traffic_$cfg.json ;;
  esac
  CONFIG=$cfg PROF_TAG=_$cfg BENCH_ARGS="$extra" bash scripts/profile.sh || { rm -f /dev/shm/gm_${cfg}_$$.img; exit 1; }
  rm -f /dev/shm/gm_${cfg}_$$.img
  python3 scripts/traffic.py gpurun_out/prof_$cfg --config $cfg --out $out > gpurun_out/traffic_$cfg.log 2>&1 || { cat gpurun_out/traffic_$cfg.log; exit 1; }
  cp $out $P/
  cp gpurun_out/prof_$cfg/stats/run_kernel_stats.csv $P/kernel_stats_$cfg.csv
  for f in gpurun_out/prof_$cfg/*.log; do cp "$f" $P/${cfg}_$(basename $f); done
  python3 scripts/pmc_summary.py gpurun_out/prof_$cfg > $P/pmc_per_launch_$cfg.json
  head -3 $P/kernel_stats_$cfg.csv
done
