#!/bin/bash
# Diagnostics on the GPU box: phase-timing and probe-census runs of the given
# configs ($CFGS, default "c2 c3") with and without chain nodes; each run under
# its own time limit, output in gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${TAG:-phase}
mkdir -p $OUT
for cfg in ${CFGS:-c2 c3}; do
  for spec in ${SPECS:-- GM_NO_CHAIN=1}; do
    envs=(); [ "$spec" != "-" ] && envs=("$spec")
    for kind in ${KINDS:-phase census}; do
      env "${envs[@]}" EMQX_GM_LIB=emqx_amd/libemqx_gpu_match_$kind.so timeout -k 10 300 python3 -u scripts/phase_stats.py $cfg ${N:-20000000} \
        > $OUT/${kind}_${cfg}_${spec}.log 2>&1
      rc=$?
      echo "[$cfg $spec $kind] rc=$rc"; grep -E "phase_stats|probe_stats" $OUT/${kind}_${cfg}_${spec}.log | tail -n 6
      [ $rc -ne 0 ] && { tail -n 5 $OUT/${kind}_${cfg}_${spec}.log; exit $rc; }
    done
  done
done
exit 0
