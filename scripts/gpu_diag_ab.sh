#!/bin/bash
# Diagnostic A/B of library builds on the GPU box: for each kind in $KINDS
# (emqx_amd/libemqx_gpu_match_<kind>.so; "product" = the product library), a
# phase_stats run (phase-timing builds only) and a short C2 bench (no parity:
# diagnostic builds may compute wrong rows), each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${TAG:-diag}
mkdir -p $OUT
for cfg in ${CFGS:-c2}; do
  for kind in ${KINDS:-phase nostore}; do
    lib=emqx_amd/libemqx_gpu_match_$kind.so; [ $kind = product ] && lib=emqx_amd/libemqx_gpu_match.so
    if [ $kind = phase ]; then
      EMQX_GM_LIB=$lib timeout -k 10 300 python3 -u scripts/phase_stats.py $cfg ${N:-20000000} > $OUT/phase_${cfg}_$kind.log 2>&1
      rc=$?; echo "[$cfg $kind phase] rc=$rc"; grep phase_stats $OUT/phase_${cfg}_$kind.log | tail -n 1
      [ $rc -ne 0 ] && { tail -n 5 $OUT/phase_${cfg}_$kind.log; exit $rc; }
    fi
    EMQX_GM_LIB=$lib timeout -k 10 400 python3 -u bench.py --config $cfg --steps ${STEPS:-5} --warmup ${WARM:-2} --no-cpu --no-parity --no-host-io \
      --no-update > $OUT/bench_${cfg}_$kind.log 2>&1
    rc=$?
    echo "[$cfg $kind bench] rc=$rc $(tail -n 1 $OUT/bench_${cfg}_$kind.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9, 3), 'Gtopics/s kernel_ms', round(d['roofline']['kernel_ms'], 3))" 2>&1)"
    [ $rc -ne 0 ] && { tail -n 5 $OUT/bench_${cfg}_$kind.log; exit $rc; }
  done
done
exit 0
