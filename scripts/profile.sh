#!/bin/bash
# rocprofv3 passes for a bench config (CONFIG, default c2; run on the GPU box).  Each PMC pass is its
# own run (no counter splitting), bounded by timeout -s KILL.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TOPICS=${TOPICS:-100000000}
CONFIG=${CONFIG:-c2}
OUT=gpurun_out/prof${PROF_TAG:-}
mkdir -p $OUT
ARGS="bench.py --config $CONFIG --topics $TOPICS --steps 2 --warmup 1 --no-cpu --no-parity --no-host-io --no-update ${BENCH_ARGS:-}"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -s KILL "$t" rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "ABORT"; exit $rc; fi
}
if [ "${1:-}" = "list" ]; then timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "listed rc=$?"; exit 0; fi
[ -z "${SKIP_STATS:-}" ] && run stats 300 --kernel-trace --stats
run pmc_fetch 120 --pmc FETCH_SIZE
run pmc_write 120 --pmc WRITE_SIZE
run pmc_l2 120 --pmc TCC_HIT_sum TCC_MISS_sum
run pmc_sq 120 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM
run pmc_ea 120 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
