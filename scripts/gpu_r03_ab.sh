#!/bin/bash
# Round-3 A/B driver on the GPU box: optional pytest subset ($TESTS: a -k
# expression, or "all"), then bench A/B specs for C2 ($AB) and C3 ($AB3), then
# the TCC_EA0_RDREQ pass of each C2 spec ($PMC=1).  Every GPU step has its own
# time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  K=(); [ "$TESTS" != "all" ] && K=(-k "$TESTS")
  timeout -k 10 ${TEST_LIMIT:-900} python3 -u -m pytest tests -v -m gpu "${K[@]}" --timeout 600 --timeout-method thread \
    > $OUT/pytest.log 2>&1
  rc=$?; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest.log | tail -n 30
  [ $rc -ne 0 ] && exit $rc
fi
ab() {  # ab <config> <spec...>
  local cfg=$1; shift
  local i=0
  for spec in "$@"; do
    i=$((i + 1))
    envs=(); [ "$spec" != "-" ] && IFS=',' read -r -a envs <<< "$spec"
    env "${envs[@]}" timeout -k 10 400 python3 -u bench.py --config $cfg --steps ${STEPS:-5} --warmup ${WARM:-2} --no-cpu --no-parity \
      --no-host-io --no-update > $OUT/ab_${cfg}_$i.log 2>&1
    rc=$?
    echo "[$cfg $spec] rc=$rc $(tail -n 1 $OUT/ab_${cfg}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9, 3), 'Gtopics/s ms/step', round(d['ms_per_step'], 3), 'kernel_ms', round(d['roofline']['kernel_ms'], 3), 'listed', d['detail']['overflow_rows'])" 2>&1)"
    [ $rc -ne 0 ] && { tail -n 5 $OUT/ab_${cfg}_$i.log; exit $rc; }
  done
}
[ -n "${AB1:-}" ] && STEPS=200 ab c1 $AB1
[ -n "${AB:-}" ] && ab c2 $AB
[ -n "${AB3:-}" ] && ab c3 $AB3
if [ -n "${PMC:-}" ]; then
  i=0
  for spec in ${AB:--}; do
    i=$((i + 1))
    envs=(); [ "$spec" != "-" ] && IFS=',' read -r -a envs <<< "$spec"
    for e in "${envs[@]}"; do export "$e"; done
    timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_$i -o run --output-format csv \
      -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-parity --no-host-io --no-update > $OUT/pmc_$i.log 2>&1
    rc=$?
    for e in "${envs[@]}"; do unset "${e%%=*}"; done
    echo "[pmc $spec] rc=$rc"
    [ $rc -ne 0 ] && { tail -n 5 $OUT/pmc_$i.log; exit $rc; }
    python3 scripts/pmc_lines.py $OUT/pmc_$i || true
  done
fi
exit 0
