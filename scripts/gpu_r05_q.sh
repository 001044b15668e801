#!/bin/bash
# Round 5, GPU call q: hot-table load factor and chain nodes at C3 on the shipped
# library (index knobs GM_HOT_LOAD_PCT, GM_CHAIN), same box, two rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_q
mkdir -p $O
ab() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu --no-parity --no-host-io \
    --no-update > $O/ab_$tag.log 2>&1 || { tail -5 $O/ab_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('c3 $tag', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel', round(d['value']/1e9,3), 'G/s')" | tee -a $O/ab.txt
}
for rep in 1 2; do
  ab load25_$rep GM_NONE=1
  ab load15_$rep GM_HOT_LOAD_PCT=15
  ab load35_$rep GM_HOT_LOAD_PCT=35
  ab load50_$rep GM_HOT_LOAD_PCT=50
  ab nochain_$rep GM_CHAIN=0
done
