#!/bin/bash
# Round 5, GPU call p: item 2's gate, re-measured on the shipped library at C3:
# an exact-edge filter for the depth-3 table (the probes the saturated depth-2
# signatures let through) at 2 and 4 MB (GM_EFILT_MAX_KB) against none, on one
# box, two rounds each.  The index image is rebuilt per setting (the filter is
# part of the index).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_p
mkdir -p $O
ab() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu --no-parity --no-host-io \
    --no-update > $O/ab_$tag.log 2>&1 || { tail -5 $O/ab_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('c3 $tag', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel', round(d['value']/1e9,3), 'G/s')" | tee -a $O/ab.txt
}
for rep in 1 2; do
  ab default_$rep GM_NONE=1
  ab efilt2mb_$rep GM_EFILT_MAX_KB=2048 GM_EFILT_DIV=16
  ab efilt4mb_$rep GM_EFILT_MAX_KB=4096
done
