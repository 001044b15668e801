#!/bin/bash
# Round 5, GPU call h2: same-box A/B of the final shipped library (parallel build,
# one-pass updates) against round 4's at C2.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_h2
mkdir -p $O
ab() {
  local cfg=$1 tag=$2; shift 2
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-parity --no-host-io \
    --no-update "$@" > $O/ab_${cfg}_$tag.log 2>&1 || { tail -5 $O/ab_${cfg}_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab_${cfg}_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg $tag', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel', round(d['value']/1e9,3), 'G/s')" | tee -a $O/ab.txt
}
for rep in 1 2 3; do
  EMQX_GM_LIB=emqx_amd/libemqx_gpu_match_r04.so ab c2 r04_$rep
  ab c2 r05_$rep
done
