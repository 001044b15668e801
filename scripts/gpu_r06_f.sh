#!/bin/bash
# Round 6, GPU call f: same-box A/B at C2 of the round-5 library (EMQX_GM_LIB,
# its knobs read ungated, load 0.25), this round's library as shipped (knobs
# gated, load 0.15) and this round's library at the old load (EMQX_GM_AB=1
# GM_HOT_LOAD_PCT=25: the gate itself costs nothing); then the hot-table load
# 0.10 against 0.15 at C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_f
mkdir -p $O
ab() {
  local cfg=$1 tag=$2; shift 2
  env "$@" timeout -k 10 600 python3 -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-parity --no-host-io \
    --no-update --no-multi $EXTRA > $O/ab_${cfg}_$tag.log 2>&1 || { tail -5 $O/ab_${cfg}_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab_${cfg}_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg $tag', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel', round(d['value']/1e9,3), 'G/s', 'dev GB', round(d['detail']['index_device_bytes']/1e9,2))" | tee -a $O/ab.txt
}
EXTRA=""
for rep in 1 2; do
  ab c2 r05lib_$rep EMQX_GM_LIB=emqx_amd/libemqx_gpu_match_r05.so
  ab c2 r06lib_$rep GM_NONE=1
  ab c2 r06lib_load25_$rep EMQX_GM_AB=1 GM_HOT_LOAD_PCT=25
done
EXTRA="--index-cache /dev/shm/gm_c3_l15_$$.img"
for rep in 1 2; do
  ab c3 load15_$rep GM_NONE=1
done
rm -f /dev/shm/gm_c3_l15_$$.img
EXTRA="--index-cache /dev/shm/gm_c3_l10_$$.img"
for rep in 1 2; do
  ab c3 load10_$rep EMQX_GM_AB=1 GM_HOT_LOAD_PCT=10
done
rm -f /dev/shm/gm_c3_l10_$$.img
