#!/bin/bash
# Round 6, GPU call a: the topic-grouping A/B (scripts/grouping_ab.py) at C3
# and C5, and the hot-table load A/B at C5 (0.25 vs 0.15), on the round-5
# library; same box, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 EMQX_GM_AB=1
O=gpurun_out/r06_a
mkdir -p $O
timeout -k 10 900 python3 -u scripts/grouping_ab.py --config c3 --rounds 3 --index-cache /dev/shm/gm_c3_$$.img > $O/grouping_c3.log 2>&1 || { tail -5 $O/grouping_c3.log; rm -f /dev/shm/gm_c3_$$.img; exit 1; }
rm -f /dev/shm/gm_c3_$$.img
tail -1 $O/grouping_c3.log
timeout -k 10 900 python3 -u scripts/grouping_ab.py --config c5 --rounds 3 > $O/grouping_c5.log 2>&1 || { tail -5 $O/grouping_c5.log; exit 1; }
tail -1 $O/grouping_c5.log
ab() {
  local tag=$1; shift
  env "$@" timeout -k 10 600 python3 -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu --no-parity --no-host-io \
    --no-update --no-host-replicas > $O/ab_$tag.log 2>&1 || { tail -5 $O/ab_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('c5 $tag', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel', round(d['value']/1e9,3), 'G/s', 'dev GB', round(d.get('detail',{}).get('index_device_bytes',0)/1e9,2))" | tee -a $O/ab.txt
}
for rep in 1 2; do
  ab load25_$rep GM_NONE=1
  ab load15_$rep GM_HOT_LOAD_PCT=15
done
