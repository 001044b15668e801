#!/bin/bash
# Round 5, GPU call e: the hot-word cache (IndexView::hot_dict, LDS in the
# tokenizer phase) and the prefix-plan changes: parity tests (tokenizer /
# edge / random / config-scale subsample / images / multi-device / routing),
# the prefix step at world 1, then same-box A/Bs of the cache (GM_HDICT_CALL=0
# vs on) at C2 and C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out/r05_e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_parity.py -k "tokenizer or edge or random_small or hash_collision or deep or config_subsample or suite or c1_fixture or speculative or compact or chain" \
  tests/test_gpu_image.py tests/test_gpu_multi.py \
  tests/test_gpu_sharded.py -k "tokenizer or edge or random_small or hash_collision or deep or config_subsample or suite or c1_fixture or speculative or compact or chain or route or prefix or permute or image or multi or replica or update or devices or concurrent" \
  > $O/pytest.log 2>&1
rc=$?
tail -n 6 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py --config c5 --plan prefix --gpus 1 --filters 1000000 --topics 100000000 \
  --steps 5 --warmup 1 --no-cpu > $O/bench_prefix.log 2>&1 || { tail -5 $O/bench_prefix.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench_prefix.log
ab() {  # ab <config> <tag> <extra args...>
  local cfg=$1 tag=$2; shift 2
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu --no-parity --no-host-io \
    --no-update "$@" > $O/ab_${cfg}_$tag.log 2>&1 || { tail -5 $O/ab_${cfg}_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab_${cfg}_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg $tag', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel', round(r['kernel_ms_median'],3), 'median', round(d['value']/1e9,3), 'G/s')" | tee -a $O/ab.txt
}
for rep in 1 2; do
  GM_HDICT_CALL=0 ab c2 off$rep
  ab c2 on$rep
done
GM_HDICT_CALL=0 ab c3 off1 --index-cache /dev/shm/gm_c3_e.img
ab c3 on1 --index-cache /dev/shm/gm_c3_e.img
GM_HDICT_CALL=0 ab c3 off2 --index-cache /dev/shm/gm_c3_e.img
ab c3 on2 --index-cache /dev/shm/gm_c3_e.img
rm -f /dev/shm/gm_c3_e.img
