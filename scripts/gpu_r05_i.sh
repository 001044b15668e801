#!/bin/bash
# Round 5, GPU call i: the one-pass device update (k_renumber_copy) -- the
# update tests (both device forms, and their blobs byte for byte), then the
# A/B of the two forms on one index chain at C3 (10M filters) and C5 (100M).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_i
mkdir -p $O
for m in lib_first torch_first ctx_first; do
  timeout -k 10 120 python3 -u scripts/smoke_order_diag.py $m >> $O/smoke_diag.txt 2>&1 || echo "$m rc=$?" >> $O/smoke_diag.txt
done
cat $O/smoke_diag.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_updates.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
GM_UPDATE_TIMING=1 timeout -k 10 900 python3 -u scripts/update_c23.py --ab c3 c5 > $O/update_ab.jsonl 2> $O/update_ab.err \
  || { tail -20 $O/update_ab.err; exit 1; }
cat $O/update_ab.jsonl
