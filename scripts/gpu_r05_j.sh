#!/bin/bash
# Round 5, GPU call j: one HIP runtime whatever the load order (the smoke
# failure of the suite run), smoke() in a fresh process, then the update A/B
# at C5 (100M filters).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread \
  -k "one_hip_runtime or graft_smoke or library_first" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
GM_UPDATE_TIMING=1 timeout -k 10 900 python3 -u scripts/update_c23.py --ab c5 > $O/update_ab.jsonl 2> $O/update_ab.err \
  || { tail -20 $O/update_ab.err; exit 1; }
cat $O/update_ab.jsonl
