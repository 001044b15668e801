#!/bin/bash
# Round 6 A/B: the C5 index blob from a contiguous allocation (GM_BLOB_CONTIG)
# against plain hipMalloc, same box, kernel time of the bench line.  (The knob
# lived in gm_index.cpp for this A/B only; no difference, so it was removed.)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp EMQX_GM_AB=1
O=gpurun_out/r06_contig
mkdir -p $O
for arm in plain contig plain contig; do
  if [ $arm = contig ]; then export GM_BLOB_CONTIG=1; else unset GM_BLOB_CONTIG; fi
  timeout -k 10 400 python3 -u bench.py --config c5 --no-update --no-host-io --no-multi --no-cpu --no-parity --steps 5 --warmup 2 > $O/$arm.log 2>&1 || { tail -5 $O/$arm.log; exit 1; }
  tail -n 1 $O/$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value']/1e9, d['ms_per_step'], d['roofline'].get('kernel_ms'))" | tee -a $O/ab.txt
done
