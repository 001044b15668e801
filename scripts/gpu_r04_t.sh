#!/bin/bash
# Round 4 A/B at C3: an exact-edge filter for the 7.4M-key depth-3 table past
# the 1 MB L2 budget (GM_EFILT_MAX_KB), against its 0.94 failed probes per topic.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_t
mkdir -p $O
run() {  # run <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config c3 --steps 6 --warmup 2 --no-cpu --no-parity --no-host-io --no-update \
    > $O/b_$lab.log 2>&1 || { tail -5 $O/b_$lab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$lab.log').read().strip().splitlines()[-1]); print('c3 $lab', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'kernel ms')" | tee -a $O/efilt_c3.txt
}
run base GM_X=0
run efilt2m GM_EFILT_MAX_KB=2048
run efilt4m GM_EFILT_MAX_KB=4096
run efilt4m_d16 GM_EFILT_MAX_KB=4096 GM_EFILT_DIV=16
run base2 GM_X=0
