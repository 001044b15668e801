#!/bin/bash
# Round 6, GPU call u: device timelines of small host fan-outs, both paths.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${OUT:-r06_u}
mkdir -p $O
for mode in ${MODES:-small locked}; do
  if [ $mode = locked ]; then export EMQX_GM_AB=1 GM_FANOUT_SIMPLE=1; else unset GM_FANOUT_SIMPLE; fi
  timeout -k 10 300 python3 -u scripts/small_fanout_probe.py 100 16384 > $O/plain_$mode.log 2>&1 || { tail -5 $O/plain_$mode.log; exit 1; }
  tail -1 $O/plain_$mode.log
  timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_$mode -o run --output-format csv -- python3 scripts/small_fanout_probe.py 100 16384 > $O/trace_$mode.log 2>&1 || { tail -5 $O/trace_$mode.log; exit 1; }
  grep "fan-outs of" $O/trace_$mode.log
done
