#!/bin/bash
# Round-2 GPU check: the whole -m gpu suite (incl. the config-scale parity
# tests), the default bench line (C2) and the C4 bench.  Each GPU step has its
# own time limit; a fault / abort / time limit ends the script.
set -o pipefail
OUT=gpurun_out/${1:-r02a}
mkdir -p $OUT
{ nproc; python3 -c "import os;print('affinity', len(os.sched_getaffinity(0)))"; cat /proc/self/cgroup;
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | head -20; free -g; } > $OUT/probe.txt 2>&1
timeout -k 10 1000 python3 -u -m pytest tests -x -v -s -m gpu --timeout 900 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 200 python3 bench.py --config c4 --steps 10 --warmup 3 > $OUT/c4.json 2> $OUT/c4.err || exit $?
cat $OUT/c4.json
