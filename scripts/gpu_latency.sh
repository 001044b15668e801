#!/bin/bash
# Per-call overhead: the GPU parity and shard tests, the C1 kernel trace (kernel
# + copy timeline), the host latency table, C1 and C2 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/latency
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -q -m gpu --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c1trace -o run --output-format csv -- python3 bench.py --config c1 --steps 5 --warmup 2 --no-cpu --no-parity --no-host-io --no-update > $O/c1trace.log 2>&1 || { tail -3 $O/c1trace.log; exit 1; }
timeout -k 10 300 python3 -u bench.py --config c1 --steps 20 --warmup 3 --no-cpu --no-host-io --no-update > $O/c1.log 2>&1 || { tail -3 $O/c1.log; exit 1; }
tail -1 $O/c1.log | cut -c1-400
timeout -k 10 300 python3 -u scripts/host_latency.py > $O/host_latency.jsonl 2>&1 || { tail -3 $O/host_latency.jsonl; exit 1; }
cat $O/host_latency.jsonl | tail -8
bash scripts/ab_env.sh - 2>&1 | tee $O/ab_c2.txt
