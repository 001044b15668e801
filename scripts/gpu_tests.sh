#!/bin/bash
# The -m gpu suite alone (progress on stdout via -s), optional -k filter in $2.
set -o pipefail
OUT=gpurun_out/${1:-tests}
mkdir -p $OUT
K=${2:-}
timeout -k 10 1100 python3 -u -m pytest tests -v -s -m gpu ${K:+-k "$K"} --timeout 900 --timeout-method thread 2>&1 | tee $OUT/pytest.log | grep -E "PASSED|FAILED|ERROR|scale|passed|failed"
