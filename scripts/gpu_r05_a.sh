#!/bin/bash
# Round 5, GPU call a: the multi-device context (devices [0,0] rehearsal), the
# host-buffer pipeline (page-locked input, direct row copy-out), the C-ABI
# smoke with a two-device context; then a C2 bench line with the host-io detail.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05_a
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_multi.py \
  "tests/test_gpu_parity.py::test_c_abi_smoke_program" \
  "tests/test_gpu_parity.py::test_host_path_chunks_equal_device_path" \
  "tests/test_gpu_parity.py::test_host_path_rejects_bad_offsets_and_survives" \
  "tests/test_gpu_parity.py::test_host_csr_ownership_across_contexts" \
  "tests/test_gpu_parity.py::test_broker_incremental_snapshots" \
  "tests/test_gpu_parity.py::test_concurrent_calls_one_context" \
  > gpurun_out/r05_a/pytest.log 2>&1
rc=$?
tail -n 30 gpurun_out/r05_a/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r05_a/bench_c2.log 2>&1
rc=$?
tail -c 3000 gpurun_out/r05_a/bench_c2.log
exit $rc
