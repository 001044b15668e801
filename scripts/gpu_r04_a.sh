#!/bin/bash
# Round 4, first GPU call: the new device-path tests (prefix matcher on device
# tensors at world 1 and 8-rank lock step, the bench's 1-GPU prefix path, the
# hash matcher's replayed exchange) and the full-size C4 check.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r04_a
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_sharded.py::test_prefix_device_path_world1 \
  tests/test_gpu_sharded.py::test_device_tensor_path_with_replayed_exchange \
  tests/test_gpu_bench.py::test_bench_c5_prefix_one_gpu_device_path \
  tests/test_gpu_sharded.py::test_prefix_device_path_world8_lockstep \
  tests/test_gpu_scale.py::test_c4_full_fanout_every_delivery \
  tests/test_gpu_image.py tests/test_gpu_updates.py \
  > gpurun_out/r04_a/pytest.log 2>&1
rc=$?
tail -n 30 gpurun_out/r04_a/pytest.log
exit $rc
