#!/bin/bash
# Round 5, GPU call b: a C2 bench line with the host-io detail (page-locked,
# pageable, two replicas) and the serial host path A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05_b
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_image.py \
  tests/test_gpu_multi.py tests/test_gpu_updates.py \
  tests/test_gpu_sharded.py::test_prefix_device_path_library_first_default_stream_inputs \
  tests/test_gpu_sharded.py::test_prefix_device_path_world1 > gpurun_out/r05_b/pytest.log 2>&1
rc=$?
tail -n 15 gpurun_out/r05_b/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r05_b/bench_c2.log 2>&1
rc=$?
tail -c 1500 gpurun_out/r05_b/bench_c2.log
[ $rc -ne 0 ] && exit $rc
GM_HOST_PIPE=serial timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-parity --no-update \
  --no-host-replicas > gpurun_out/r05_b/bench_c2_serial.log 2>&1
rc=$?
python3 -c "
import json
for n in ('bench_c2', 'bench_c2_serial'):
    d = json.loads(open('gpurun_out/r05_b/%s.log' % n).read().strip().splitlines()[-1])['detail']
    print(n, {k: v for k, v in d.items() if k.startswith('host_io')})
"
exit $rc
