#!/bin/bash
# Round 4, GPU call b: the device-path tests again (bench prefix fixed), the
# image / lazy-mirror tests, the assembly-stream variants, the C4 full check,
# then a C2 bench A/B of the assembly stream (GM_ASM_STREAM=0 vs default).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r04_b
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_bench.py::test_bench_c5_prefix_one_gpu_device_path \
  tests/test_gpu_image.py \
  "tests/test_gpu_parity.py::test_submit_wait_pipelined_vs_oracle" \
  "tests/test_gpu_parity.py::test_many_calls_in_flight_counter_ring" \
  tests/test_gpu_sharded.py::test_prefix_device_path_world8_lockstep \
  tests/test_gpu_scale.py::test_c4_full_fanout_every_delivery \
  > gpurun_out/r04_b/pytest.log 2>&1
rc=$?
tail -n 25 gpurun_out/r04_b/pytest.log
[ $rc -ne 0 ] && exit $rc
for v in 0 default 0 default; do
  if [ $v = 0 ]; then export GM_ASM_STREAM=0; else unset GM_ASM_STREAM; fi
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu --no-parity --no-host-io --no-update \
    > gpurun_out/r04_b/bench_asm_$v.log 2>&1 || { tail -5 gpurun_out/r04_b/bench_asm_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r04_b/bench_asm_$v.log').read().strip().splitlines()[-1]); print('asm=$v', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms'],3), 'kernel ms', round(d['value']/1e9,3), 'G/s')" | tee -a gpurun_out/r04_b/asm_ab.txt
done
