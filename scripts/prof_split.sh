cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/ps
export GM_MATCH_MAIN=split
A="bench.py --topics 20000000 --steps 2 --warmup 1 --no-cpu --filters 1000"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ps/stats -o run --output-format csv -- python3 $A > gpurun_out/ps/stats.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU -d gpurun_out/ps/sq -o run --output-format csv -- python3 $A > gpurun_out/ps/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/ps/l2 -o run --output-format csv -- python3 $A > gpurun_out/ps/l2.log 2>&1 || exit 1
echo done
