#!/bin/bash
# Same-box A/B of two builds of the library (EMQX_GM_LIB): per variant, the C2 bench
# under a kernel trace; prints its value and the average time of each kernel.
# usage: gpu_asm_ab.sh <lib-or-"-"|VAR=VALUE> ...   ("-" = the in-tree build; VAR=VALUE: the
# in-tree build with that knob)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/asm_ab
mkdir -p $O
env ${PARITY_ENV:-} timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -m gpu -k "${PARITY_K:-compact_staging or speculative or config_c1 or assemble}" --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for lib in "$@"; do
  i=$((i + 1))
  envs=()
  if [ "$lib" = "-" ]; then unset EMQX_GM_LIB; elif [[ "$lib" == *=* ]]; then unset EMQX_GM_LIB; envs=("$lib"); else export EMQX_GM_LIB=$PWD/$lib; fi
  [ ${#envs[@]} -gt 0 ] && export "${envs[@]}"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/s$i -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu --no-parity --no-host-io --no-update ${BENCH_ARGS:-} > $O/b$i.log 2>&1 || { tail -5 $O/b$i.log; exit 1; }
  [ ${#envs[@]} -gt 0 ] && unset "${envs[0]%%=*}"
  python3 - "$O/s$i" "$O/b$i.log" "$lib" <<'PY'
import csv, glob, json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith('{"metric"')][-1]
ks = {}
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        for k in ("k_match_fused", "k_assemble_c", "k_scan_local", "k_match_lds"):
            if k in n:
                ks[k] = round(float(r["AverageNs"]) / 1e3, 1)
print(sys.argv[3], round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"], 3), "ms/step", ks)
PY
done
