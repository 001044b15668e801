#!/bin/bash
# Round 4 diagnostics of the shipped walk (separate diagnostic libraries, the
# product library untouched): per-wave phase times (-DGM_PHASE_STATS) and the
# per-level probe census (-DGM_PROBE_STATS) at C2 and C3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04_s
mkdir -p $O
for cfg in c2 c3; do
  EMQX_GM_LIB=emqx_amd/libemqx_gpu_match_phase.so timeout -k 10 400 python3 -u scripts/phase_stats.py $cfg 20000000 > $O/phase_$cfg.log 2>&1 || { tail -10 $O/phase_$cfg.log; exit 1; }
  tail -n 25 $O/phase_$cfg.log
done
cat > $O/census.py <<'PY'
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from emqx_amd import Context
from emqx_amd.engine import gen_filter_codes, render_codes
cfg = sys.argv[1]
n_f, w = {"c2": (1_000_000, True), "c3": (10_000_000, False)}[cfg]
ctx = Context(0)
codes = gen_filter_codes(1, n_f, wildcard_only=w)
idx = ctx.build_index(render_codes(codes))
n = 10_000_000
db, do, _ = ctx.gen_topics_device(codes, 1, 0, n)
r = ctx.match_device(idx, db, do, n); ctx.synchronize(); r.free()
print("census done", cfg, flush=True)
PY
for cfg in c2 c3; do
  EMQX_GM_LIB=emqx_amd/libemqx_gpu_match_census.so timeout -k 10 400 python3 -u $O/census.py $cfg > $O/census_$cfg.log 2>&1 || { tail -10 $O/census_$cfg.log; exit 1; }
  tail -n 20 $O/census_$cfg.log
done
