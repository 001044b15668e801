#!/usr/bin/env python3
"""Diagnostics: per-phase wave cycles of k_match_fused (GM_PHASE_STATS build)
or the probe census (GM_PROBE_STATS build) on a config's index and topic
stream.  Run with EMQX_GM_LIB=emqx_amd/libemqx_gpu_match_phase.so (or
_census.so); the library prints one line per match call on stderr.
usage: phase_stats.py [c2|c3] [topics]"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes, render_codes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
nf, wild = {"c2": (1_000_000, True), "c3": (10_000_000, False)}[cfg]
ctx = Context(0)
codes = gen_filter_codes(1, nf, wildcard_only=wild)
idx = ctx.build_index(render_codes(codes))
db, do, _ = ctx.gen_topics_device(codes, 1, 0, n)
for _ in range(3):
    r = ctx.match_device(idx, db, do, n)
    ctx.synchronize()
    r.free()
