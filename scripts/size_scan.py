"""Experiment: k_match_fused time per topic vs batch size at C2 (does the topic
stream evict the index from the 256 MiB Infinity Cache?).  One JSON line per N."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes, render_codes  # noqa: E402

ctx = Context(0)
codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
idx = ctx.build_index(render_codes(codes))
for n in [int(x) for x in sys.argv[1:]]:
    db, do, tbytes = ctx.gen_topics_device(codes, 1, 0, n)
    ks = []
    for k in range(9):
        r = ctx.match_device(idx, db, do, n)
        ctx.synchronize()
        ks.append(ctx.stats()["match_kernel_ms"])
        r.free()
    km = statistics.median(ks[2:])
    print(json.dumps({"topics": n, "text_mb": tbytes / 1e6, "kernel_ms": km, "ps_per_topic": km * 1e9 / n}), flush=True)
    ctx.dev_free(db)
    ctx.dev_free(do)
