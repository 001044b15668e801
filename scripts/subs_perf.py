"""Subscriber maintenance at C2 scale (emqx_gm_index_update_subs): the 1M-filter
C2 set with 8 subscribers per filter (8M entries); one batch of k ops (half
unsubscribes of present pairs, half subscribes, a tenth of them to new
filters) vs a rebuild of the same state.  One JSON line per k."""
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes, render_codes  # noqa: E402

PER = 8
ctx = Context(0)
codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
fb, fo = render_codes(codes)
n = len(fo) - 1
so = np.arange(n + 1, dtype=np.uint64) * PER
si = (np.arange(n * PER, dtype=np.uint64) % 1_000_003).astype(np.uint32)
t = time.perf_counter()
idx = ctx.build_index((fb, fo), subs=(so, si))
t_build = time.perf_counter() - t
print(json.dumps({"k": 0, "build_ms": t_build * 1e3, "entries": int(so[-1])}), flush=True)
extra = render_codes(gen_filter_codes(99, 20_000, wildcard_only=True))
extra = [bytes(extra[0][extra[1][i]:extra[1][i + 1]]) for i in range(len(extra[1]) - 1)]
rng = random.Random(1)
for k in [int(x) for x in (sys.argv[1:] or ["100", "1000", "10000"])]:
    ops = []
    for i in range(k):
        if i % 2 == 0:  # unsubscribe a present pair (filter order == id order: so is uniform)
            f = rng.randrange(n)
            ops.append((bytes(fb[fo[f]:fo[f + 1]]), int(si[f * PER + rng.randrange(PER)]), False))
        elif i % 10 == 1:  # a new filter's first subscriber
            ops.append((extra[rng.randrange(len(extra))], 2_000_000 + i, True))
        else:
            f = rng.randrange(n)
            ops.append((bytes(fb[fo[f]:fo[f + 1]]), 3_000_000 + i, True))
    t = time.perf_counter()
    new = ctx.update_subs(idx, ops)
    t_upd = time.perf_counter() - t
    print(json.dumps({"k": k, "update_ms": t_upd * 1e3, "rebuild_ms": t_build * 1e3,
                      "filters": new.n_filters, "entries": int(new.info.n_subs)}), flush=True)
    new.release()
    idx.release()  # the mirror moved to the released snapshot: a fresh base for the next k
    idx = ctx.build_index((fb, fo), subs=(so, si))
# subscriber-only batches (no route changes): the new snapshot shares the tables
for k in (100, 1000, 10000):
    ops = []
    for i in range(k):
        f = rng.randrange(n)
        fbytes = bytes(fb[fo[f]:fo[f + 1]])
        ops.append((fbytes, 4_000_000 + i, True) if i % 2 else (fbytes, int(si[f * PER + rng.randrange(PER)]), False))
    t = time.perf_counter()
    new = ctx.update_subs(idx, ops)
    t_upd = time.perf_counter() - t
    print(json.dumps({"k": k, "subscriber_only": True, "update_ms": t_upd * 1e3, "filters": new.n_filters,
                      "entries": int(new.info.n_subs)}), flush=True)
    new.release()
    idx.release()
    idx = ctx.build_index((fb, fo), subs=(so, si))
idx.release()
ctx.close()
