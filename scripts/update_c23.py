"""Update latency at C2 / C3 scale: 200-op updates (100 deletes
+ 100 inserts) patched into the 1M-wildcard (C2) or 10M-mixed (C3) index,
three in a row (each on the previous result), with the device match time of
10M topics on the flat and the last patched snapshot.  One JSON line per config;
GM_UPDATE_TIMING=1 adds the phase times on stderr.
usage: update_c23.py [c2] [c3]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes, render_codes  # noqa: E402

N_TOPICS = 10_000_000


def kern(ctx, ix, db, do):
    ks = []
    for _ in range(5):
        r = ctx.match_device(ix, db, do, N_TOPICS)
        ks.append(ctx.stats()["match_kernel_ms"])
        r.free()
    return min(ks)


def run(cfg):
    nf, wild = {"c2": (1_000_000, True), "c3": (10_000_000, False)}[cfg]
    ctx = Context(0)
    codes = gen_filter_codes(1, nf, wildcard_only=wild)
    fb, fo = render_codes(codes)
    idx = ctx.build_index((fb, fo))
    db, do, _ = ctx.gen_topics_device(codes, 1, 0, N_TOPICS)
    flat = kern(ctx, idx, db, do)
    rng = np.random.default_rng(7)
    times, cur = [], idx
    for rep in range(3):
        dels = [cur.filter(int(i)) for i in rng.choice(cur.n_filters, 100, replace=False)]
        ins = [b"upd%d/%d/+/#" % (rep, i) for i in range(100)]
        t0 = time.perf_counter()
        new = ctx.update_index(cur, [(f, False) for f in dels] + [(f, True) for f in ins])
        times.append((time.perf_counter() - t0) * 1e3)
        if cur is not idx:
            cur.release()
        cur = new
    patched = kern(ctx, cur, db, do)
    print(json.dumps({"config": cfg, "filters": nf, "ops": 200, "update_ms": times, "match_kernel_ms_flat": flat,
                      "match_kernel_ms_patched": patched, "vs_flat": patched / flat}), flush=True)
    cur.release()
    idx.release()
    ctx.dev_free(db)
    ctx.dev_free(do)
    ctx.close()


for c in sys.argv[1:] or ["c2", "c3"]:
    run(c)
