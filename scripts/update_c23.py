"""Update latency at C2 / C3 scale: 200-op updates (100 deletes
+ 100 inserts) patched into the 1M-wildcard (C2) or 10M-mixed (C3) index,
three in a row (each on the previous result), with the device match time of
10M topics on the flat and the last patched snapshot.  One JSON line per config;
GM_UPDATE_TIMING=1 adds the phase times on stderr.  --ab: ten updates in a row
alternating the one-pass device update and GM_UPDATE_UNFUSED (copy, patch,
renumber in place), each mode's times reported apart.
usage: update_c23.py [--ab] [c2] [c3] [c5]"""
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
    nf, wild = {"c2": (1_000_000, True), "c3": (10_000_000, False), "c5": (100_000_000, False)}[cfg]
    ctx = Context(0)
    codes = gen_filter_codes(1, nf, wildcard_only=wild)
    fb, fo = render_codes(codes)
    idx = ctx.build_index((fb, fo))
    db, do, _ = ctx.gen_topics_device(codes, 1, 0, N_TOPICS)
    flat = kern(ctx, idx, db, do)
    rng = np.random.default_rng(7)
    times, cur = [], idx
    modes = []
    for rep in range(10 if AB else 3):
        if AB:
            modes.append("unfused" if rep % 2 else "fused")
            if rep % 2:
                os.environ["GM_UPDATE_UNFUSED"] = "1"
            else:
                os.environ.pop("GM_UPDATE_UNFUSED", None)
        dels = [cur.filter(int(i)) for i in rng.choice(cur.n_filters, 100, replace=False)]
        ins = [b"upd%d/%d/+/#" % (rep, i) for i in range(100)]
        t0 = time.perf_counter()
        new = ctx.update_index(cur, [(f, False) for f in dels] + [(f, True) for f in ins])
        times.append((time.perf_counter() - t0) * 1e3)
        if cur is not idx:
            cur.release()
        cur = new
    os.environ.pop("GM_UPDATE_UNFUSED", None)
    patched = kern(ctx, cur, db, do)
    line = {"config": cfg, "filters": nf, "ops": 200, "update_ms": times, "match_kernel_ms_flat": flat,
            "match_kernel_ms_patched": patched, "vs_flat": patched / flat,
            "device_bytes": idx.info.device_bytes}
    if AB:  # (the first update of a lazily mirrored index downloads the mirror: left out)
        for m in ("fused", "unfused"):
            line[m + "_ms"] = [t for t, mm in zip(times[1:], modes[1:]) if mm == m]
    print(json.dumps(line), flush=True)
    cur.release()
    idx.release()
    ctx.dev_free(db)
    ctx.dev_free(do)
    ctx.close()


AB = "--ab" in sys.argv


def _heartbeat():  # (a 100M-filter build prints nothing for minutes)
    t0 = time.time()
    while True:
        time.sleep(30)
        print(f"[update_c23] running, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)


import threading  # noqa: E402

threading.Thread(target=_heartbeat, daemon=True).start()
for c in [x for x in sys.argv[1:] if x != "--ab"] or ["c2", "c3"]:
    run(c)
