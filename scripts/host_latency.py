"""Latency of one emqx_gm_match call vs batch size at C2 (1M wildcard filters):
host buffers in / host rows out (the NIF's call, gm_host.cpp) and device
buffers (DEVICE_IO).  Median of 7 calls after 2 warm-up calls; one JSON line
per batch size (DESIGN.md "Host path" table)."""
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes, render_codes  # noqa: E402

MODE = os.environ.get("LAT_MODE", "both")  # both | host | device
sizes = [int(x) for x in (sys.argv[1:] or ["1000", "10000", "100000", "1000000", "10000000", "100000000"])]
ctx = Context(0)
codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
idx = ctx.build_index(render_codes(codes))
for n in sizes:
    db, do, tbytes = ctx.gen_topics_device(codes, 1, 0, n)
    hb = np.zeros(tbytes + 64, np.uint8)
    ho = np.zeros(n + 1, np.uint64)
    ctx.memcpy_d2h(hb, db, tbytes)
    ctx.memcpy_d2h(ho, do, (n + 1) * 8)
    host, dev = [], []
    for k in range(9):
        if MODE != "device":
            t0 = time.perf_counter()
            h = ctx.match_host(idx, (hb, ho))
            t1 = time.perf_counter()
            h.free()
            if k >= 2:
                host.append(t1 - t0)
        if MODE != "host":
            t1 = time.perf_counter()
            r = ctx.match_device(idx, db, do, n)
            ctx.synchronize()
            t2 = time.perf_counter()
            r.free()
            if k >= 2:
                dev.append(t2 - t1)
    mh = statistics.median(host) if host else float("nan")
    md = statistics.median(dev) if dev else float("nan")
    print(json.dumps({"mode": MODE, "topics": n, "host_io_ms": mh * 1e3, "host_io_topics_per_s": n / mh,
                      "device_io_ms": md * 1e3, "device_io_topics_per_s": n / md}), flush=True)
    ctx.dev_free(db)
    ctx.dev_free(do)
idx.release()
ctx.close()
