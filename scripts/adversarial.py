"""Adversarial filter sets: every word sequence of depth
1..D over {w, +}, each also with a '/#' suffix, plus '#' -- a topic
'w/w/.../w' matches hundreds of them, so rows overflow the main pass and the
listed pass and go to the device slow path.  Topics: random words from
{w, x} of depth 1..D+2.  Reports topics/s, matches/topic, the rows each pass
took, and checks a sample against the oracle.  One JSON line per depth."""
import itertools
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import pack  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (test infrastructure: the checker only)

N = int(os.environ.get("ADV_TOPICS", "1000000"))
ctx = Context(0)
for D in [int(x) for x in (sys.argv[1:] or ["6", "9", "12"])]:
    fs = {b"#"}
    for d in range(1, D + 1):
        for ws in itertools.product([b"w", b"+"], repeat=d):
            f = b"/".join(ws)
            fs.add(f)
            fs.add(f + b"/#")
    filters = sorted(fs)
    rng = random.Random(D)
    topics = [b"/".join(rng.choice([b"w", b"w", b"w", b"x"]) for _ in range(rng.randint(1, D + 2))) for _ in range(N)]
    idx = ctx.build_index(filters)
    tb, to = pack(topics)
    d_b = ctx.dev_alloc(len(tb))
    d_o = ctx.dev_alloc(len(to) * 8)
    ctx.memcpy_h2d(d_b, tb, len(tb))
    ctx.memcpy_h2d(d_o, to, len(to) * 8)
    r = ctx.match_device(idx, d_b, d_o, N)  # warm
    r.free()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        r = ctx.match_device(idx, d_b, d_o, N)
        ctx.synchronize()
        ts.append(time.perf_counter() - t0)
        st = ctx.stats()
        nnz = r.nnz
        if _ < 2:
            r.free()
    # oracle sample: 2,000 topics spread over the batch
    ro, ids = r.rows(0, N)
    r.free()
    pick = sorted(random.Random(7).sample(range(N), 2000))
    router = orc.Router(True)
    for f in filters:
        router.add_route(f)
    sub = [topics[i] for i in pick]
    oro, oids, _ = router.match_batch(sub, filters, mode=1)
    ok = all(ids[int(ro[i]):int(ro[i + 1])].tolist() == oids[int(oro[k]):int(oro[k + 1])].tolist()
             for k, i in enumerate(pick))
    best = min(ts)
    print(json.dumps({"depth": D, "filters": len(filters), "topics": N, "ms": best * 1e3,
                      "topics_per_s": N / best, "matches_per_topic": nnz / N, "kernel_ms": st["match_kernel_ms"],
                      "device_ms": st["total_device_ms"], "listed_rows": st["n_overflow"],
                      "oracle_sample_ok": ok}), flush=True)
    ctx.dev_free(d_b)
    ctx.dev_free(d_o)
    idx.release()
ctx.close()
