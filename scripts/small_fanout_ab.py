"""Small host-row fan-outs (a NIF publish window: match, then emqx_broker
dispatch of the window's rows) on one context: the concurrent one-round-trip
path (gm_host.cpp run_fanout_small) against the locked path it replaced
(EMQX_GM_AB=1 GM_FANOUT_SIMPLE=1), for several caller threads and window
sizes, interleaved.  C2's index (1M wildcard filters) with 1-4 subscribers per
filter, topics of its stream; each caller fans out its own windows' rows.

usage: small_fanout_ab.py [--reps 2]
"""

import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(c, ix, rows, threads, calls):
    errs = []

    def one(t):
        try:
            for k in range(calls):
                ro, ids = rows[(t * calls + k) % len(rows)]
                c.fanout(ix, ro, ids)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=one, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    if errs:
        raise RuntimeError(errs[0])
    return threads * calls / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    torch.zeros(1, device="cuda:0")
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    c = Context(0)
    codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
    fb, fo = render_codes(codes)
    nf = len(fo) - 1
    rng = np.random.default_rng(1)
    cnt = rng.integers(1, 5, size=nf)
    so = np.zeros(nf + 1, np.uint64)
    so[1:] = np.cumsum(cnt)
    si = rng.integers(0, 1 << 24, size=int(so[-1])).astype(np.uint32)
    ix = c.build_index((fb, fo), subs=(so, si))
    n = 1 << 20
    db, do, tot = c.gen_topics_device(codes, 1, 0, n)
    ho = np.zeros(n + 1, np.uint64)
    c.memcpy_d2h(ho, do, (n + 1) * 8)
    pb = c.host_alloc(tot + 64)
    c.memcpy_d2h(pb, db, tot)
    os.environ["EMQX_GM_AB"] = "1"
    for batch in (1024, 16384):
        rows = []
        for k in range(32):
            ro, ids = c.match(ix, (pb, ho[k * batch:(k + 1) * batch + 1]), exact=True)
            rows.append((ro, ids))
        per = sum(int(r[-1]) for r, _ in rows) / len(rows)
        calls = 256 if batch == 1024 else 32
        for threads in (1, 4, 8):
            res = {"locked": [], "small": []}
            for _ in range(a.reps):
                for mode in ("locked", "small"):
                    if mode == "locked":
                        os.environ["GM_FANOUT_SIMPLE"] = "1"
                    else:
                        os.environ.pop("GM_FANOUT_SIMPLE", None)
                    run(c, ix, rows, threads, 4)  # (warm: every thread's buffers)
                    res[mode].append(run(c, ix, rows, threads, calls))
            s, k = max(res["locked"]), max(res["small"])
            print(f"batch {batch:6d} ({per:9.0f} matches) threads {threads}: locked {s:9.0f} calls/s "
                  f"({1e6 / s * threads:7.1f} us/call), small {k:9.0f} calls/s ({1e6 / k * threads:7.1f} us/call) "
                  f"({k / s:.2f}x)", flush=True)
    c.host_free(pb)
    c.dev_free(db)
    c.dev_free(do)
    ix.release()
    c.close()


if __name__ == "__main__":
    main()
