"""Publish windows (the NIF's fanout_batch: route + dispatch of a batch of
topics) on one context: emqx_gm_match_fanout's one device round trip against
emqx_gm_match then emqx_gm_fanout (two), for several caller threads and window
sizes, interleaved.  C2's index (1M wildcard filters) with 1-4 subscribers per
filter, topics of its stream.  usage: publish_window_ab.py [--reps 2]"""

import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(c, ix, pb, ho, threads, calls, batch, fused):
    n = len(ho) - 1
    errs = []

    def one(t):
        try:
            for k in range(calls):
                s0 = ((t * calls + k) * batch) % max(1, n - batch)
                win = (pb, ho[s0:s0 + batch + 1])
                if fused:
                    c.match_fanout(ix, win)
                else:
                    ro, ids = c.match(ix, win, exact=True)
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
    return threads * calls * batch / dt


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
    so = np.zeros(nf + 1, np.uint64)
    so[1:] = np.cumsum(rng.integers(1, 5, size=nf))
    si = rng.integers(0, 1 << 24, size=int(so[-1])).astype(np.uint32)
    ix = c.build_index((fb, fo), subs=(so, si))
    n = 4_000_000
    db, do, tot = c.gen_topics_device(codes, 1, 0, n)
    ho = np.zeros(n + 1, np.uint64)
    c.memcpy_d2h(ho, do, (n + 1) * 8)
    pb = c.host_alloc(tot + 64)
    c.memcpy_d2h(pb, db, tot)
    for batch, calls in ((1024, 200), (16384, 24)):
        for threads in (1, 4, 8):
            res = {"two calls": [], "fused": []}
            for _ in range(a.reps):
                for mode in ("two calls", "fused"):
                    run(c, ix, pb, ho, threads, 4, batch, mode == "fused")  # (warm)
                    res[mode].append(run(c, ix, pb, ho, threads, calls, batch, mode == "fused"))
            s, k = max(res["two calls"]), max(res["fused"])
            print(f"batch {batch:6d} threads {threads}: match + fanout {s / 1e6:8.2f} M topics/s "
                  f"({batch / s * threads * 1e6:7.1f} us/window), match_fanout {k / 1e6:8.2f} M topics/s "
                  f"({batch / k * threads * 1e6:7.1f} us/window) ({k / s:.2f}x)", flush=True)
    c.host_free(pb)
    c.dev_free(db)
    c.dev_free(do)
    ix.release()
    c.close()


if __name__ == "__main__":
    main()
