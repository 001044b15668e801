"""Small host-buffer calls (NIF publish windows) on one context: the concurrent
path (gm_host.cpp run_host_small: staging and the device round trip outside
the context lock) against the one-chunk serial path it replaced (reachable
with EMQX_GM_AB=1 GM_HOST_PIPE=serial), for several caller threads and window
sizes, interleaved.  C2's index (1M wildcard filters), topics of its stream.

usage: small_calls_ab.py [--devices 0] [--reps 2]
"""

import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(c, ix, pb, ho, threads, calls, batch):
    n = len(ho) - 1
    errs = []

    def one(t):
        try:
            for k in range(calls):
                s0 = ((t * calls + k) * batch) % max(1, n - batch)
                c.match_host(ix, (pb, ho[s0:s0 + batch + 1]), exact=True).free()
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
    ap.add_argument("--devices", default="0")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    torch.zeros(1, device="cuda:0")
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    devs = [int(x) for x in a.devices.split(",")]
    c = Context(devices=devs) if len(devs) > 1 else Context(devs[0])
    codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
    ix = c.build_index(render_codes(codes))
    n = 8_000_000
    db, do, tot = c.gen_topics_device(codes, 1, 0, n)
    ho = np.zeros(n + 1, np.uint64)
    c.memcpy_d2h(ho, do, (n + 1) * 8)
    pb = c.host_alloc(tot + 64)
    c.memcpy_d2h(pb, db, tot)
    os.environ["EMQX_GM_AB"] = "1"
    for batch, calls in ((1024, 256), (16384, 32), (65536, 8), (262144, 4)):
        for threads in (1, 2, 4, 8):
            res = {"serial": [], "concurrent": []}
            for _ in range(a.reps):
                for mode in ("serial", "concurrent"):
                    if mode == "serial":
                        os.environ["GM_HOST_PIPE"] = "serial"
                    else:
                        os.environ.pop("GM_HOST_PIPE", None)
                    run(c, ix, pb, ho, threads, 4, batch)  # (warm: every thread's buffers)
                    res[mode].append(run(c, ix, pb, ho, threads, calls, batch))
            s, k = max(res["serial"]), max(res["concurrent"])
            print(f"devices {devs} batch {batch:6d} threads {threads}: serial {s / 1e6:8.2f} M topics/s, "
                  f"concurrent {k / 1e6:8.2f} M topics/s ({k / s:.2f}x)", flush=True)
    c.host_free(pb)
    c.dev_free(db)
    c.dev_free(do)
    ix.release()
    c.close()


if __name__ == "__main__":
    main()
