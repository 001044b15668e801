"""One caller's publish windows (emqx_gm_match_fanout, 1,024 topics by default)
on C2's index with 1-4 subscribers per filter, for a device timeline
(rocprofv3 --kernel-trace --memory-copy-trace).  usage: publish_window_probe.py [calls] [batch]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
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
    n = calls * batch + batch
    db, do, tot = c.gen_topics_device(codes, 1, 0, n)
    ho = np.zeros(n + 1, np.uint64)
    c.memcpy_d2h(ho, do, (n + 1) * 8)
    pb = c.host_alloc(tot + 64)
    c.memcpy_d2h(pb, db, tot)
    for k in range(20):
        c.match_fanout(ix, (pb, ho[k * batch:(k + 1) * batch + 1]))
    c.synchronize()
    t0 = time.perf_counter()
    for k in range(calls):
        c.match_fanout(ix, (pb, ho[k * batch:(k + 1) * batch + 1]))
    dt = time.perf_counter() - t0
    print(f"{calls} publish windows of {batch} topics: {dt / calls * 1e6:.1f} us per window", flush=True)
    c.host_free(pb)
    c.dev_free(db)
    c.dev_free(do)
    ix.release()
    c.close()


if __name__ == "__main__":
    main()
