"""One caller's small host-row fan-outs (16K-topic windows' rows by default) on
C2's index with 1-4 subscribers per filter, for a device timeline
(rocprofv3 --kernel-trace --memory-copy-trace).  usage: small_fanout_probe.py [calls] [batch]
(EMQX_GM_AB=1 GM_FANOUT_SIMPLE=1 in the environment: the locked path)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
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
    db, do, tot = c.gen_topics_device(codes, 1, 0, batch * 8)
    ho = np.zeros(batch * 8 + 1, np.uint64)
    c.memcpy_d2h(ho, do, len(ho) * 8)
    pb = c.host_alloc(tot + 64)
    c.memcpy_d2h(pb, db, tot)
    rows = [c.match(ix, (pb, ho[k * batch:(k + 1) * batch + 1]), exact=True) for k in range(8)]
    for k in range(20):
        c.fanout(ix, *rows[k % 8])
    c.synchronize()
    t0 = time.perf_counter()
    for k in range(calls):
        c.fanout(ix, *rows[k % 8])
    dt = time.perf_counter() - t0
    print(f"{calls} fan-outs of {batch}-topic windows: {dt / calls * 1e6:.1f} us per call "
          f"(GM_FANOUT_SIMPLE={os.environ.get('GM_FANOUT_SIMPLE', '')})", flush=True)
    c.host_free(pb)
    c.dev_free(db)
    c.dev_free(do)
    ix.release()
    c.close()


if __name__ == "__main__":
    main()
