"""One caller's small host-buffer calls (1,024-topic windows) on C2's index,
for a device timeline (rocprofv3 --kernel-trace --memory-copy-trace): what one
call costs the device against its wall time.  usage: small_call_probe.py [calls] [batch]"""
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
    ix = c.build_index(render_codes(codes))
    n = calls * batch + batch
    db, do, tot = c.gen_topics_device(codes, 1, 0, n)
    ho = np.zeros(n + 1, np.uint64)
    c.memcpy_d2h(ho, do, (n + 1) * 8)
    pb = c.host_alloc(tot + 64)
    c.memcpy_d2h(pb, db, tot)
    for k in range(20):  # warm
        c.match_host(ix, (pb, ho[k * batch:(k + 1) * batch + 1]), exact=True).free()
    c.synchronize()
    t0 = time.perf_counter()
    for k in range(calls):
        c.match_host(ix, (pb, ho[k * batch:(k + 1) * batch + 1]), exact=True).free()
    dt = time.perf_counter() - t0
    print(f"{calls} calls of {batch} topics: {dt / calls * 1e6:.1f} us per call, {calls * batch / dt / 1e6:.2f} M topics/s",
          flush=True)
    c.host_free(pb)
    c.dev_free(db)
    c.dev_free(do)
    ix.release()
    c.close()


if __name__ == "__main__":
    main()
