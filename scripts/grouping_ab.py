"""Topic-grouping A/B: does an in-call first-word grouping
pass pay at C3 / C5?  The same 100M-topic device batch is matched two ways,
interleaved over several rounds on one box:

  plain    emqx_gm_match on the batch as generated (the shipped call)
  grouped  the whole in-call pipeline a grouping pass would take, built from the
           library's own device steps: emqx_gm_route_partition (a stable
           counting sort of the topics by first word, via a 64-shard prefix
           plan of the index's filters), emqx_gm_permute_topics (the batch in
           grouped order), emqx_gm_match on it, emqx_gm_csr_row_lengths and
           emqx_gm_unpermute_rows (the rows back in batch order)

Both give the same rows (checked: row lengths and a digest of the ids).
Printed per round: the wall time of each pipeline (device synchronised on
both sides), the main pass's kernel time of each, and the grouped pipeline's
parts.  The kernel time of `grouped` against `plain` is what the locality buys;
the pipeline totals say whether it pays.

usage: grouping_ab.py --config c3|c5 [--topics N] [--rounds R] [--groups G] [--index-cache PATH]
"""

import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    ap.add_argument("--topics", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--index-cache", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes, Route
    from emqx_amd import _lib
    n_f = {"c2": 1_000_000, "c3": 10_000_000, "c5": 100_000_000}[a.config]
    ctx = Context(0)
    t = time.time()
    codes = gen_filter_codes(a.seed, n_f, wildcard_only=a.config == "c2")
    fb, fo = render_codes(codes)
    if a.index_cache and os.path.exists(a.index_cache):
        idx = ctx.import_index(np.fromfile(a.index_cache, np.uint8))
    else:
        idx = ctx.build_index((fb, fo))
        if a.index_cache:
            idx.export().tofile(a.index_cache)
    print(f"index {a.config}: {idx.n_filters} filters, {idx.info.device_bytes / 1e9:.2f} GB, "
          f"{time.time() - t:.1f} s", flush=True)
    # the grouping key: the prefix plan's shard of each topic's first word
    t = time.time()
    shard = np.empty(len(fo) - 1, np.uint32)
    h = _lib.C.c_void_p()
    _lib.check(_lib.lib().emqx_gm_prefix_plan(fb.ctypes.data, fo.ctypes.data, len(fo) - 1, a.groups,
                                                shard.ctypes.data, _lib.C.byref(h)), None, "prefix_plan")
    route = Route(h, a.groups)
    del fb, fo, shard
    print(f"prefix plan ({a.groups} groups): {time.time() - t:.1f} s", flush=True)
    n = a.topics
    db, do, tot = ctx.gen_topics_device(codes, a.seed, 0, n)
    del codes
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    plen = torch.empty(n, dtype=torch.int32, device=dev)
    split = torch.empty(2 * a.groups, dtype=torch.int64, device=dev)
    pb = torch.empty(tot + 64, dtype=torch.uint8, device=dev)
    pb[tot:].zero_()
    po = torch.empty(n + 1, dtype=torch.int64, device=dev)
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def plain():
        ctx.synchronize()
        t0 = time.perf_counter()
        r = ctx.match_device(idx, db, do, n, exact=True)
        ctx.synchronize()
        return r, (time.perf_counter() - t0) * 1e3, ctx.last_kernel_ms()

    def grouped():
        parts = {}
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.route_partition(route, db, do, n, perm.data_ptr(), plen.data_ptr(), split.data_ptr())
        ctx.permute_topics(db, do, n, perm.data_ptr(), pb.data_ptr(), po.data_ptr())
        ctx.synchronize()
        t1 = time.perf_counter()
        r = ctx.match_device(idx, pb.data_ptr(), po.data_ptr(), n, exact=True)
        k = ctx.last_kernel_ms()
        ctx.synchronize()
        t2 = time.perf_counter()
        ctx.csr_row_lengths(r, lens.data_ptr())
        u = ctx.unpermute_rows(n, perm.data_ptr(), lens.data_ptr(), _lib.C.cast(r.csr.ids, _lib.C.c_void_p).value)
        ctx.synchronize()
        t3 = time.perf_counter()
        r.free()
        parts["group"] = (t1 - t0) * 1e3
        parts["match"] = (t2 - t1) * 1e3
        parts["ungroup"] = (t3 - t2) * 1e3
        return u, (t3 - t0) * 1e3, k, parts

    def digest(r):
        lo, hi = n // 3, n // 3 + 200_000
        ro, ids = r.rows(lo, hi - lo)
        return int(r.nnz), int(np.bitwise_xor.reduce(ids.astype(np.uint64) * np.uint64(2654435761)
                                                      + np.repeat(np.arange(len(ro) - 1, dtype=np.uint64),
                                                                  np.diff(ro).astype(np.int64))))

    res = {"plain": [], "grouped": []}
    ker = {"plain": [], "grouped": []}
    for rnd in range(a.rounds):
        r0, w0, k0 = plain()
        r1, w1, k1, parts = grouped()
        d0, d1 = digest(r0), digest(r1)
        assert d0 == d1, (d0, d1)
        r0.free()
        r1.free()
        res["plain"].append(w0)
        res["grouped"].append(w1)
        ker["plain"].append(k0)
        ker["grouped"].append(k1)
        print(f"round {rnd}: plain {w0:.2f} ms (kernel {k0:.2f}) | grouped {w1:.2f} ms (kernel {k1:.2f}; "
              f"group {parts['group']:.2f}, match {parts['match']:.2f}, ungroup {parts['ungroup']:.2f}) "
              f"nnz {d0[0]}", flush=True)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(f"{a.config} {n} topics, {a.groups} groups: plain median {med(res['plain']):.2f} ms "
          f"(kernel {med(ker['plain']):.2f}); grouped median {med(res['grouped']):.2f} ms "
          f"(kernel {med(ker['grouped']):.2f}); grouped/plain {med(res['grouped']) / med(res['plain']):.3f}",
          flush=True)
    route.release()
    ctx.dev_free(db)
    ctx.dev_free(do)
    idx.release()
    ctx.close()


if __name__ == "__main__":
    main()
