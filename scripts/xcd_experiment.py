"""Experiment: does routing topics to XCDs by their level-1 word cut k_walk time?
Reorders a C2 batch on the host (bucket = hash(level-1 word) % 8) so that
workgroup i (dispatched to XCD i % 8) sees only bucket i % 8, and compares the
match-kernel time with the original order and with a bucket-sorted order whose
blocks do not follow the XCDs.  Measurement only; not part of the product."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import Context
from emqx_amd.engine import gen_filter_codes, render_codes

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
with Context(0) as ctx:
    codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
    idx = ctx.build_index(render_codes(codes))
    db, do, tbytes = ctx.gen_topics_device(codes, 1, 0, N)
    off = np.empty(N + 1, np.uint64); ctx.memcpy_d2h(off, do, off.nbytes)
    tb = np.empty(int(off[-1]) + 64, np.uint8); ctx.memcpy_d2h(tb, db, int(off[-1]))
    ctx.dev_free(db); ctx.dev_free(do)
    off = off.astype(np.int64)
    slash = np.flatnonzero(tb[: off[-1]] == ord('/'))
    k1 = np.searchsorted(slash, off[:-1])          # first '/' of each topic
    s1 = slash[np.minimum(k1, len(slash) - 1)]
    s2 = slash[np.minimum(k1 + 1, len(slash) - 1)]
    ok = (k1 + 1 < len(slash)) & (s2 < off[1:])
    ln = s2 - s1 - 1
    t64 = tb.astype(np.int64)
    h = ln * 0x85EBCA77
    for k in (1, 2, 3, 4):  # the word's last four bytes (the digits of "l1w<k>") and length
        h = h * 0x100000001B3 + np.where(ln >= k, t64[np.maximum(s2 - k, 0)], 0)
    h = np.where(ok, h, 0)
    h = h.astype(np.uint64)
    h ^= h >> np.uint64(33); h *= np.uint64(0xff51afd7ed558ccd); h ^= h >> np.uint64(33)
    h *= np.uint64(0xc4ceb9fe1a85ec53); h ^= h >> np.uint64(33)
    bucket = (h & np.uint64(7)).astype(np.int64)
    lists = [np.flatnonzero(bucket == b) for b in range(8)]
    m = min(len(l) for l in lists) // 2048 * 2048
    print("bucket sizes", [len(l) for l in lists], "use", m * 8, flush=True)
    L = np.stack([l[:m] for l in lists])            # [8][m]
    # xcd order: chunk j (256 topics) = bucket j % 8
    xcd = L.reshape(8, m // 256, 256).transpose(1, 0, 2).reshape(-1)
    # sorted order, blocks not aligned to XCDs: 8 consecutive chunks per bucket
    srt = L.reshape(8, m // 2048, 2048).transpose(1, 0, 2).reshape(-1)
    orig = np.arange(8 * m)

    def run(order, name):
        lens = (off[1:] - off[:-1])[order]
        no = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        starts = off[:-1][order]
        idxs = np.repeat(starts - no[:-1].astype(np.int64), lens) + np.arange(int(no[-1]))
        nb = np.zeros(int(no[-1]) + 64, np.uint8); nb[: int(no[-1])] = tb[idxs]
        d_b = ctx.dev_alloc(nb.nbytes); d_o = ctx.dev_alloc(no.nbytes)
        ctx.memcpy_h2d(d_b, nb, nb.nbytes); ctx.memcpy_h2d(d_o, no, no.nbytes)
        ks = []
        for i in range(6):
            r = ctx.match_device(idx, d_b, d_o, len(order), exact=True)
            if i: ks.append(ctx.stats()["match_kernel_ms"])
            nnz = r.nnz; r.free()
        ctx.dev_free(d_b); ctx.dev_free(d_o)
        print(f"{name:6s} n={len(order)} nnz={nnz} kernel_ms={np.median(ks):.3f} ({min(ks):.3f}..{max(ks):.3f})", flush=True)

    for order, name in ((orig, "orig"), (xcd, "xcd"), (srt, "sorted"), (orig, "orig"), (xcd, "xcd")):
        run(order, name)
