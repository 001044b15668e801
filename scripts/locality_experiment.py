"""Experiment (not a product path): how much of the C2 walk is L2 locality?
The same N C2 topics matched in generator order vs reordered by their leading
bytes (topics with the same first words -> the same subtree of the index ->
consecutive workgroups), k_match_fused time from the library's HIP events.
Prints one JSON line per ordering."""
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes, render_codes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
ctx = Context(0)
codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
idx = ctx.build_index(render_codes(codes))
db, do, tbytes = ctx.gen_topics_device(codes, 1, 0, N)
hb = np.zeros(tbytes + 64, np.uint8)
ho = np.zeros(N + 1, np.uint64)
ctx.memcpy_d2h(hb, db, tbytes)
ctx.memcpy_d2h(ho, do, (N + 1) * 8)
starts = ho[:-1].astype(np.int64)
lens = np.diff(ho).astype(np.int64)


def key_bytes(k):
    """Big-endian key of the first k bytes of every topic (zero padded)."""
    key = np.zeros(N, np.uint64)
    for j in range(k):
        b = np.where(lens > j, hb[np.minimum(starts + j, tbytes)], 0).astype(np.uint64)
        key = (key << np.uint64(8)) | b
    return key


def reorder(perm):
    nl = lens[perm]
    no = np.zeros(N + 1, np.uint64)
    np.cumsum(nl, out=no[1:])
    src = np.repeat(starts[perm] - no[:-1].astype(np.int64), nl) + np.arange(int(no[-1]), dtype=np.int64)
    nb = np.zeros(int(no[-1]) + 64, np.uint8)
    nb[:int(no[-1])] = hb[src]
    return nb, no


def run(name, b, o):
    d_b = ctx.dev_alloc(len(b))
    d_o = ctx.dev_alloc(len(o) * 8)
    ctx.memcpy_h2d(d_b, b, len(b))
    ctx.memcpy_h2d(d_o, o, len(o) * 8)
    ks = []
    nnz = 0
    for k in range(7):
        r = ctx.match_device(idx, d_b, d_o, N)
        ctx.synchronize()
        st = ctx.stats()
        nnz = r.nnz
        r.free()
        if k >= 2:
            ks.append(st["match_kernel_ms"])
    ctx.dev_free(d_b)
    ctx.dev_free(d_o)
    print(json.dumps({"order": name, "topics": N, "kernel_ms": statistics.median(ks), "nnz": nnz,
                      "probes_per_topic": st["probes"] / N}), flush=True)


def first_word_key():
    """The first word's bytes (up to 8, zero padded) of every topic, as a u64."""
    key = np.zeros(N, np.uint64)
    live = np.ones(N, bool)
    for j in range(8):
        b = np.where(lens > j, hb[np.minimum(starts + j, tbytes)], 0)
        live &= b != ord("/")
        key |= np.where(live, b, 0).astype(np.uint64) << np.uint64(8 * j)
    return key


def xcd_order(buckets, nb=8, blk=256):
    """Workgroup i (XCD i % 8 under round-robin dispatch) takes 256 topics of bucket i % 8."""
    lists = [list(np.nonzero(buckets == x)[0]) for x in range(nb)]
    pos = [0] * nb
    out = []
    while len(out) < N:
        for x in range(nb):
            src = x
            if pos[src] >= len(lists[src]):  # bucket drained: any other
                cands = [y for y in range(nb) if pos[y] < len(lists[y])]
                if not cands:
                    break
                src = cands[0]
            out.extend(lists[src][pos[src]:pos[src] + blk])
            pos[src] += blk
    return np.array(out[:N], np.int64)


run("generator", hb, ho)
fw = first_word_key()
bk = ((fw * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(61)).astype(np.int64)
b, o = reorder(xcd_order(bk))
run("xcd_routed_first_word", b, o)
b, o = reorder(np.argsort(fw, kind="stable"))
run("grouped_first_word", b, o)
for k in (8, 16):
    perm = np.argsort(key_bytes(min(k, 8)), kind="stable") if k <= 8 else None
    if k == 16:
        k1, k2 = key_bytes(8), None
        # second 8 bytes
        key = np.zeros(N, np.uint64)
        for j in range(8, 16):
            bb = np.where(lens > j, hb[np.minimum(starts + j, tbytes)], 0).astype(np.uint64)
            key = (key << np.uint64(8)) | bb
        perm = np.lexsort((key, k1))
    b, o = reorder(perm)
    run(f"sorted_{k}B", b, o)
ctx.dev_free(db)
ctx.dev_free(do)
idx.release()
ctx.close()
