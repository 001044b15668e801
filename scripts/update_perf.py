"""Incremental update at C2 (1M wildcard filters): the
latency of emqx_gm_index_update for k delete + k insert ops, and the device
match time (DEVICE_IO, 10M C2 topics, median of 7 after 2 warm-ups) on the
updated snapshot -- in-place patch (default) vs overlay (GM_UPDATE_OVERLAY=1)
-- against a flat rebuild of the same set.  One JSON line per k
(DESIGN.md "Incremental updates")."""
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes, pack, render_codes  # noqa: E402

N_TOPICS = int(os.environ.get("UPD_TOPICS", "10000000"))
ks = [int(x) for x in (sys.argv[1:] or ["100", "1000", "10000"])]
ctx = Context(0)
codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
fb, fo = render_codes(codes)
base = [bytes(fb[fo[i]:fo[i + 1]]) for i in range(len(fo) - 1)]
idx = ctx.build_index((fb, fo))
db, do, _ = ctx.gen_topics_device(codes, 1, 0, N_TOPICS)


def unpack(p):
    b, o = p
    return [bytes(b[o[i]:o[i + 1]]) for i in range(len(o) - 1)]


def match_ms(ix):
    ts = []
    for k in range(9):
        t0 = time.perf_counter()
        r = ctx.match_device(ix, db, do, N_TOPICS)
        ctx.synchronize()
        t1 = time.perf_counter()
        nnz = r.nnz
        r.free()
        if k >= 2:
            ts.append(t1 - t0)
    return statistics.median(ts) * 1e3, nnz


flat0_ms, _ = match_ms(idx)
print(json.dumps({"k": 0, "flat_ms": flat0_ms}), flush=True)
rng = random.Random(3)
for k in ks:
    dels = rng.sample(base, k)
    extra = unpack(render_codes(gen_filter_codes(1000 + k, k, wildcard_only=True)))
    ops = [(f, False) for f in dels] + [(f, True) for f in extra]
    row = {"k": k, "ops": len(ops)}
    for form in ("patch", "overlay"):
        if form == "overlay":
            os.environ["GM_UPDATE_OVERLAY"] = "1"
        else:
            os.environ.pop("GM_UPDATE_OVERLAY", None)
        t0 = time.perf_counter()
        new = ctx.update_index(idx, ops)
        row[f"{form}_update_ms"] = (time.perf_counter() - t0) * 1e3
        row[f"{form}_match_ms"], row[f"{form}_nnz"] = match_ms(new)
        new.release()
        os.environ.pop("GM_UPDATE_OVERLAY", None)
    cur = sorted((set(base) - set(dels)) | set(extra))
    t0 = time.perf_counter()
    flat = ctx.build_index(pack(cur))
    row["rebuild_ms"] = (time.perf_counter() - t0) * 1e3
    row["flat_match_ms"], row["flat_nnz"] = match_ms(flat)
    flat.release()
    row["patch_vs_flat"] = row["patch_match_ms"] / row["flat_match_ms"]
    row["overlay_vs_flat"] = row["overlay_match_ms"] / row["flat_match_ms"]
    print(json.dumps(row), flush=True)
    # the patch moved idx's mirror to the released snapshot: rebuild idx for the next k
    idx.release()
    idx = ctx.build_index((fb, fo))
ctx.dev_free(db)
ctx.dev_free(do)
idx.release()
ctx.close()
