"""C5 at full size on one device: the 100M-filter mixed set
(SURVEY.md §8d generator, seed 1) hash-sharded 8 ways (emqx_gm_shard_of), each
shard built with its filters' global ids (emqx_gm_filter_ranks,
emqx_gm_index_build_shard) and matched against the same topic sample; the 8
pieces merged on the device (emqx_gm_merge_rows) must equal, row for row, the
rows of the unsharded 100M-filter index.  Too long for the -m gpu suite (the
unsharded build alone takes minutes): run once, its JSON line kept under
profiles/.  A heartbeat thread prints every 30 s (the library releases the GIL
in its calls)."""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes, render_codes  # noqa: E402
from emqx_amd.sharded import filter_ranks, select_filters, shard_of  # noqa: E402

N_F = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
N_T = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
W, SEED = 8, 1
T0 = time.time()
stage = {"what": "start"}


def log(msg):
    stage["what"] = msg
    print(f"[c5 {time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def heartbeat():
    while True:
        time.sleep(30)
        print(f"[c5 {time.time() - T0:7.1f}s] ... {stage['what']}", file=sys.stderr, flush=True)


threading.Thread(target=heartbeat, daemon=True).start()
ctx = Context(0)
codes = gen_filter_codes(SEED, N_F)
fb, fo = render_codes(codes)
log(f"{N_F} filters generated ({fo[-1] / 1e9:.2f} GB)")
gids, n_unique = filter_ranks(fb, fo)
sh = shard_of(fb, fo, W)
log(f"global ranks and shards ({n_unique} distinct)")
db, do, _ = ctx.gen_topics_device(codes, SEED, 0, N_T)
del codes
lens = np.zeros((W, N_T), np.uint32)
pieces, build_s = [], []
for q in range(W):
    sfb, sfo = select_filters(fb, fo, sh, q)
    t = time.time()
    sidx = ctx.build_index_shard((sfb, sfo), gids[sh == q])
    build_s.append(time.time() - t)
    r = ctx.match_device(sidx, db, do, N_T, exact=True)
    ro, ids = r.rows(0, N_T)
    lens[q] = np.diff(ro.astype(np.int64)).astype(np.uint32)
    pieces.append(ids)
    r.free()
    sidx.release()
    del sfb, sfo
    log(f"shard {q}: {int((sh == q).sum())} filters built in {build_s[-1]:.1f} s, "
        f"{len(ids)} matches")
d_l = ctx.dev_alloc(lens.nbytes)
allids = np.concatenate(pieces).astype(np.uint32)
d_i = ctx.dev_alloc(max(allids.nbytes, 4))
ctx.memcpy_h2d(d_l, lens, lens.nbytes)
if allids.nbytes:
    ctx.memcpy_h2d(d_i, allids, allids.nbytes)
merged = ctx.merge_rows(N_T, N_T, W, d_l, d_i)
mro, mids = merged.rows(0, N_T)
merged.free()
log("pieces merged")
t = time.time()
idx = ctx.build_index((fb, fo))
t_full = time.time() - t
log(f"unsharded index built in {t_full:.1f} s ({idx.info.device_bytes / 1e9:.1f} GB on the device)")
full = ctx.match_device(idx, db, do, N_T, exact=True)
fro, fids = full.rows(0, N_T)
full.free()
equal = bool(np.array_equal(mro, fro) and np.array_equal(mids, fids))
log(f"merged == unsharded: {equal}")
print(json.dumps({"check": "C5 8 shards merged vs unsharded", "filters": N_F, "distinct": int(n_unique),
                  "shards": W, "topics": N_T, "equal": equal, "nnz": int(fro[-1]),
                  "shard_build_s": build_s, "unsharded_build_s": t_full,
                  "unsharded_device_bytes": int(idx.info.device_bytes)}), flush=True)
ctx.dev_free(d_l)
ctx.dev_free(d_i)
ctx.dev_free(db)
ctx.dev_free(do)
idx.release()
ctx.close()
sys.exit(0 if equal else 1)
