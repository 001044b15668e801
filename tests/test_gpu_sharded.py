"""Sharded index on the GPU: shard indexes that carry
global filter ids, the device row merge, and the ShardedMatcher pipeline with
two ranks sharing one device over gloo.  Bar: merged rows bit-exact with the
unsharded index and the oracle."""

import os
import random
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from emqx_amd import Context
    c = Context(0)
    yield c
    c.close()


def _oracle_rows(orc, filters, tb, to):
    """The oracle's emqx_router:match_routes/1 rows (trie walk + exact routes)."""
    uniq = sorted(set(filters))
    r = orc.Router(True)
    for f in uniq:
        r.add_route(f)
    ro, ids, _ = r.match_batch((tb, to), uniq, mode=1, nthreads=8)
    return ro, ids


def _to_device(ctx, tb, to):
    d_tb = ctx.dev_alloc(len(tb))
    d_to = ctx.dev_alloc(len(to) * 8)
    ctx.memcpy_h2d(d_tb, tb, len(tb))
    ctx.memcpy_h2d(d_to, to, len(to) * 8)
    return d_tb, d_to


def _sets(kind):
    from tests.test_gpu_parity import _rand_filter, _rand_topic
    if kind == "random":
        rng = random.Random(31)
        fs = [_rand_filter(rng).encode() for _ in range(400)]
        ts = [_rand_topic(rng).encode() for _ in range(3000)]
        return fs, ts
    from emqx_amd.engine import gen_filter_codes, render_codes
    from oracle import oracle as orc
    codes = gen_filter_codes(4, 20_000)
    fs = orc.unpack(*render_codes(codes))
    ts = orc.unpack(*orc.render_codes(orc.gen_topic_codes(4, 0, 50_000, codes)))
    return fs, ts


@pytest.mark.parametrize("kind", ["random", "c1"])
@pytest.mark.parametrize("shards", [2, 3, 5])
def test_shard_indexes_merge_to_unsharded_rows(ctx, orc, kind, shards):
    from emqx_amd.engine import pack
    from emqx_amd.sharded import plan_shard
    filters, topics = _sets(kind)
    fb, fo = pack(filters)
    tb, to = pack(topics)
    n = len(topics)
    full = ctx.build_index(filters)
    fro, fids = ctx.match(full, (tb, to), exact=True)
    d_tb, d_to = _to_device(ctx, tb, to)
    d_lens = ctx.dev_alloc(shards * n * 4)
    parts, idxs, total = [], [], 0
    for r in range(shards):
        sfb, sfo, gids, nu = plan_shard(fb, fo, shards, r)
        idx = ctx.build_index_shard((sfb, sfo), gids)
        idxs.append(idx)
        res = ctx.match_device(idx, d_tb, d_to, n, exact=True)
        ctx.csr_row_lengths(res, d_lens + r * n * 4)
        parts.append(res)
        total += res.nnz
        if len(gids):  # global ids resolve to the shard's own filter bytes
            g = int(gids[0])
            assert idx.filter(g) == sorted(set(filters))[g]
    d_ids = ctx.dev_alloc(max(total, 1) * 4)
    off = 0
    for res in parts:
        import ctypes as C
        ctx.memcpy_d2d(d_ids + off * 4, C.cast(res.csr.ids, C.c_void_p).value or 0, res.nnz * 4)
        off += res.nnz
        res.free()
    merged = ctx.merge_rows(n, n, shards, d_lens, d_ids)
    ro, ids = merged.to_host()
    assert np.array_equal(ro, fro) and np.array_equal(ids, fids)
    oro, oids = _oracle_rows(orc, filters, tb, to)
    assert np.array_equal(ro, oro) and np.array_equal(ids, oids)
    merged.free()
    from emqx_amd import GpuMatchError
    with pytest.raises(GpuMatchError, match="EUNSUPPORTED"):
        ctx.fanout(idxs[0], ro[:2].copy() * 0, np.zeros(0, np.uint32))
    for idx in idxs:
        idx.release()
    full.release()
    for p in (d_tb, d_to, d_lens, d_ids):
        ctx.dev_free(p)


def test_shard_global_ids_must_follow_byte_order(ctx):
    from emqx_amd import GpuMatchError
    with pytest.raises(GpuMatchError, match="ascend"):
        ctx.build_index_shard([b"a/#", b"b/+"], np.array([5, 2], np.uint32))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))

    def mark(msg):
        with open(os.path.join(out_dir, f"log{rank}"), "a") as f:
            f.write(msg + "\n")
    import torch.distributed as dist
    from emqx_amd import Context
    from emqx_amd.engine import pack
    from emqx_amd.sharded import ShardedMatcher, plan_shard
    from oracle import oracle as orc
    mark("init")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mark("pg")
    ctx = Context(0)
    mark("ctx")
    try:
        filters, topics = _sets("c1")
        fb, fo = pack(filters)
        tb, to = pack(topics)
        sfb, sfo, gids, _ = plan_shard(fb, fo, world, rank)
        idx = ctx.build_index_shard((sfb, sfo), gids)
        d_tb, d_to = _to_device(ctx, tb, to)
        mark("index")
        m = ShardedMatcher(ctx, idx, world, rank, dist=dist, device_tensors=False)
        res, first, rows = m.match_device(d_tb, d_to, len(topics))
        mark("matched")
        ro, ids = res.to_host()
        oro, oids = _oracle_rows(orc, filters, tb, to)
        for k in range(rows):
            t = first + k
            assert ids[ro[k]:ro[k + 1]].tolist() == oids[oro[t]:oro[t + 1]].tolist(), (rank, t)
        res.free()
        idx.release()
        ctx.dev_free(d_tb)
        ctx.dev_free(d_to)
        open(os.path.join(out_dir, f"ok{rank}"), "w").write(str(rows))
    finally:
        ctx.close()
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_sharded_matcher_two_ranks_gloo(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert sorted(x for x in os.listdir(tmp_path) if x.startswith("ok")) == ["ok0", "ok1"]


def test_device_tensor_path_with_replayed_exchange():
    """ShardedMatcher(device_tensors=True) -- the RCCL code path: the library on
    torch's stream, row lengths and ids in device tensors, bounds from one
    device reduction, the device merge -- run for both ranks of a 2-way shard
    on one device, with the collective itself replayed from the other rank's
    recorded send buffers (two ranks cannot share one GPU under RCCL).  Rank
    0's merged slice must equal the unsharded index and the oracle.  Runs in
    its own process with torch's device runtime initialised first, the order
    bench.py uses (tests/_sharded_device_worker.py)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "tests", "_sharded_device_worker.py")], cwd=root,
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "SHARDED_DEVICE_PATH_OK" in p.stdout


# ---------------------------------------------------------------------------
# prefix sharding (gm_route.hip)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("kind", ["random", "c1"])
def test_device_route_equals_host_route(ctx, kind):
    """emqx_gm_route_topics (one thread per topic) == emqx_gm_route_topics_host."""
    from emqx_amd.engine import pack, prefix_plan
    fs, ts = _sets(kind)
    fb, fo = pack(fs)
    tb, to = pack(ts)
    for world in (2, 3, 8):
        _, route = prefix_plan(fb, fo, world)
        d_tb, d_to = _to_device(ctx, tb, to)
        n = len(to) - 1
        d_dest = ctx.dev_alloc(max(n, 1) * 4)
        ctx.route_topics(route, d_tb, d_to, n, d_dest)
        got = np.zeros(max(n, 1), np.uint32)
        ctx.memcpy_d2h(got, d_dest, n * 4)
        assert np.array_equal(got[:n], route.route_host(tb, to))
        for p in (d_tb, d_to, d_dest):
            ctx.dev_free(p)
        route.release()


@pytest.mark.parametrize("kind", ["random", "c1"])
def test_route_partition_is_a_stable_sort_by_shard(ctx, kind):
    """emqx_gm_route_partition (a counting sort by shard) == a stable argsort of
    the host route's shards; the lengths follow the order; the split sizes are
    the per-shard topic and byte counts.  Batches past one 1,024-topic block,
    worlds 1 to 256, an empty batch."""
    from emqx_amd.engine import pack, prefix_plan
    fs, ts = _sets(kind)
    fb, fo = pack(fs)
    ts = ts * max(1, 5000 // max(len(ts), 1))  # several partition blocks
    tb, to = pack(ts)
    n = len(to) - 1
    lens = np.diff(to.astype(np.int64))
    for world in (1, 2, 3, 8, 256):
        _, route = prefix_plan(fb, fo, world)
        want_dest = route.route_host(tb, to).astype(np.int64)
        order = np.argsort(want_dest, kind="stable")
        d_tb, d_to = _to_device(ctx, tb, to)
        d_perm, d_plen, d_split = ctx.dev_alloc(n * 4), ctx.dev_alloc(n * 4), ctx.dev_alloc(16 * world)
        ctx.route_partition(route, d_tb, d_to, n, d_perm, d_plen, d_split)
        perm, plen, split = np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(2 * world, np.uint64)
        ctx.memcpy_d2h(perm, d_perm, n * 4)
        ctx.memcpy_d2h(plen, d_plen, n * 4)
        ctx.memcpy_d2h(split, d_split, 16 * world)
        assert np.array_equal(perm, order) and np.array_equal(plen, lens[order])
        assert np.array_equal(split[0::2], np.bincount(want_dest, minlength=world))
        assert np.array_equal(split[1::2], np.bincount(want_dest, weights=lens, minlength=world).astype(np.uint64))
        ctx.route_partition(route, d_tb, d_to, 0, d_perm, d_plen, d_split)  # empty batch: zero sizes
        ctx.memcpy_d2h(split, d_split, 16 * world)
        assert not split.any()
        for p in (d_tb, d_to, d_perm, d_plen, d_split):
            ctx.dev_free(p)
        route.release()


@pytest.mark.timeout(600)
def test_prefix_shards_each_walk_their_routed_topics(ctx, orc):
    """C5-shaped set (4M mixed filters) in 8 prefix shards built one after
    another on one device: the batch is routed on the device, permuted so each
    shard's topics are one range (emqx_gm_permute_topics), each shard walks
    ONLY its range, and the rows put back in batch order
    (emqx_gm_unpermute_rows) equal the unsharded index's rows, row for row;
    a window is checked against the oracle."""
    from emqx_amd.engine import gen_filter_codes, render_codes
    from emqx_amd.sharded import plan_prefix_shard
    n_f, n, W = 4_000_000, 1_000_000, 8
    codes = gen_filter_codes(1, n_f)
    fb, fo = render_codes(codes)
    db, do, tot = ctx.gen_topics_device(codes, 1, 0, n)
    _, _, _, _, route = plan_prefix_shard(fb, fo, W, 0)
    d_dest = ctx.dev_alloc(n * 4)
    ctx.route_topics(route, db, do, n, d_dest)
    dest = np.zeros(n, np.uint32)
    ctx.memcpy_d2h(dest, d_dest, n * 4)
    perm = np.argsort(dest, kind="stable").astype(np.uint32)
    bnd = np.r_[0, np.cumsum(np.bincount(dest, minlength=W))].astype(np.int64)
    d_perm = ctx.dev_alloc(n * 4)
    ctx.memcpy_h2d(d_perm, perm, n * 4)
    d_pb, d_po = ctx.dev_alloc(tot + 64), ctx.dev_alloc((n + 1) * 8)
    ctx.permute_topics(db, do, n, d_perm, d_pb, d_po)
    lens, ids = [], []
    for q in range(W):
        sfb, sfo, gids, _, r_q = plan_prefix_shard(fb, fo, W, q)
        r_q.release()
        sidx = ctx.build_index_shard((sfb, sfo), gids)
        m = int(bnd[q + 1] - bnd[q])
        res = ctx.match_device(sidx, d_pb, d_po + 8 * int(bnd[q]), m, exact=True)  # only its own range
        ro, rid = res.rows(0, m)
        lens.append(np.diff(ro.astype(np.int64)).astype(np.uint32))
        ids.append(rid)
        res.free()
        sidx.release()
    lens, ids = np.concatenate(lens), np.concatenate(ids).astype(np.uint32)
    d_l, d_i = ctx.dev_alloc(n * 4), ctx.dev_alloc(max(len(ids), 1) * 4)
    ctx.memcpy_h2d(d_l, lens, n * 4)
    if len(ids):
        ctx.memcpy_h2d(d_i, ids, len(ids) * 4)
    back = ctx.unpermute_rows(n, d_perm, d_l, d_i)
    bro, bids = back.to_host()
    back.free()
    idx = ctx.build_index((fb, fo))
    full = ctx.match_device(idx, db, do, n, exact=True)
    fro, fids = full.to_host()
    full.free()
    assert np.array_equal(bro, fro) and np.array_equal(bids, fids)
    # each shard walked only its share: no shard more than twice its fair share
    assert int(np.diff(bnd).max()) < 2 * n // W
    tb, to = orc.render_codes(orc.gen_topic_codes(1, 0, 20_000, codes))
    r = orc.Router(True)
    r.add_routes((fb, fo))
    import bench
    oro, oids, _ = r.match_batch((tb, to), orc.Ranker(bench.sorted_unique(fb, fo)), mode=1, nthreads=8)
    assert np.array_equal(bro[:20_001], oro) and np.array_equal(bids[:int(oro[-1])], oids)
    for p in (db, do, d_dest, d_perm, d_pb, d_po, d_l, d_i):
        ctx.dev_free(p)
    idx.release()
    route.release()


@pytest.mark.parametrize("shape", ["short", "mixed", "long"])
def test_permute_and_unpermute_ragged_vs_numpy(ctx, shape):
    """k_gather_segs (the permute / unpermute copy): random permutations of
    ragged segments -- 1-byte topics, empty rows, segments at every byte
    alignment, blocks whose 256 segments pass the 32 KB LDS image (the
    element-by-element path) -- against numpy."""
    rng = np.random.default_rng({"short": 1, "mixed": 2, "long": 3}[shape])
    n = 50_000
    lens = {"short": rng.integers(1, 12, n), "mixed": np.where(rng.random(n) < 0.02, rng.integers(200, 2000, n),
                                                                 rng.integers(1, 60, n)),
            "long": rng.integers(100, 400, n)}[shape].astype(np.uint64)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    tb = rng.integers(0, 256, int(off[-1]) + 64).astype(np.uint8)
    perm = rng.permutation(n).astype(np.uint32)
    d_tb, d_to = _to_device(ctx, tb, off)
    d_perm = ctx.dev_alloc(n * 4)
    ctx.memcpy_h2d(d_perm, perm, n * 4)
    d_pb, d_po = ctx.dev_alloc(int(off[-1]) + 64), ctx.dev_alloc((n + 1) * 8)
    ctx.permute_topics(d_tb, d_to, n, d_perm, d_pb, d_po)
    pb, po = np.zeros(int(off[-1]), np.uint8), np.zeros(n + 1, np.uint64)
    ctx.memcpy_d2h(pb, d_pb, len(pb))
    ctx.memcpy_d2h(po, d_po, 8 * (n + 1))
    want = np.concatenate([tb[int(off[p]):int(off[p + 1])] for p in perm])
    assert np.array_equal(po[1:], np.cumsum(lens[perm])) and np.array_equal(pb, want)
    # rows: input row i (ragged, empty rows included) goes to output row perm[i]
    rlen = (rng.integers(0, 5, n) * (rng.random(n) < 0.7)).astype(np.uint32)
    if shape == "long":
        rlen = rng.integers(0, 300, n).astype(np.uint32)
    ids = rng.integers(0, 2**32, int(rlen.sum()), dtype=np.uint64).astype(np.uint32)
    d_l, d_i = ctx.dev_alloc(n * 4), ctx.dev_alloc(max(len(ids), 1) * 4)
    ctx.memcpy_h2d(d_l, rlen, n * 4)
    ctx.memcpy_h2d(d_i, ids, len(ids) * 4)
    back = ctx.unpermute_rows(n, d_perm, d_l, d_i)
    ro, got = back.to_host()
    back.free()
    rin = np.r_[0, np.cumsum(rlen.astype(np.uint64))].astype(np.uint64)
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    want_ids = np.concatenate([ids[int(rin[i]):int(rin[i + 1])] for i in inv])
    assert np.array_equal(np.diff(ro.astype(np.int64)), rlen[inv].astype(np.int64)) and np.array_equal(got, want_ids)
    for p in (d_tb, d_to, d_perm, d_pb, d_po, d_l, d_i):
        ctx.dev_free(p)


@pytest.mark.timeout(300)
def test_permute_and_unpermute_past_2_pow_26_rows(ctx):
    """A C5 prefix rank permutes 100M topics: the permute/unpermute launches
    once gave each item a 64-lane wave, 64 * n work-items, past the dispatch's
    2^32 limit above 67,108,864 items, and silently copied only the first ones.
    70M topics reversed twice give the batch back byte for byte; 70M one-id rows
    unpermuted by the reversal give the ids reversed."""
    from emqx_amd.engine import gen_filter_codes
    n = 70_000_000
    codes = gen_filter_codes(5, 1000)
    db, do, tot = ctx.gen_topics_device(codes, 5, 0, n)
    rev = np.arange(n - 1, -1, -1, dtype=np.uint32)
    d_perm = ctx.dev_alloc(n * 4)
    ctx.memcpy_h2d(d_perm, rev, n * 4)
    d_pb, d_po = ctx.dev_alloc(tot + 64), ctx.dev_alloc((n + 1) * 8)
    d_pb2, d_po2 = ctx.dev_alloc(tot + 64), ctx.dev_alloc((n + 1) * 8)
    ctx.permute_topics(db, do, n, d_perm, d_pb, d_po)
    tail = np.zeros(2, np.uint64)  # the last permuted topic = the first generated one
    ctx.memcpy_d2h(tail, d_po + 8 * (n - 1), 16)
    first = np.zeros(2, np.uint64)
    ctx.memcpy_d2h(first, do, 16)
    assert int(tail[1] - tail[0]) == int(first[1] - first[0]) and int(tail[1]) == tot
    ctx.permute_topics(d_pb, d_po, n, d_perm, d_pb2, d_po2)
    a, b = np.zeros(tot, np.uint8), np.zeros(tot, np.uint8)
    ctx.memcpy_d2h(a, db, tot)
    ctx.memcpy_d2h(b, d_pb2, tot)
    assert np.array_equal(a, b)
    del a, b
    oa, ob = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
    ctx.memcpy_d2h(oa, do, 8 * (n + 1))
    ctx.memcpy_d2h(ob, d_po2, 8 * (n + 1))
    assert np.array_equal(oa, ob)
    del oa, ob
    for p in (db, do, d_pb, d_po, d_pb2, d_po2):
        ctx.dev_free(p)
    d_l, d_i = ctx.dev_alloc(n * 4), ctx.dev_alloc(n * 4)
    ctx.memcpy_h2d(d_l, np.ones(n, np.uint32), n * 4)
    ctx.memcpy_h2d(d_i, np.arange(n, dtype=np.uint32), n * 4)
    back = ctx.unpermute_rows(n, d_perm, d_l, d_i)
    ro, ids = back.to_host()
    back.free()
    assert np.array_equal(ro, np.arange(n + 1, dtype=np.uint64)) and np.array_equal(ids, rev)
    for p in (d_perm, d_l, d_i):
        ctx.dev_free(p)


def _run_worker(script, *args, timeout=560):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "tests", script)] + [str(a) for a in args],
                       cwd=root, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p.stdout


@pytest.mark.timeout(300)
def test_prefix_device_path_world1():
    """PrefixShardedMatcher.match_device at world 1 (the nccl bench's 1-GPU
    path): the library on the matcher's own stream, route -> torch.sort /
    bincount -> permute -> walk -> unpermute, rows == the unsharded index and
    the oracle (tests/_prefix_device_worker.py)."""
    assert "PREFIX_DEVICE_PATH_OK world=1" in _run_worker("_prefix_device_worker.py", 1, 200_000, 300_000)


def test_prefix_device_path_library_first_default_stream_inputs():
    """The library's Context made before anything touches torch's device
    (PrefixShardedMatcher then failed with "No HIP GPUs are
    available"; emqx_amd.Context now brings torch's runtime up first), and the
    topics written by torch ops on torch's default stream with non-blocking
    copies (the matcher's stream waits for the caller's, the
    caller's for the matcher's rows): rows == the unsharded index == the oracle."""
    out = _run_worker("_prefix_device_worker.py", 1, 200_000, 300_000, "libfirst")
    assert "PREFIX_DEVICE_PATH_OK world=1" in out and "libfirst" in out


@pytest.mark.parametrize("order", ["lib_first", "torch_first", "ctx_first"])
def test_one_hip_runtime_whatever_the_order(order):
    """A host-only library call before the first Context (the order of
    __graft_entry__.smoke: gen_filter_codes, then Context) used to load
    /opt/rocm's HIP runtime beside torch's own copy; torch came up first on its
    copy and emqx_gm_open then found no device (round 5 smoke: EDEVICE).  The
    library now binds to torch's runtime in every order: the context opens and
    one libamdhip64 is mapped (scripts/smoke_order_diag.py)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "scripts", "smoke_order_diag.py"), order], cwd=root,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and f"{order} open ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]
    assert f"{order} hip runtimes: 1" in p.stdout, p.stdout[-2000:]


def test_graft_smoke_in_a_fresh_process():
    """The driver's smoke(), as the driver runs it: a fresh interpreter."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-u", "-c", "import __graft_entry__ as g; g.smoke()"], cwd=root,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and "smoke ok" in p.stdout, p.stdout[-2000:] + p.stderr[-2000:]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("chunks", [2, 1], ids=["chunked", "unchunked"])
def test_prefix_device_path_world8_lockstep(chunks):
    """The 4M-filter set in 8 prefix shards, 8 ranks as threads on one device,
    each with its own context, stream and 500k-topic batch; the
    all_to_all_single calls of a step run in lock step across the ranks (six
    unchunked; chunked -- the default, each chunk's exchange issued before the
    previous chunk's walk -- one for the sizes plus five per chunk).  Every
    rank's rows == the unsharded index on its batch; rank 0's window == the
    oracle; no rank walks twice its share."""
    out = _run_worker("_prefix_device_worker.py", 8, 4_000_000, 500_000, f"chunks={chunks}")
    assert "PREFIX_DEVICE_PATH_OK world=8" in out and f"chunks={chunks}" in out
