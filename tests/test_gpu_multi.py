"""Multi-device contexts (emqx_gm_opts.n_devices, SURVEY.md §8b: the open
options select the device list): one NIF context serving a node's GPUs, as the
reference's match_routes/1 runs in every publisher process on all schedulers at
once (apps/emqx/src/emqx_trie.erl:66-70, emqx_router.erl:128-145).

The one-GPU box rehearses it with device 0 listed more than once: each listed
entry is a replica with its own stream, pools and host pipeline, so every
piece of the multi-device path runs -- the replication of each snapshot
(build, in-place update, overlay update, subscriber update with and without
route changes, import), and a host batch spread over the replicas and put back
in batch order.  Peer copies between distinct GPUs are the same calls with two
device ordinals; they run on the driver's 8-GPU node.

Bar: bit-exact rows against the single-device context and the oracle."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx1():
    from emqx_amd import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx2():
    from emqx_amd import Context
    c = Context(devices=[0, 0])
    yield c
    c.close()


def _oracle_rows(orc, filters, topics):
    r = orc.Router(True)
    for f in filters:
        r.add_route(f)
    ro, ids, _ = r.match_batch(topics, filters, mode=1, nthreads=8)
    return ro, ids


def _eq(a, b, what=""):
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), what


def test_devices_and_bad_lists():
    from emqx_amd import Context, GpuMatchError
    with Context(devices=[0, 0, 0]) as c:
        assert c.devices == [0, 0, 0]
    with Context(0) as c:
        assert c.devices == [0]
    with pytest.raises(GpuMatchError):
        Context(devices=[0, 4096])
    with pytest.raises(ValueError):
        Context(devices=[0] * 9)


def test_c2_fixture_and_4m_batch_two_replicas(ctx1, ctx2, orc, monkeypatch):
    """The C2 index (1M wildcard filters) replicated twice on the one GPU; the
    committed C2 fixture (2,000 strided topics, in 1,024-topic chunks so both
    replicas serve it) and a 4M-topic host batch (~16 chunks of 256K, eight on
    each replica) give the single-device rows, which equal the oracle on a
    strided 200k-topic sample; page-locked input (emqx_gm_host_alloc: sent by
    DMA, no staging copy), pageable input and the bounce-buffer output all
    agree."""
    import json
    import os
    from emqx_amd.engine import gen_filter_codes, render_codes
    codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
    fpack = render_codes(codes)
    filters = sorted(set(orc.unpack(*fpack)))
    i1 = ctx1.build_index(fpack)
    i2 = ctx2.build_index(fpack)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config_c2.json")) as f:
        fx = json.load(f)
    monkeypatch.setenv("GM_HOST_CHUNK", "1024")
    ro, ids = ctx2.match(i2, [t.encode() for t in fx["topics"]], exact=True)
    monkeypatch.delenv("GM_HOST_CHUNK")
    got = [[filters[k].decode() for k in ids[ro[i]:ro[i + 1]]] for i in range(len(fx["topics"]))]
    assert got == fx["matches"]

    n = 4_000_000
    tb, to = orc.render_codes(orc.gen_topic_codes(1, 0, n, codes))
    want = ctx1.match(i1, (tb, to), exact=True)
    assert int(want[0][-1]) > 2 * n
    _eq(ctx2.match(i2, (tb, to), exact=True), want, "pageable input")
    pb = ctx2.host_alloc(len(tb))
    pb[:] = tb
    _eq(ctx2.match(i2, (pb, to), exact=True), want, "page-locked input")
    monkeypatch.setenv("GM_HOST_BOUNCE", "1")
    _eq(ctx2.match(i2, (pb, to), exact=True), want, "bounce-buffer output")
    monkeypatch.delenv("GM_HOST_BOUNCE")
    # the single-device context on the pipelined path and on the serial one agree too
    monkeypatch.setenv("GM_HOST_PIPE", "serial")
    _eq(ctx1.match(i1, (pb, to), exact=True), want, "serial path")
    monkeypatch.delenv("GM_HOST_PIPE")
    ctx2.host_free(pb)
    # the oracle on 20 strided windows of 10k topics
    r = orc.Router(True)
    r.add_routes(fpack)
    for s in np.linspace(0, n - 10_000, 20).astype(np.int64).tolist():
        wtb, wto = orc.render_codes(orc.gen_topic_codes(1, s, 10_000, codes))
        oro, oids, _ = r.match_batch((wtb, wto), filters, mode=1, nthreads=8)
        a, b = int(want[0][s]), int(want[0][s + 10_000])
        assert np.array_equal(want[0][s:s + 10_001] - want[0][s], oro), s
        assert np.array_equal(want[1][a:b], oids), s
    i1.release()
    i2.release()


def _same_tables(ix, k_max):
    """Every replica of a snapshot holds the first device's bytes (tables and
    subscriber CSR)."""
    d0 = ix.replica_digest(0)
    for k in range(1, k_max + 1):
        assert ix.replica_digest(k) == d0, k


def test_updates_replicated(ctx1, ctx2, orc, monkeypatch):
    """Every kind of new snapshot reaches every replica: an in-place patch
    (applied on each device from its own predecessor replica, O(delta): the
    replica's tables byte-equal to the first device's), an overlay update (a
    filter with '#' inside: stays on the first device, where it is matched),
    an import (copied); each snapshot's rows through the multi-device host path
    (forced into 1,024-topic chunks, so both replicas serve the batch) equal
    the oracle's."""
    import random
    rng = random.Random(11)
    words = ["a", "b", "c", "d", "+"]

    def rand_filter():
        k = rng.randint(1, 5)
        ws = [rng.choice(words) for _ in range(k)]
        if rng.random() < 0.3:
            ws.append("#")
        return "/".join(ws).encode()

    filters = sorted({rand_filter() for _ in range(300)})
    topics = ["/".join(rng.choice("abcde") for _ in range(rng.randint(1, 6))).encode() for _ in range(6000)]
    monkeypatch.setenv("GM_HOST_CHUNK", "1024")
    idx = ctx2.build_index(filters)
    live = set(filters)

    def check(ix):
        fl = sorted(live)
        ro, ids = ctx2.match(ix, topics, exact=True)
        oro, oids = _oracle_rows(orc, fl, topics)
        assert np.array_equal(ro, oro) and np.array_equal(ids, oids)

    check(idx)
    st = ctx2.update_stats()
    assert st["kind"] == "build" and st["replica_mode"] == "copied" and st["replicas"] == 1, st
    _same_tables(idx, 1)
    # an in-place patch: deletes and inserts of ordinary filters
    dels = rng.sample(sorted(live), 20)
    adds = sorted({rand_filter() for _ in range(30)} - live)
    ops = [(f, False) for f in dels] + [(f, True) for f in adds]
    nidx = ctx2.update_index(idx, ops)
    st = ctx2.update_stats()
    assert st["kind"] == "patch" and st["replica_mode"] == "patched" and st["replicas"] == 1, st
    live -= set(dels)
    live |= set(adds)
    check(nidx)
    _same_tables(nidx, 1)
    # a second patch continues the line on every device
    ops2 = [(sorted(live)[3], False), (b"q/+/z", True)]
    n2 = ctx2.update_index(nidx, ops2)
    live.discard(sorted(live)[3])
    live.add(b"q/+/z")
    assert ctx2.update_stats()["replica_mode"] == "patched"
    check(n2)
    _same_tables(n2, 1)
    nidx.release()
    nidx = n2
    check_old = sorted(set(filters))  # the old snapshot is untouched (RCU)
    ro, ids = ctx2.match(idx, topics, exact=True)
    oro, oids = _oracle_rows(orc, check_old, topics)
    assert np.array_equal(ro, oro) and np.array_equal(ids, oids)
    idx.release()
    # an overlay: a filter with '#' inside (matched on the first device only)
    ov = ctx2.update_index(nidx, [(b"a/#/b", True), (sorted(live)[0], False)])
    st = ctx2.update_stats()
    assert st["kind"] == "overlay" and st["replica_mode"] == "none", st
    live.add(b"a/#/b")
    live.discard(sorted(live - {b"a/#/b"})[0])
    check(ov)
    nidx.release()
    # import: the image replicated to both
    flat = ctx1.build_index(sorted(live - {b"a/#/b"}))
    imp = ctx2.import_index(flat.export())
    st = ctx2.update_stats()
    assert st["kind"] == "import" and st["replica_mode"] == "copied", st
    live.discard(b"a/#/b")
    check(imp)
    _same_tables(imp, 1)
    flat.release()
    ov.release()
    imp.release()


def test_update_cycle_reuses_blobs_on_every_replica(ctx2, orc, monkeypatch):
    """An update chain on a two-replica context: once the previous snapshot
    is released, its blob and its replica's blob are the spares the next
    update's two device passes take (gm_index.cpp take/give_spare_blob, one
    spare per open context on a device; GM_SPARE_BLOB_MIN=1: any size), with
    rows equal to the oracle after each update."""
    import random
    monkeypatch.setenv("GM_SPARE_BLOB_MIN", "1")
    monkeypatch.setenv("GM_HOST_CHUNK", "1024")
    rng = random.Random(5)
    live = {("/".join(rng.choice(["a", "b", "c", "+"]) for _ in range(rng.randint(1, 5)))).encode()
            for _ in range(2000)}
    topics = ["/".join(rng.choice("abc") for _ in range(rng.randint(1, 6))).encode() for _ in range(3000)]
    idx = ctx2.build_index(sorted(live))
    reused = []
    for it in range(4):
        adds = {b"cyc/%d/%d/+" % (it, i) for i in range(30)}
        ops = [(f, True) for f in sorted(adds)] + [(f, False) for f in sorted(live)[:10]]
        nidx = ctx2.update_index(idx, ops)
        st = ctx2.update_stats()
        assert st["replica_mode"] == "patched", st
        reused.append(st["blobs_reused"])
        live = (live - set(sorted(live)[:10])) | adds
        idx.release()  # (its blob and its replica's become the device's spares)
        idx = nidx
        ro, ids = ctx2.match(idx, topics, exact=True)
        oro, oids = _oracle_rows(orc, sorted(live), topics)
        assert np.array_equal(ro, oro) and np.array_equal(ids, oids), it
        _same_tables(idx, 1)
    assert reused[1:] == [2, 2, 2], reused
    idx.release()


def test_update_subs_replicated(ctx2, monkeypatch):
    """Subscriber maintenance on a two-replica context: a subscriber-only batch
    (the new snapshot shares its predecessor's tables; each replica shares its
    predecessor replica's and writes its own new subscriber CSR on its device)
    and a batch with route changes (patched on every device at once, each
    device's new CSR written there): the fan-out rows (match through the
    multi-device host path) equal the broker bookkeeping's deliveries -- each
    matching filter's subscribers/1 (emqx_broker.erl:296-322, 506-530) -- and
    every replica's tables and CSR equal the first device's, byte for byte."""
    from emqx_amd import topic
    from emqx_amd.routing import Broker
    monkeypatch.setenv("GM_HOST_CHUNK", "1024")
    b = Broker(ctx=ctx2)
    fl = [f"s/{i}/+".encode() for i in range(50)] + [f"s/{i}/x".encode() for i in range(50)] + [b"s/#"]
    for k, f in enumerate(fl):
        b.subscribe(f, k)
        b.subscribe(f, 1000 + k)
    topics = [f"s/{i % 60}/x".encode() for i in range(3000)]

    def check():
        got = b.publish_batch(topics)
        live = [f for f in fl + [b"s/+/x"] if b.subscribers(f)]
        for i in range(0, len(topics), 37):
            want = sorted(s for f in live if topic.match(topics[i], f) for s in b.subscribers(f))
            assert sorted(got[i]) == want, i

    check()
    for k in range(0, 40):  # subscriber-only: every filter keeps a subscriber
        b.unsubscribe(fl[k], 1000 + k)
        b.subscribe(fl[k], 5000 + k)
    check()
    st = ctx2.update_stats()
    assert st["kind"] == "subs_only" and st["replica_mode"] == "shared", st
    _same_tables(b.snapshot().index, 1)
    for k in range(40, 60):  # routes change: the last subscribers leave, a new filter comes
        b.unsubscribe(fl[k], k)
        b.unsubscribe(fl[k], 1000 + k)
    b.subscribe(b"s/+/x", 7)
    check()
    st = ctx2.update_stats()
    assert st["kind"] == "patch" and st["replica_mode"] == "patched", st
    _same_tables(b.snapshot().index, 1)


def test_concurrent_callers_three_replicas(orc, monkeypatch):
    """NIF-style use: one context over three replicas (device 0 listed three
    times) shared by four threads (dirty schedulers), each matching its own
    host batches -- small ones run whole on one replica picked round-robin
    under that replica's lock only, larger ones spread over the replicas in
    1,024-topic chunks -- while a fifth thread swaps in updated snapshots (RCU:
    each update is applied on all three replicas; the old snapshot is released
    as soon as it is swapped out, the callers' retained references keep it
    alive): every result equals the oracle's rows for the snapshot that call
    used."""
    import random
    import threading
    from emqx_amd import Context
    from emqx_amd._lib import lib
    monkeypatch.setenv("GM_HOST_CHUNK", "1024")
    rng = random.Random(3)
    words = ["a", "b", "c", "+"]
    base = sorted({"/".join(rng.choice(words) for _ in range(rng.randint(1, 4))).encode() for _ in range(200)})
    extra = [b"z/%d/#" % i for i in range(20)]
    topics = [["/".join(rng.choice("abcz") for _ in range(rng.randint(1, 5))).encode() for _ in range(k)]
              for k in (50, 700, 5000, 9000)]
    want = {}
    for fs_key, fs in (("base", base), ("more", sorted(base + extra))):
        for k, ts in enumerate(topics):
            want[(fs_key, k)] = _oracle_rows(orc, fs, ts)

    class _Held:  # a retained snapshot handle (emqx_gm_index_retain), released after the call
        def __init__(self, ix):
            lib().emqx_gm_index_retain(ix.h)
            self.h = ix.h

        def release(self):
            lib().emqx_gm_index_release(self.h)

    with Context(devices=[0, 0, 0]) as c:
        lock = threading.Lock()
        cur = {"key": "base", "ix": c.build_index(base)}
        errors, swaps = [], [0]
        stop = threading.Event()

        def caller(tid):
            try:
                for it in range(8):
                    with lock:
                        key, held = cur["key"], _Held(cur["ix"])
                    try:
                        k = (tid + it) % len(topics)
                        ro, ids = c.match(held, topics[k], exact=True)
                    finally:
                        held.release()
                    wro, wids = want[(key, k)]
                    if not (np.array_equal(ro, wro) and np.array_equal(ids, wids)):
                        errors.append((tid, it, key, k))
            except Exception as e:  # noqa: BLE001
                errors.append((tid, repr(e)))

        def updater():
            try:
                while not stop.is_set() and swaps[0] < 12:
                    with lock:
                        key, old = cur["key"], cur["ix"]
                    ops = [(f, key == "base") for f in extra]  # base -> more (insert), more -> base (delete)
                    nix = c.update_index(old, ops)
                    st = c.update_stats()
                    if st["replica_mode"] != "patched" or st["replicas"] != 2:
                        errors.append(("update", st))
                    with lock:
                        cur["key"], cur["ix"] = ("more" if key == "base" else "base"), nix
                    old.release()  # (callers holding it retained it)
                    swaps[0] += 1
            except Exception as e:  # noqa: BLE001
                errors.append(("updater", repr(e)))

        th = [threading.Thread(target=caller, args=(t,)) for t in range(4)]
        up = threading.Thread(target=updater)
        up.start()
        for t in th:
            t.start()
        for t in th:
            t.join()
        stop.set()
        up.join()
        assert not errors, errors
        assert swaps[0] >= 1
        cur["ix"].release()


@pytest.mark.skipif("not __import__('torch').cuda.device_count() >= 2", reason="needs two GPUs")
def test_two_gpus_replicas_and_small_calls(ctx1, orc, monkeypatch):
    """Devices [0, 1] (the driver's multi-GPU node): the tree copy crosses xGMI
    (hipMemcpyPeerAsync between two devices, peer access enabled at open), an
    in-place update is applied on both GPUs, a small call runs whole on either
    GPU (round-robin) and a large one is spread over both: every row equals
    the single-device context's, every replica's tables the first GPU's."""
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    codes = gen_filter_codes(7, 200_000)
    fpack = render_codes(codes)
    tb, to = orc.render_codes(orc.gen_topic_codes(7, 0, 600_000, codes))
    i1 = ctx1.build_index(fpack)
    want = ctx1.match(i1, (tb, to), exact=True)
    with Context(devices=[0, 1]) as c:
        ix = c.build_index(fpack)
        _same_tables(ix, 1)
        _eq(c.match(ix, (tb, to), exact=True), want, "spread over two GPUs")
        small = (tb, to[:2001].copy())
        ws = ctx1.match(i1, small, exact=True)
        for _ in range(4):  # round-robin: both GPUs serve small calls
            _eq(c.match(ix, small, exact=True), ws, "small call")
        ops = [(b"two/+/gpus/%d" % i, True) for i in range(100)]
        nx = c.update_index(ix, ops)
        assert c.update_stats()["replica_mode"] == "patched"
        _same_tables(nx, 1)
        n1 = ctx1.update_index(i1, ops)
        _eq(c.match(nx, (tb, to), exact=True), ctx1.match(n1, (tb, to), exact=True), "after the update")
        for x in (ix, nx, n1):
            x.release()
    i1.release()


@pytest.mark.parametrize("devices,chunk", [([0, 0], None), ([0, 0, 0], "4096")])
def test_sharded_index_behind_the_c_abi(ctx1, orc, monkeypatch, devices, chunk):
    """emqx_gm_index_build_sharded: the prefix plan behind ONE multi-device
    context (SURVEY §8e C5's sharded form, reachable from the NIF): filters
    partitioned by first word over the devices ('+' / '#'-first ones on every
    device), each topic matched on its one shard -- rows equal the unsharded
    single-device index's and the oracle's (global ids, batch order), with
    '$SYS', empty, wildcard and unknown-first-word topics, an empty batch and
    chunked shard batches; the fan-out of those rows equals the unsharded
    fan-out; the set-wide lookups answer for every filter; updates, images
    and device-buffer calls are refused."""
    from emqx_amd import Context, GpuMatchError
    from emqx_amd.engine import gen_filter_codes, render_codes
    if chunk:
        monkeypatch.setenv("GM_HOST_CHUNK", chunk)
    codes = gen_filter_codes(5, 60_000)
    fb, fo = render_codes(codes)
    extra = [b"#", b"+/x", b"$SYS/#", b"solo/word", b"solo/+/#"]
    filters = sorted(set(orc.unpack(fb, fo)) | set(extra))
    rng = np.random.default_rng(8)
    subs = [rng.integers(0, 10**6, size=int(rng.integers(0, 4))).tolist() for _ in filters]
    tb, to = orc.render_codes(orc.gen_topic_codes(5, 0, 200_000, codes))
    topics = orc.unpack(tb, to) + [b"$SYS/broker", b"", b"/", b"a/+", b"solo/word", b"solo/x/y", b"nosuch/1",
                                   b"+/x", b"l0w1"]
    i1 = ctx1.build_index(filters, subs=subs)
    want = ctx1.match(i1, topics, exact=True)
    wf = ctx1.fanout(i1, *want)
    oro, oids = _oracle_rows(orc, filters, topics[::97])
    with Context(devices=devices) as c:
        ix = c.build_index_sharded(filters, subs=subs)
        assert ix.n_filters == len(filters) and ix.info.n_subs == sum(len(x) for x in subs)
        assert ix.info.n_wildcard == i1.info.n_wildcard
        for f in (0, 7, len(filters) // 2, len(filters) - 1):
            assert ix.filter(f) == filters[f] and ix.subscriber_count(f) == len(subs[f])
        got = c.match(ix, topics, exact=True)
        _eq(got, want, "sharded rows")
        sub = [got[1][got[0][i]:got[0][i + 1]].tolist() for i in range(0, len(topics), 97)]
        assert sub == [oids[oro[j]:oro[j + 1]].tolist() for j in range(len(oro) - 1)]
        _eq(c.match(ix, topics, exact=False), ctx1.match(i1, topics, exact=False), "trie mode")
        _eq(c.fanout(ix, *got), wf, "sharded fan-out")
        e = c.match(ix, [], exact=True)
        assert e[0].tolist() == [0] and len(e[1]) == 0
        for bad in (lambda: c.update_index(ix, [(b"q/+", True)]), lambda: ix.export(),
                    lambda: c.match_device(ix, 0, 0, 0)):
            with pytest.raises(GpuMatchError):
                bad()
        ix.release()
    i1.release()


@pytest.mark.parametrize("replicas", [2, 3])
def test_fanout_spread_over_replicas(ctx1, orc, monkeypatch, replicas):
    """emqx_gm_fanout of host rows through a multi-device context: one slice of
    the rows per replica (balanced by matches), each fanned out on its device,
    the slices' deliveries put back in order into one result -- equal to the
    single-device fan-out and the oracle's dispatch fold, including empty rows,
    rows of one hot filter and slices that start and end anywhere; and
    emqx_gm_match_fanout's publish windows served by every replica in turn."""
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    monkeypatch.setenv("GM_FANOUT_MULTI_MIN", "1")
    codes = gen_filter_codes(5, 20_000)
    fb, fo = render_codes(codes)
    filters = sorted(set(orc.unpack(fb, fo)))
    rng = np.random.default_rng(2)
    subs = [rng.integers(0, 10**6, size=int(rng.integers(0, 6))).tolist() for _ in filters]
    subs[7] = list(range(5000))  # one hot filter
    tb, to = orc.render_codes(orc.gen_topic_codes(5, 0, 40_000, codes))
    i1 = ctx1.build_index(filters, subs=subs)
    ro, ids = ctx1.match(i1, (tb, to), exact=True)
    ids = ids.copy()
    ids[::97] = 7  # hot rows
    want = ctx1.fanout(i1, ro, ids)
    so = np.zeros(len(filters) + 1, np.uint64)
    so[1:] = np.cumsum([len(s) for s in subs])
    si = np.array([x for s in subs for x in s], np.uint32)
    oro, oids = orc.fanout(ro, ids, so, si)
    assert np.array_equal(want[0], oro) and np.array_equal(want[1], oids)
    with Context(devices=[0] * replicas) as c:
        ix = c.build_index(filters, subs=subs)
        got = c.fanout(ix, ro, ids)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
        e = np.zeros(1, np.uint64), np.zeros(0, np.uint32)  # no rows at all
        got0 = c.fanout(ix, *e)
        assert got0[0].tolist() == [0] and len(got0[1]) == 0
        # publish windows (match + fan-out in one round trip) round-robin over the replicas:
        # every device's replica gives the single-device rows and deliveries
        win = (tb, to[:2049])
        wro, wids = ctx1.match(i1, win, exact=True)
        wd = ctx1.fanout(i1, wro, wids)
        for _ in range(2 * replicas + 1):
            (mro, mids), (dro, dids) = c.match_fanout(ix, win)
            assert np.array_equal(mro, wro) and np.array_equal(mids, wids)
            assert np.array_equal(dro, wd[0]) and np.array_equal(dids, wd[1])
        ix.release()
    i1.release()
