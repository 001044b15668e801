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


def test_updates_replicated(ctx1, ctx2, orc, monkeypatch):
    """Every kind of new snapshot reaches every replica: an in-place patch
    (copied), an overlay update (a filter with '#' inside: repeated on each
    replica), an import; each snapshot's rows through the multi-device host
    path (forced into 1,024-topic chunks, so both replicas serve the batch)
    equal the oracle's."""
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
    # an in-place patch: deletes and inserts of ordinary filters
    dels = rng.sample(sorted(live), 20)
    adds = sorted({rand_filter() for _ in range(30)} - live)
    ops = [(f, False) for f in dels] + [(f, True) for f in adds]
    nidx = ctx2.update_index(idx, ops)
    live -= set(dels)
    live |= set(adds)
    check(nidx)
    check_old = sorted(set(filters))  # the old snapshot is untouched (RCU)
    ro, ids = ctx2.match(idx, topics, exact=True)
    oro, oids = _oracle_rows(orc, check_old, topics)
    assert np.array_equal(ro, oro) and np.array_equal(ids, oids)
    idx.release()
    # an overlay: a filter with '#' inside
    ov = ctx2.update_index(nidx, [(b"a/#/b", True), (sorted(live)[0], False)])
    live.add(b"a/#/b")
    live.discard(sorted(live - {b"a/#/b"})[0])
    check(ov)
    nidx.release()
    # import: the image replicated to both
    flat = ctx1.build_index(sorted(live - {b"a/#/b"}))
    imp = ctx2.import_index(flat.export())
    live.discard(b"a/#/b")
    check(imp)
    flat.release()
    ov.release()
    imp.release()


def test_update_subs_replicated(ctx2, monkeypatch):
    """Subscriber maintenance on a two-replica context: a subscriber-only batch
    (the new snapshot shares its predecessor's tables; each replica shares its
    predecessor replica's and copies only the new subscriber CSR) and a batch
    with route changes (patched, then copied): the fan-out rows (match through
    the multi-device host path) equal the broker bookkeeping's deliveries --
    each matching filter's subscribers/1 (emqx_broker.erl:296-322, 506-530)."""
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
    for k in range(40, 60):  # routes change: the last subscribers leave, a new filter comes
        b.unsubscribe(fl[k], k)
        b.unsubscribe(fl[k], 1000 + k)
    b.subscribe(b"s/+/x", 7)
    check()


def test_concurrent_callers_three_replicas(orc, monkeypatch):
    """NIF-style use: one context over three replicas (device 0 listed three
    times) shared by four threads (dirty schedulers), each matching its own
    host batches -- some small (the one-chunk serial path), some spread over
    the replicas in 1,024-topic chunks -- while a fifth thread swaps in
    updated snapshots (RCU): every result equals the oracle's rows for the
    snapshot that call used."""
    import random
    import threading
    from emqx_amd import Context
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
    with Context(devices=[0, 0, 0]) as c:
        snaps = {"base": c.build_index(base)}
        snaps["more"] = c.update_index(snaps["base"], [(f, True) for f in extra])
        errors = []

        def caller(tid):
            try:
                for it in range(6):
                    key = "base" if (tid + it) % 2 else "more"
                    k = (tid + it) % len(topics)
                    ro, ids = c.match(snaps[key], topics[k], exact=True)
                    wro, wids = want[(key, k)]
                    if not (np.array_equal(ro, wro) and np.array_equal(ids, wids)):
                        errors.append((tid, it, key, k))
            except Exception as e:  # noqa: BLE001
                errors.append((tid, repr(e)))

        th = [threading.Thread(target=caller, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
        for s in snaps.values():
            s.release()


@pytest.mark.parametrize("replicas", [2, 3])
def test_fanout_spread_over_replicas(ctx1, orc, monkeypatch, replicas):
    """emqx_gm_fanout of host rows through a multi-device context: one slice of
    the rows per replica (balanced by matches), each fanned out on its device,
    the slices' deliveries put back in order into one result -- equal to the
    single-device fan-out and the oracle's dispatch fold, including empty rows,
    rows of one hot filter and slices that start and end anywhere."""
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
        ix.release()
    i1.release()
