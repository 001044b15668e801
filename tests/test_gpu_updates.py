"""Incremental index maintenance on the GPU:
emqx_gm_index_update applies insert/delete sequences with the reference's
semantics (insert idempotent, delete only if present; emqx_trie.erl:107-136)
and returns a new snapshot whose rows equal a rebuild over the updated set,
while the previous snapshot keeps answering for the old set (RCU).

Two forms (gm_overlay.cpp): the in-place patch (default: the newest plain
snapshot's tables patched on a device copy -> a flat snapshot, one match pass)
and the overlay (base + delta index, GM_UPDATE_OVERLAY=1, also the form taken
for a filter with '#' before its last word or an update of a superseded
snapshot)."""

import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["patch", "patch_mph", "patch_unfused", "overlay"])
def form(request, monkeypatch):
    # patch_unfused: the device side as copy, patch, renumber in place (the A/B
    # twin of the default one-pass copy-and-renumber, gm_match.hip apply_patch_device)
    if request.param == "patch_unfused":
        monkeypatch.setenv("GM_UPDATE_UNFUSED", "1")
    else:
        monkeypatch.delenv("GM_UPDATE_UNFUSED", raising=False)
    if request.param == "overlay":
        monkeypatch.setenv("GM_UPDATE_OVERLAY", "1")
    else:
        monkeypatch.delenv("GM_UPDATE_OVERLAY", raising=False)
    if request.param == "patch_mph":  # every per-depth table hash-and-displace placed: inserts take the overflow region
        monkeypatch.setenv("GM_MPH_MIN_KEYS", "1")
        monkeypatch.setenv("GM_CHAIN", "1")  # and chain nodes, which the patch turns back into plain nodes
    return "patch" if request.param in ("patch_mph", "patch_unfused") else request.param


def _is_flat(ctx, idx):
    """A flat snapshot answers fanout (no subscribers: zero deliveries); an
    overlay one refuses it (gm_api.cpp)."""
    from emqx_amd import GpuMatchError
    try:
        ctx.fanout(idx, np.zeros(2, np.uint64), np.zeros(0, np.uint32))
        return True
    except GpuMatchError as e:
        assert "EUNSUPPORTED" in str(e)
        return False


@pytest.fixture(scope="module")
def ctx():
    from emqx_amd import Context
    c = Context(0)
    yield c
    c.close()


def _oracle(orc, filters, topics, exact):
    from tests.test_gpu_parity import _oracle_rows
    return _oracle_rows(orc, sorted(filters), topics, 1 if exact else 0)


def _check(ctx, orc, idx, current, topics):
    for exact in (True, False):
        ro, ids = ctx.match(idx, topics, exact=exact)
        oro, oids = _oracle(orc, current, topics, exact)
        assert np.array_equal(ro, oro) and np.array_equal(ids, oids)
    assert idx.n_filters == len(current)
    assert idx.empty() == (not any(orc.wildcard(f) for f in current))


def _rand_ops(rng, current, k):
    from tests.test_gpu_parity import _rand_filter
    ops = []
    for _ in range(k):
        if current and rng.random() < 0.4:
            f, ins = rng.choice(sorted(current)), rng.random() < 0.3  # re-insert (no-op) or delete
        else:
            f, ins = _rand_filter(rng).encode(), rng.random() < 0.75  # new insert, or delete of an absent one
        ops.append((f, ins))
        if ins:
            current.add(f)
        else:
            current.discard(f)
    return ops


def test_update_sequences_vs_oracle(ctx, orc, form):
    from tests.test_gpu_parity import _rand_filter, _rand_topic
    rng = random.Random(21)
    current = {_rand_filter(rng).encode() for _ in range(500)}
    topics = [_rand_topic(rng).encode() for _ in range(2000)]
    idx = ctx.build_index(sorted(current))
    for rnd in range(12):
        before = set(current)
        ops = _rand_ops(rng, current, rng.randint(1, 60))
        new = ctx.update_index(idx, ops)
        _check(ctx, orc, new, current, topics)
        assert [new.filter(i) for i in range(new.n_filters)] == sorted(current)
        if new is not idx and form == "patch":
            assert _is_flat(ctx, new)
        if rnd % 4 == 0:  # RCU: the previous snapshot still answers for the previous set
            _check(ctx, orc, idx, before, topics)
        idx.release()
        idx = new
    idx.release()


def _blob(ctx, idx):
    ptr, nb = idx.device_blob()
    out = np.empty(nb, np.uint8)
    ctx.memcpy_d2h(out, ptr, nb)
    return out


def test_fused_update_equals_copy_patch_renumber(ctx, monkeypatch):
    """The one-pass device update (hot slots and nodes renumbered while copied,
    the patched ranges renumbered on the host by IdShift::map) writes the same
    device tables, byte for byte, as the copy + patch + in-place renumber
    (GM_UPDATE_UNFUSED): two imports of one image, the same ops on each,
    inserts and deletes spread over the id range (every id after the first
    change shifts)."""
    from tests.test_gpu_image import _workload
    monkeypatch.delenv("GM_UPDATE_OVERLAY", raising=False)
    fp, tp = _workload(30_000, 20_000)
    base = ctx.build_index(fp)
    img = base.export()
    rng = random.Random(5)
    from tests.test_gpu_parity import _rand_filter
    fb, fo = fp
    names = [bytes(fb[int(fo[i]):int(fo[i + 1])]) for i in range(0, len(fo) - 1, 97)]
    rounds = [[(f, False) for f in rng.sample(names, 40)] + [(_rand_filter(rng).encode(), True) for _ in range(60)],
              [(_rand_filter(rng).encode(), True) for _ in range(30)] + [(f, False) for f in rng.sample(names, 10)]]
    out = {}
    for mode in ("fused", "unfused"):
        if mode == "unfused":
            monkeypatch.setenv("GM_UPDATE_UNFUSED", "1")
        else:
            monkeypatch.delenv("GM_UPDATE_UNFUSED", raising=False)
        idx = ctx.import_index(img)
        for ops in rounds:
            new = ctx.update_index(idx, ops)
            assert _is_flat(ctx, new)
            idx.release()
            idx = new
        out[mode] = (_blob(ctx, idx), ctx.match(idx, tp, exact=True))
        idx.release()
    base.release()
    a, b = out["fused"], out["unfused"]
    assert a[0].nbytes == b[0].nbytes
    diff = np.flatnonzero(a[0] != b[0])
    assert diff.size == 0, f"{diff.size} bytes differ, first at {diff[:8]}"
    assert np.array_equal(a[1][0], b[1][0]) and np.array_equal(a[1][1], b[1][1])


def test_spare_blob_reuse_and_release_after_close(orc, monkeypatch):
    """A released snapshot's device blob is kept for the next in-place update
    of its size (gm_index.cpp take/give_spare_blob; GM_SPARE_BLOB_MIN=1: every
    blob, not only those of 256 MiB or more): a chain of updates reuses them
    with rows equal to the oracle after each; a snapshot released after its
    own context closed is freed (or kept while another context is open on the
    device: the module's), and a new context then updates normally."""
    from emqx_amd import Context
    from tests.test_gpu_parity import _rand_filter, _rand_topic
    monkeypatch.setenv("GM_SPARE_BLOB_MIN", "1")
    monkeypatch.delenv("GM_UPDATE_OVERLAY", raising=False)
    rng = random.Random(9)
    current = {_rand_filter(rng).encode() for _ in range(3000)}
    topics = [_rand_topic(rng).encode() for _ in range(2000)]
    c = Context(0)
    idx = c.build_index(sorted(current))
    for _ in range(6):
        new = c.update_index(idx, _rand_ops(rng, current, 40))
        idx.release()  # (its blob becomes the spare the next update takes)
        idx = new
        _check(c, orc, idx, current, topics)
    c.close()
    idx.release()  # after its context's close
    c2 = Context(0)
    idx = c2.build_index(sorted(current))
    new = c2.update_index(idx, _rand_ops(rng, current, 40))
    _check(c2, orc, new, current, topics)
    idx.release()
    new.release()
    c2.close()


def test_update_breaks_chain_nodes(ctx, orc, form, monkeypatch):
    """In-place updates through chain nodes (gm_common.h): a new branch below a
    chain node, its tail's filter deleted or re-inserted, a '+' child (whose
    inline record takes the chain's tail fields), a '#' child, a filter ending
    on the chain's middle node -- each patch must leave rows equal to the
    oracle (the patcher turns the chain node back into a plain node)."""
    from tests.test_gpu_parity import CHAIN_FILTERS, CHAIN_TOPICS
    monkeypatch.setenv("GM_CHAIN", "1")
    topics = [t.encode() for t in CHAIN_TOPICS] + [t.encode() + b"/x" for t in CHAIN_TOPICS] + [b"a/b/c/q", b"a/b/c/e"]
    current = {f.encode() for f in CHAIN_FILTERS}
    idx = ctx.build_index(sorted(current))
    steps = [
        [(b"a/b/c/e/g", True)],                      # a second leaf under the two-word chain's middle node
        [(b"a/b/x/y/z", False)],                     # the chain's own filter deleted
        [(b"a/b/x/y/z", True), (b"a/b/x/+", True)],  # re-inserted, and a '+' child of the chain node
        [(b"m/n/o/p/q/r", True)],                    # a filter on a chain's middle node
        [(b"w/1/#", True), (b"a/b/c/d", False)],
        [(b"a/b/c/q", True), (b"a/b/c/e/f", False)],
    ]
    for ops in steps:
        for f, ins in ops:
            (current.add if ins else current.discard)(f)
        new = ctx.update_index(idx, ops)
        _check(ctx, orc, new, current, topics)
        idx.release()
        idx = new
    idx.release()


def test_update_c1_scale_and_compaction(ctx, orc, form):
    from emqx_amd.engine import gen_filter_codes, render_codes
    from tests.test_gpu_parity import _rand_filter
    codes = gen_filter_codes(6, 20_000)
    base = set(orc.unpack(*render_codes(codes)))
    tb, to = orc.render_codes(orc.gen_topic_codes(6, 0, 30_000, codes))
    topics = orc.unpack(tb, to) + [b"$SYS/a", b"a/+", b""]
    idx = ctx.build_index(sorted(base))
    current = set(base)
    rng = random.Random(5)
    # small deltas: overlay snapshots
    for _ in range(3):
        ops = [(f, False) for f in rng.sample(sorted(current), 200)]
        extra = orc.unpack(*render_codes(gen_filter_codes(rng.randrange(1 << 30), 150)))
        ops += [(f, True) for f in extra]
        for f, ins in ops:
            if ins:
                current.add(f)
            else:
                current.discard(f)
        new = ctx.update_index(idx, ops)
        _check(ctx, orc, new, current, topics)
        idx.release()
        idx = new
    # a large delta: the flat rebuild
    ops = [(f, False) for f in rng.sample(sorted(current), 5000)] + [(_rand_filter(rng).encode(), True)
                                                                     for _ in range(100)]
    for f, ins in ops:
        if ins:
            current.add(f)
        else:
            current.discard(f)
    new = ctx.update_index(idx, ops)
    _check(ctx, orc, new, current, topics)
    idx.release()
    new.release()


def test_update_edges(ctx, orc, form):
    from emqx_amd import GpuMatchError
    idx = ctx.build_index([b"a/#", b"b"])
    same = ctx.update_index(idx, [(b"a/#", True), (b"zz", False)])  # no change: the same snapshot
    _check(ctx, orc, same, {b"a/#", b"b"}, [b"a/x", b"b", b"zz"])
    gone = ctx.update_index(idx, [(b"a/#", False), (b"b", False)])
    _check(ctx, orc, gone, set(), [b"a/x", b"b", b""])
    back = ctx.update_index(gone, [(b"b", True), (b"a/#", True), (b"+/+", True)])
    _check(ctx, orc, back, {b"a/#", b"b", b"+/+"}, [b"a/x", b"b", b"q/r", b"$SYS/x"])
    assert _is_flat(ctx, back) == (form == "patch")
    if form == "overlay":
        with pytest.raises(GpuMatchError, match="EUNSUPPORTED"):
            ctx.fanout(back, np.zeros(2, np.uint64), np.zeros(0, np.uint32))
    shard = ctx.build_index_shard([b"a/#"], np.array([3], np.uint32))
    with pytest.raises(GpuMatchError, match="EUNSUPPORTED"):
        ctx.update_index(shard, [(b"b", True)])
    for x in (idx, same, gone, back, shard):
        x.release()


TOPIC_WORDS = ["a", "b", "c", "", "$x", "long-word-over-8-bytes"]


def _deep_filter(rng, depth):
    ws = [rng.choice(TOPIC_WORDS + ["+"]) for _ in range(depth)]
    if rng.random() < 0.3:
        ws.append("#")
    return "/".join(ws).encode()


def test_patch_deep_root_inline_and_fallbacks(ctx, orc, monkeypatch):
    """The in-place patch across every table kind: filters deeper than the
    per-depth hot tables (the shared last table, the shared last edge table),
    '#' and '+' at the root, '+' under '+' (inline and slot records), words
    longer than the 8-byte dictionary head, the empty word; then the fallbacks:
    a filter with '#' before its last word -> overlay, an update of a
    superseded snapshot -> overlay, a delta too large for the tables' headroom
    -> rebuild (flat again, with a fresh mirror)."""
    monkeypatch.delenv("GM_UPDATE_OVERLAY", raising=False)
    rng = random.Random(77)
    current = {_deep_filter(rng, rng.randint(1, 22)) for _ in range(300)}
    topics = ["/".join(rng.choice(TOPIC_WORDS) for _ in range(rng.randint(1, 24))).encode() for _ in range(3000)]
    idx = ctx.build_index(sorted(current))
    steps = [
        [(b"#", True), (b"+", True), (b"+/+", True), (b"+/+/+/#", True)],
        [(_deep_filter(rng, rng.randint(14, 24)), True) for _ in range(40)],
        [(f, False) for f in rng.sample(sorted(current), 50)] + [(b"#", False)],
        [(b"long-word-over-8-bytes/+/long-word-over-8-bytes-2", True), (b"//+//#", True), (b"", True)],
    ]
    for ops in steps:
        for f, ins in ops:
            (current.add if ins else current.discard)(f)
        new = ctx.update_index(idx, ops)
        _check(ctx, orc, new, current, topics)
        assert _is_flat(ctx, new)
        idx.release()
        idx = new
    # '#' inside a filter: the overlay form
    ill = ctx.update_index(idx, [(b"a/#/b", True)])
    _check(ctx, orc, ill, current | {b"a/#/b"}, topics)
    assert not _is_flat(ctx, ill)
    ill.release()
    # the mirror moved on: an update of the superseded snapshot is an overlay
    newer = ctx.update_index(idx, [(b"q/r", True)])
    older = ctx.update_index(idx, [(b"q/s", True)])
    assert _is_flat(ctx, newer) and not _is_flat(ctx, older)
    _check(ctx, orc, older, current | {b"q/s"}, topics + [b"q/s", b"q/r"])
    older.release()
    idx.release()
    idx = newer
    current.add(b"q/r")
    # no headroom for 4,000 new filters over ~400: the flat rebuild
    ops = [(_deep_filter(rng, rng.randint(1, 8)), True) for _ in range(4000)]
    before = set(current)
    for f, _ in ops:
        current.add(f)
    new = ctx.update_index(idx, ops)
    _check(ctx, orc, new, current, topics)
    assert _is_flat(ctx, new)
    # the failed patch rolled idx's mirror back: idx still patches correctly
    again = ctx.update_index(idx, [(b"z/q/+", True), (b"a", False)])
    assert _is_flat(ctx, again)
    _check(ctx, orc, again, (before | {b"z/q/+"}) - {b"a"}, topics + [b"z/q/x"])
    again.release()
    idx.release()
    idx = new
    ops = [(b"z/+", True)]  # the rebuilt snapshot has a mirror again
    current.add(b"z/+")
    new = ctx.update_index(idx, ops)
    _check(ctx, orc, new, current, topics + [b"z/q"])
    assert _is_flat(ctx, new)
    idx.release()
    new.release()


@pytest.mark.timeout(600)
def test_patch_c2_scale_equals_rebuild(ctx, orc):
    """At C2 scale (1M wildcard filters), 2,000 deletes + 2,000 inserts patched
    in place: the patched snapshot's rows on 1M C2 topics are identical to a
    rebuilt index's (itself parity-checked against the oracle at this size in
    test_gpu_scale.py), in both match modes."""
    import time
    from emqx_amd.engine import gen_filter_codes, render_codes, pack
    os.environ.pop("GM_UPDATE_OVERLAY", None)
    codes = gen_filter_codes(1, 1_000_000, wildcard_only=True)
    fb, fo = render_codes(codes)
    idx = ctx.build_index((fb, fo))
    rng = random.Random(9)
    base = orc.unpack(fb, fo)
    dels = rng.sample(base, 2000)
    extra = orc.unpack(*render_codes(gen_filter_codes(77, 2000, wildcard_only=True)))
    ops = [(f, False) for f in dels] + [(f, True) for f in extra]
    t0 = time.perf_counter()
    new = ctx.update_index(idx, ops)
    t_upd = time.perf_counter() - t0
    assert _is_flat(ctx, new)
    current = (set(base) - set(dels)) | set(extra)
    flat = ctx.build_index(pack(sorted(current)))
    assert new.n_filters == flat.n_filters == len(current)
    tb, to = orc.render_codes(orc.gen_topic_codes(1, 0, 1_000_000, codes))
    for exact in (True, False):
        ra, ia = ctx.match(new, (tb, to), exact=exact)
        rb, ib = ctx.match(flat, (tb, to), exact=exact)
        assert np.array_equal(ra, rb) and np.array_equal(ia, ib)
    print(f"[patch_c2] update of {len(ops)} ops: {t_upd * 1e3:.1f} ms", flush=True)
    for x in (idx, new, flat):
        x.release()


class _Broker:
    """The reference's bookkeeping for the test: emqx_subscriber lists (a pair
    at most once, appended on subscribe) and the routed filters (a filter's
    first subscriber adds its route, the last one leaving deletes it;
    emqx_broker.erl:147-165, 445-454, emqx_router.erl:112-125, 164-172)."""

    def __init__(self, subs):
        self.lists = {f: list(l) for f, l in subs.items()}
        self.indexed = set(subs)
        # routed to another destination (a remote node, a shared group): a
        # filter built without local subscribers, or marked by route_add
        self.pinned = {f for f, l in subs.items() if not l}

    def apply(self, ops):
        touched = {f for f, _, _ in ops}
        for f, s, kind in ops:
            l = self.lists.setdefault(f, [])
            if kind == "route_add":
                self.pinned.add(f)
            elif kind == "route_delete":
                self.pinned.discard(f)
            elif kind and s not in l:
                l.append(s)
            elif not kind and s in l:
                l.remove(s)
        for f in touched:  # a route while a local subscriber or another destination holds it
            if self.lists.get(f) or f in self.pinned:
                self.indexed.add(f)
            else:
                self.indexed.discard(f)

    def csr(self):
        fs = sorted(self.indexed)
        so = np.zeros(len(fs) + 1, np.uint64)
        so[1:] = np.cumsum([len(self.lists.get(f, [])) for f in fs])
        si = np.array([x for f in fs for x in self.lists.get(f, [])], np.uint32)
        return fs, so, si


def _check_subs(ctx, orc, idx, br, topics):
    fs, so, si = br.csr()
    assert idx.n_filters == len(fs) and [idx.filter(i) for i in range(idx.n_filters)] == fs
    ro, ids = ctx.match(idx, topics, exact=True)
    oro, oids = _oracle(orc, set(fs), topics, True)
    assert np.array_equal(ro, oro) and np.array_equal(ids, oids)
    fro, fids = ctx.fanout(idx, ro, ids)
    ero, eids = orc.fanout(ro, ids, so, si)
    assert np.array_equal(fro, ero) and np.array_equal(fids, eids)
    for i in range(0, len(fs), max(1, len(fs) // 50)):
        assert idx.subscriber_count(i) == so[i + 1] - so[i]


def test_update_subs_vs_oracle(ctx, orc, monkeypatch):
    """emqx_gm_index_update_subs: random subscribe / unsubscribe batches (new
    filters, last subscribers leaving, re-subscribes, absent pairs) against
    the reference's bookkeeping; matches and fan-out rows vs the oracle after
    every batch; the previous snapshot keeps its own lists (RCU); then the
    rebuild fallbacks ('#' inside a filter, a superseded snapshot)."""
    from tests.test_gpu_parity import _rand_filter, _rand_topic
    monkeypatch.delenv("GM_UPDATE_OVERLAY", raising=False)
    rng = random.Random(41)
    subs = {}
    for _ in range(300):
        f = _rand_filter(rng).encode()
        subs[f] = rng.sample(range(5000), rng.randint(0, 6))  # some routes without local subscribers
    br = _Broker(subs)
    fs0 = sorted(subs)
    idx = ctx.build_index(fs0, subs=[subs[f] for f in fs0])
    topics = [_rand_topic(rng).encode() for _ in range(1500)]
    _check_subs(ctx, orc, idx, br, topics)
    for rnd in range(10):
        ops = []
        for _ in range(rng.randint(1, 80)):
            k = rng.random()
            if k < 0.35 and br.indexed:  # subscribe to a routed filter
                ops.append((rng.choice(sorted(br.indexed)), rng.randrange(5000), True))
            elif k < 0.6:  # a new filter's first subscriber (or an existing one)
                ops.append((_rand_filter(rng).encode(), rng.randrange(5000), True))
            elif k < 0.85 and br.lists:  # unsubscribe a present pair
                f = rng.choice(sorted(br.lists))
                if br.lists[f]:
                    ops.append((f, rng.choice(br.lists[f]), False))
            elif k < 0.92 and br.indexed:  # all subscribers of a filter leave: its route goes (unless pinned)
                f = rng.choice(sorted(br.indexed))
                ops += [(f, s, False) for s in list(br.lists.get(f, []))]
                ops.append((f, 99_999, False))  # an absent pair: no-op
            elif k < 0.96:  # another destination takes / holds a route (new or existing filter)
                f = rng.choice(sorted(br.indexed)) if br.indexed and rng.random() < 0.5 else _rand_filter(rng).encode()
                ops.append((f, 0, "route_add"))
            elif br.pinned:  # ... and leaves it
                ops.append((rng.choice(sorted(br.pinned)), 0, "route_delete"))
        prev_state = _Broker({})
        prev_state.lists = {f: list(l) for f, l in br.lists.items()}
        prev_state.indexed = set(br.indexed)
        prev_state.pinned = set(br.pinned)
        br.apply(ops)
        new = ctx.update_subs(idx, ops)
        _check_subs(ctx, orc, new, br, topics)
        if rnd % 3 == 0:  # RCU: the previous snapshot answers with its own lists
            _check_subs(ctx, orc, idx, prev_state, topics)
        idx.release()
        idx = new
    # subscriber-only batches (no route changes): the new snapshot shares the
    # previous one's tables; the previous one is released before the new one is
    # used, so the shared tables must outlive it
    for rnd in range(4):
        ops = []
        for f in rng.sample(sorted(f for f in br.indexed if br.lists.get(f)), 10):
            ops.append((f, 10_000 + rnd, True))
            if len(br.lists[f]) > 1:
                ops.append((f, br.lists[f][0], False))
        br.apply(ops)
        new = ctx.update_subs(idx, ops)
        idx.release()
        idx = new
        _check_subs(ctx, orc, idx, br, topics)
    # fallbacks: a filter with '#' inside, then an update of a superseded snapshot
    ops = [(b"a/#/b", 7, True)]
    br.apply(ops)
    new = ctx.update_subs(idx, ops)
    _check_subs(ctx, orc, new, br, topics + [b"a/x/b"])
    older_state = _Broker({})
    older_state.lists = {f: list(l) for f, l in br.lists.items()}
    older_state.indexed = set(br.indexed)
    older_state.pinned = set(br.pinned)
    newer = ctx.update_subs(new, [(b"z/z", 1, True)])
    older = ctx.update_subs(new, [(b"z/q", 2, True)])  # new has no mirror now: rebuilt
    older_state.apply([(b"z/q", 2, True)])
    _check_subs(ctx, orc, older, older_state, topics + [b"z/q"])
    for x in (idx, new, newer, older):
        x.release()
    with pytest.raises(Exception, match="EUNSUPPORTED"):
        plain = ctx.build_index([b"a"])
        try:
            ctx.update_subs(plain, [(b"a", 1, True)])
        finally:
            plain.release()


@pytest.mark.timeout(300)
def test_update_subs_hot_list(ctx, orc):
    """A C4-shaped hot filter (200k subscribers) loses 2,000 and gains 2,000
    in one batch: the untouched filters' lists are copied on the device, the
    hot one comes back from the host; every delivery vs the oracle."""
    K = 50
    filters = [b"hot/#"] + [b"hot/%d/x" % k for k in range(K)]
    subs = {b"hot/#": list(range(200_000))}
    for k in range(K):
        subs[b"hot/%d/x" % k] = list(range(300_000 + 10 * k, 300_000 + 10 * k + 10))
    br = _Broker(subs)
    fs0 = sorted(filters)
    idx = ctx.build_index(fs0, subs=[subs[f] for f in fs0])
    rng = random.Random(5)
    ops = [(b"hot/#", s, False) for s in rng.sample(range(200_000), 2000)]
    ops += [(b"hot/#", 500_000 + i, True) for i in range(2000)]
    ops += [(b"hot/%d/x" % k, 900_000 + k, True) for k in range(0, K, 7)]
    br.apply(ops)
    new = ctx.update_subs(idx, ops)
    topics = [b"hot/%d/x" % k for k in range(K)]
    _check_subs(ctx, orc, new, br, topics)
    idx.release()
    new.release()
