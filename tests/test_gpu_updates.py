"""Incremental index maintenance on the GPU:
emqx_gm_index_update applies insert/delete sequences with the reference's
semantics (insert idempotent, delete only if present; emqx_trie.erl:107-136)
and returns a new snapshot whose rows equal a rebuild over the updated set,
while the previous snapshot keeps answering for the old set (RCU)."""

import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


def test_update_sequences_vs_oracle(ctx, orc):
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
        if rnd % 4 == 0:  # RCU: the previous snapshot still answers for the previous set
            _check(ctx, orc, idx, before, topics)
        idx.release()
        idx = new
    idx.release()


def test_update_c1_scale_and_compaction(ctx, orc):
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


def test_update_edges(ctx, orc):
    from emqx_amd import GpuMatchError
    idx = ctx.build_index([b"a/#", b"b"])
    same = ctx.update_index(idx, [(b"a/#", True), (b"zz", False)])  # no change: the same snapshot
    _check(ctx, orc, same, {b"a/#", b"b"}, [b"a/x", b"b", b"zz"])
    gone = ctx.update_index(idx, [(b"a/#", False), (b"b", False)])
    _check(ctx, orc, gone, set(), [b"a/x", b"b", b""])
    back = ctx.update_index(gone, [(b"b", True), (b"a/#", True), (b"+/+", True)])
    _check(ctx, orc, back, {b"a/#", b"b", b"+/+"}, [b"a/x", b"b", b"q/r", b"$SYS/x"])
    with pytest.raises(GpuMatchError, match="EUNSUPPORTED"):
        ctx.fanout(back, np.zeros(2, np.uint64), np.zeros(0, np.uint32))
    shard = ctx.build_index_shard([b"a/#"], np.array([3], np.uint32))
    with pytest.raises(GpuMatchError, match="EUNSUPPORTED"):
        ctx.update_index(shard, [(b"b", True)])
    for x in (idx, same, gone, back, shard):
        x.release()
