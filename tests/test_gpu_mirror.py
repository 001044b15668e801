"""Host mirrors over the GPU engine: Router/Trie snapshots derived by
incremental updates, the persistent-session router, and batch rule/authz
topic matching -- each checked against the oracle (or the emqx_topic:match/2
predicate it restates)."""

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


def test_router_incremental_snapshots_vs_oracle(ctx, orc):
    from emqx_amd import Router
    from tests.test_gpu_parity import _rand_filter, _rand_topic
    rng = random.Random(3)
    r = Router(ctx)
    o = orc.Router(True)
    live = []
    topics = [_rand_topic(rng) for _ in range(300)]
    for rnd in range(8):
        for _ in range(rng.randint(5, 80)):
            if live and rng.random() < 0.35:
                f, d = live.pop(rng.randrange(len(live)))
                r.delete_route(f, d)
                o.delete_route(f, d)
            else:
                f, d = _rand_filter(rng), rng.choice([b"n1", b"n2"])
                r.add_route(f, d)
                o.add_route(f, d)
                live.append((f, d))
        for t in topics:
            assert sorted(r.match_routes(t)) == sorted(o.match_routes(t)), (rnd, t)


def test_session_router_vs_oracle(ctx, orc):
    from emqx_amd import SessionRouter
    s = SessionRouter(ctx)
    o = orc.Router(True)
    subs = [("device/+/temp", b"s1"), ("device/#", b"s2"), ("device/7/temp", b"s3"), ("device/+/temp", b"s4"),
            ("$SYS/#", b"s5"), ("#", b"s6")]
    for f, sid in subs:
        s.add_route(f, sid)
        o.add_route(f, sid)
    for t in ["device/7/temp", "device/8/temp", "device", "$SYS/x", "other"]:
        assert sorted(s.match_routes(t)) == sorted(o.match_routes(t)), t
    s.delete_route("device/+/temp", b"s1")
    o.delete_route("device/+/temp", b"s1")
    assert sorted(s.match_routes("device/7/temp")) == sorted(o.match_routes("device/7/temp"))


def test_topic_rule_index_vs_predicate(ctx, orc):
    from emqx_amd import TopicRuleIndex
    from tests.test_gpu_parity import _rand_filter, _rand_topic
    rng = random.Random(9)
    rules = []
    for _ in range(60):
        fs = []
        for _ in range(rng.randint(1, 4)):
            f = _rand_filter(rng)
            fs.append(("eq", f) if rng.random() < 0.2 else f)
        rules.append(fs)
    idx = TopicRuleIndex(ctx, rules)
    topics = [t for t in (_rand_topic(rng) for _ in range(800)) if not orc.wildcard(t)]

    def hit(t, f):
        if isinstance(f, tuple):
            return f[1] == t  # {eq, F}: literal equality (emqx_authz_rule.erl:177-178)
        return orc.topic_match(t, f)

    expect = [[i for i, fs in enumerate(rules) if any(hit(t, f) for f in fs)] for t in topics]
    assert idx.rules_for_topics(topics) == expect
    eligible = [rng.random() < 0.5 for _ in rules]
    firsts = idx.first_match(topics, eligible)
    assert firsts == [next((i for i in row if eligible[i]), -1) for row in expect]
    with pytest.raises(ValueError):
        idx.rules_for_topics(["a/+"])
    idx.release()


@pytest.mark.gpu
def test_publish_batcher_c_abi_sequence_vs_oracle(orc):
    """The NIF's fanout_batch/2 sequence (index built with subscriber lists ->
    emqx_gm_match WITH_EXACT -> emqx_gm_fanout -> rows cut into per-filter
    groups by emqx_gm_index_subscriber_count) behind the aggregator: every
    publish's deliveries equal the oracle's dispatch fold, group by group."""
    from emqx_amd import Context
    from emqx_amd.batcher import FanoutGroups, PublishBatcher
    rng = np.random.default_rng(5)
    filters = sorted({b"a/#", b"a/+", b"a/b", b"+/b", b"#", b"c/d", b"a/+/c", b"$SYS/#", b"c/+"})
    subs = [sorted(set(rng.integers(0, 500, size=int(rng.integers(0, 40))).tolist())) for _ in filters]
    topics = [b"a/b", b"a/x", b"c/d", b"q", b"a/b/c", b"$SYS/a", b"c/e", b"a/+"] * 40
    with Context(0) as ctx:
        idx = ctx.build_index(filters, subs=subs)
        inbox = {i: [] for i in range(500)}
        b = PublishBatcher(FanoutGroups(ctx, idx, filters), max_batch=64, window_s=0.002, subscribers=inbox)
        futs = [b.publish(t, k) for k, t in enumerate(topics)]
        results = [f.result(timeout=60) for f in futs]
        b.close()
        assert b.batches >= len(topics) // 64
        r = orc.Router(True)
        for f in filters:
            r.add_route(f)
        oro, oids, _ = r.match_batch(topics, filters, mode=1)
        so = np.zeros(len(filters) + 1, np.uint64)
        so[1:] = np.cumsum([len(s) for s in subs])
        si = np.array([x for s in subs for x in s] or [0], np.uint32)
        ero, eids = orc.fanout(oro, oids, so, si)
        for k, t in enumerate(topics):
            want = [(filters[f], ("ok", len(subs[f])) if subs[f] else ("error", "no_subscribers"))
                    for f in oids[oro[k]:oro[k + 1]]]
            assert results[k] == want, t
        got = sorted((sid, k) for sid, box in inbox.items() for _, k in box)
        exp = sorted((int(s), k) for k in range(len(topics)) for s in eids[ero[k]:ero[k + 1]])
        assert got == exp
        idx.release()
