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
    """The aggregator end to end on the GPU (emqx_amd/batcher.py, the mirror of
    nif/emqx_gpu_match_batcher.erl): GpuRoutes keeps ONE index over the route
    filters -- local subscribers as fan-out lists, remote-node and shared-group
    destinations as route marks -- derived by update_subs from the previous
    snapshot after every subscription change (never rebuilt); each publish's
    local deliveries equal the oracle's match_routes + dispatch fold, and its
    remote / shared routes come back as route entries (forward, shared
    dispatch) exactly for the filters the oracle matches."""
    from emqx_amd import Context
    from emqx_amd.batcher import GpuRoutes, PublishBatcher
    rng = np.random.default_rng(5)
    filters = sorted({b"a/#", b"a/+", b"a/b", b"+/b", b"#", b"c/d", b"a/+/c", b"$SYS/#", b"c/+", b"r/+", b"s/#"})
    topics = [b"a/b", b"a/x", b"c/d", b"q", b"a/b/c", b"$SYS/a", b"c/e", b"a/+", b"r/1", b"s/x/y"] * 40
    with Context(0) as ctx:
        routes = GpuRoutes(ctx)
        local = {f: set() for f in filters}       # filter -> local subscriber names
        other = {f: [] for f in filters}          # filter -> non-local destinations
        for f in filters:
            if f in (b"r/+",):
                continue  # a remote-only filter
            for sname in sorted(set(rng.integers(0, 300, size=int(rng.integers(0, 30))).tolist())):
                routes.subscribe(f, sname)
                local[f].add(sname)
        for f, d in [(b"r/+", b"n2"), (b"a/+", b"n2"), (b"a/+", b"n3"), (b"s/#", (b"g1", b"node")),
                     (b"s/#", (b"g1", b"n2")), (b"c/d", (b"g2", b"n3"))]:
            routes.route_add(f, d)
            other[f].append(d)
        inbox = {k: [] for k in range(300)}
        fwd, shared = [], []

        def run(tag):
            b = PublishBatcher(routes.groups, max_batch=64, window_s=0.002, subscribers=routes.subs,
                               deliver=lambda sub, f, m: inbox[sub].append((f, m)) or True,
                               lookup_routes=lambda f: ([b"node"] if local[f] else []) + other[f],
                               others=routes.other,
                               forward=lambda n, f, m: fwd.append((n, f, m)) or ("ok", 1),
                               shared_dispatch=lambda g, f, m: shared.append((g, f, m)) or ("ok", 1))
            for box in inbox.values():
                box.clear()
            fwd.clear()
            shared.clear()
            res = b.publish_batch([(t, (tag, k)) for k, t in enumerate(topics)])
            b.close()
            live = sorted(f for f in filters if local[f] or other[f])
            r = orc.Router(True)
            for f in live:
                r.add_route(f)
            oro, oids, _ = r.match_batch(topics, live, mode=1)
            for k, t in enumerate(topics):
                matched = [live[i] for i in oids[oro[k]:oro[k + 1]]]
                want = [(b"node", f, ("ok", len(local[f]))) for f in matched if local[f]]
                want += [(d, f, ("ok", 1)) for f in matched for d in other[f] if not isinstance(d, tuple)]
                want += [("share", f, ("ok", 1)) for f in matched for g in sorted({d[0] for d in other[f]
                                                                                 if isinstance(d, tuple)})]
                assert sorted(res[k], key=repr) == sorted(want, key=repr), t
                for f in matched:
                    for d in other[f]:
                        if isinstance(d, tuple):
                            continue
                        assert (d, f, (tag, k)) in fwd
            got = sorted((s, m) for s, box in inbox.items() for _, m in box)
            exp = sorted((s, (tag, k)) for k, t in enumerate(topics)
                         for i in oids[oro[k]:oro[k + 1]] for s in local[live[i]])
            assert got == exp

        run("first")
        u0 = routes.updates
        # subscription changes between batches: a last local subscriber leaving a
        # filter that keeps a remote route, a new filter, a remote route dropped
        for sname in sorted(local[b"a/+"]):
            routes.unsubscribe(b"a/+", sname)
        local[b"a/+"].clear()
        routes.subscribe(b"new/+", 7)
        filters.append(b"new/+")
        local[b"new/+"], other[b"new/+"] = {7}, []
        routes.route_delete(b"r/+", b"n2")
        other[b"r/+"] = []
        topics += [b"new/1"] * 5
        run("second")
        assert routes.updates == u0 + 1 and routes.builds == 1  # one update_subs, no rebuild
        assert routes.index.n_filters == len([f for f in filters if local[f] or other[f]])
