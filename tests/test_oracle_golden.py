"""Pin the CPU oracle against the reference's own known-answer vectors.

Every case comes from tests/golden/suite_vectors.json, which transcribes the
assertions of apps/emqx/test/emqx_trie_SUITE.erl, emqx_topic_SUITE.erl,
emqx_router_SUITE.erl, emqx_broker_SUITE.erl and the EUnit block of
apps/emqx/src/emqx_trie.erl.  Trie cases run in both compaction modes, as the
reference suite does (emqx_trie_SUITE.erl:25-39).
"""

import pytest


def B(s):
    return s.encode()


@pytest.mark.parametrize("compact", [True, False], ids=["compact", "not_compact"])
def test_trie_suite(orc, golden, compact):
    for case in golden["trie_cases"]:
        t = orc.Trie(compact)
        for op, arg in case["ops"]:
            getattr(t, op)(arg)
        for q in case["queries"]:
            got = sorted(t.match(q["topic"]))
            if "expect_len" in q:
                assert len(got) == q["expect_len"], (case["name"], q, got)
            else:
                assert got == sorted(B(x) for x in q["expect"]), (case["name"], q, got)
        for q in case.get("lookup_topic", []):
            assert t.lookup_topic(q["topic"]) == [B(x) for x in q["expect"]], case["name"]


@pytest.mark.parametrize("compact", [True, False], ids=["compact", "not_compact"])
def test_trie_empty(orc, golden, compact):
    t = orc.Trie(compact)
    for step in golden["trie_empty"]["steps"]:
        if step[0] == "check":
            assert t.empty() == step[1]
        else:
            getattr(t, step[0])(step[1])


@pytest.mark.parametrize("mode", ["compact", "not_compact"])
def test_make_keys(orc, golden, mode):
    compact = mode == "compact"
    for topic, topic_key, prefixes in golden["make_keys"][mode]:
        t = orc.Trie(compact)
        t.insert(topic)
        keys = t.keys()
        assert (B(topic_key), 1, 1) in keys
        assert sorted(k for k, kind, _ in keys if kind == 0) == sorted(B(p) for p in prefixes)
        assert orc.make_prefixes(topic, compact) == [B(p) for p in prefixes]


@pytest.mark.parametrize("mode", ["compact", "not_compact"])
def test_make_prefixes(orc, golden, mode):
    for topic, expect in golden["make_prefixes"][mode]:
        assert orc.make_prefixes(topic, mode == "compact") == [B(p) for p in expect]


def test_do_compact(orc, golden):
    for topic, expect in golden["do_compact"]["cases"]:
        assert orc.do_compact(topic) == [B(p) for p in expect]


def test_topic_wildcard(orc, golden):
    for t, expect in golden["topic_wildcard"]["cases"]:
        assert orc.wildcard(t) == expect, t


def test_topic_match(orc, golden):
    for name, filt, expect in golden["topic_match"]["cases"]:
        assert orc.topic_match(name, filt) == expect, (name, filt)


def test_topic_words(orc, golden):
    for t, ws, kinds in golden["topic_words"]["cases"]:
        got = orc.words(t)
        exp = []
        for w, k in zip(ws, kinds):
            exp.append(w if k == "atom" else B(w))
        assert got == exp


def test_router_match_routes(orc, golden):
    g = golden["router_match_routes"]
    for compact in (True, False):
        r = orc.Router(compact)
        for f in g["routes"]:
            r.add_route(f)
        got = sorted(f for f, _ in r.match_routes(g["topic"]))
        assert got == sorted(B(x) for x in g["expect"])
        for f in g["routes"]:
            r.delete_route(f)
        assert r.match_routes(g["topic"]) == []
        assert r.trie.empty()


def test_router_topics(orc, golden):
    g = golden["router_topics"]
    r = orc.Router(True)
    for f in g["add"]:
        r.add_route(f)
    assert sorted(r.topics()) == sorted(B(x) for x in g["expect"])


def test_broker_cases(orc, golden):
    for case in golden["broker_cases"]:
        b = orc.Broker(True, schedulers=8)
        if case.get("force_shard"):
            # t_shard mocks get_sub_shard -> 1: pre-fill the per-topic sequence
            # past the 1024 threshold so the subscriber goes to a shard.
            for pid in range(10_000, 10_000 + 1024):
                b.subscribe(case["publish"] + "/__pad", pid)
            for i in range(1024):
                b.subscribe(case["subs"][0][0], 1_000_000 + i)
            b.subscribe(case["subs"][0][0], case["subs"][0][1])
            got = b.publish(case["publish"])
            assert case["subs"][0][1] in got
            assert b.shard_entries(case["subs"][0][0]) >= 1
            continue
        for topic, pid in case["subs"]:
            b.subscribe(topic, pid)
        got = sorted(b.publish(case["publish"]))
        assert got == sorted(case["expect_deliveries"]), case["name"]


def test_shard_threshold(orc, golden):
    """Subscribers past the 1024th of a topic go to shards; dispatch still
    delivers exactly once per subscriber (emqx_broker_helper.erl:82-86)."""
    b = orc.Broker(True, schedulers=2)
    pids = list(range(1, 3001))
    for p in pids:
        b.subscribe("hot/t", p)
    assert b.shard_entries("hot/t") > 0
    assert sorted(b.subscribers("hot/t")) == pids
    # idempotent re-subscribe (emqx_broker.erl:131-137)
    b.subscribe("hot/t", 5)
    assert sorted(b.publish("hot/t")) == pids
