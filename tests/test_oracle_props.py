"""Randomised agreement of the two independent oracle restatements:
the emqx_trie walk (both compaction modes) vs brute-force emqx_topic:match/2.

Generators follow the reference's PropEr shapes (apps/emqx/test/
emqx_proper_types.erl:314-338: '+' with probability 1/3 per level, or a
trailing '#'), plus '$'-topics, empty levels and deep topics.
"""

import random

import numpy as np
import pytest

ALPH = ["a", "b", "c", "", "$x", "$SYS", "dd"]


def rand_filter(rng):
    n = rng.randint(1, 5)
    ws = [rng.choice(ALPH) for _ in range(n)]
    kind = rng.random()
    if kind < 0.2:
        return "/".join(ws)
    if kind < 0.6:
        return "/".join("+" if rng.random() < 1 / 3 else w for w in ws)
    if kind < 0.8:
        return "/".join(ws[: rng.randint(0, n)] + ["#"])
    ws = ["+" if rng.random() < 1 / 3 else w for w in ws]
    return "/".join(ws + ["#"])


def rand_topic(rng):
    n = rng.randint(1, 6)
    ws = [rng.choice(ALPH) for _ in range(n)]
    if rng.random() < 0.05:
        ws[rng.randrange(n)] = rng.choice(["+", "#"])
    return "/".join(ws)


@pytest.mark.parametrize("seed", range(60))
def test_trie_walk_equals_bruteforce(orc, seed):
    rng = random.Random(seed)
    filters = sorted({rand_filter(rng).encode() for _ in range(rng.randint(1, 40))})
    topics = [rand_topic(rng).encode() for _ in range(40)]
    wild = np.array([orc.wildcard(f) for f in filters], np.uint8)
    for compact in (True, False):
        r = orc.Router(compact)
        for f in filters:
            r.add_route(f)
        # match_routes semantics
        ro, ids, _ = r.match_batch(topics, filters, mode=1)
        bro, bids = orc.bruteforce(topics, filters, mode=1)
        assert np.array_equal(ro, bro) and np.array_equal(ids, bids), (seed, compact)
        # emqx_trie:match/1 semantics over the wildcard filters in the trie
        ro, ids, _ = r.match_batch(topics, filters, mode=0)
        bro, bids = orc.bruteforce(topics, filters, mode=0, in_trie=wild)
        assert np.array_equal(ro, bro) and np.array_equal(ids, bids), (seed, compact)
        # no duplicates in any row
        for i in range(len(topics)):
            row = ids[ro[i]:ro[i + 1]]
            assert len(set(row.tolist())) == len(row)


def test_dollar_single_word_quirk(orc):
    """emqx_trie.erl:271-278: a single-word '$X' topic also looks up {'$X',1},
    so a non-wildcard '$X' inserted into the trie is returned."""
    for compact in (True, False):
        t = orc.Trie(compact)
        t.insert("$SYS")
        t.insert("$SYS/#")
        t.insert("plain")
        assert sorted(t.match("$SYS")) == [b"$SYS", b"$SYS/#"]
        assert t.match("plain") == []


def test_workload_generator_shapes(orc):
    codes = orc.gen_filter_codes(1, 2000, wildcard_only=False)
    data, off = orc.render_codes(codes)
    fs = orc.unpack(data, off)
    assert len(set(fs)) == len(fs)
    assert all(f.startswith(b"l0w") or f.startswith(b"+") for f in fs)
    w = orc.gen_filter_codes(1, 2000, wildcard_only=True)
    fw = orc.unpack(*orc.render_codes(w))
    assert all(orc.wildcard(f) for f in fw)
    tc = orc.gen_topic_codes(7, 0, 1000, codes)
    ts = orc.unpack(*orc.render_codes(tc))
    assert all(t.count(b"/") == 4 for t in ts)
    # counter-based: any window regenerates identically
    tc2 = orc.gen_topic_codes(7, 500, 10, codes)
    assert np.array_equal(tc[500:510], tc2)


@pytest.mark.parametrize("seed", range(30))
def test_cpu_nfa_equals_faithful_restatement(orc, seed):
    """The optimized CPU hash-NFA (oracle/cpu_nfa.cpp, the cpu_baseline leg's
    second figure) returns the faithful restatement's match_routes rows on the
    PropEr-shaped sets ('$' topics, empty levels, wildcard topics)."""
    rng = random.Random(1000 + seed)
    filters = sorted({rand_filter(rng).encode() for _ in range(rng.randint(1, 60))})
    topics = [rand_topic(rng).encode() for _ in range(200)] + [b"", b"/", b"#", b"+", b"$SYS", b"a//b"]
    r = orc.Router(True)
    for f in filters:
        r.add_route(f)
    ro, ids, _ = r.match_batch(topics, filters, mode=1)
    nfa = orc.CpuNfa(filters)
    nro, nids = nfa.match_batch(topics, nthreads=3)
    assert np.array_equal(ro, nro) and np.array_equal(ids, nids), seed
    cro, cids = nfa.match_batch(topics, nthreads=2, want_ids=False)
    assert np.array_equal(cro, ro) and len(cids) == 0


@pytest.mark.parametrize("wild_only,nf", [(False, 10_000), (True, 50_000)], ids=["C1-mix", "C2-wildcard"])
def test_cpu_nfa_on_workload_configs(orc, wild_only, nf):
    codes = orc.gen_filter_codes(1, nf, wildcard_only=wild_only)
    fb, fo = orc.render_codes(codes)
    tb, to = orc.render_codes(orc.gen_topic_codes(1, 0, 20_000, codes))
    r = orc.Router(True)
    r.add_routes((fb, fo))
    filters = sorted(set(orc.unpack(fb, fo)))
    ro, ids, _ = r.match_batch((tb, to), filters, mode=1, nthreads=4)
    nro, nids = orc.CpuNfa((fb, fo)).match_batch((tb, to), nthreads=4)
    assert np.array_equal(ro, nro) and np.array_equal(ids, nids)
