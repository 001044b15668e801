#!/usr/bin/env python3
"""Generates tests/golden/config_c5.json: 2,000 strided topics of the C5
publish stream (BASELINE configs[4]: 100M filters of the SURVEY.md §8d mixed
generator, seed 1) with their emqx_router:match_routes/1 rows
(emqx_router.erl:128-145) as filter strings.

The faithful restatement (oracle/emqx_oracle.cpp) over 100M keys does not fit
this container's memory, so the rows are computed by a third, independent
method: emqx_topic:match/2 (emqx_topic.erl:65-87) read backwards.  Every
generator topic has 5 concrete levels, and a filter of the generator's shape
(at most 5 levels of words, '+' or a last '#') matches it iff it is one of
  * the 32 five-level filters with each level the topic's word or '+'
    (the exact filter among them: the literal route, lookup_routes(Topic)),
  * the 31 filters 'p/#' with p a prefix of 0..4 levels, each level the
    topic's word or '+'.
So a row is the set of those 63 candidates present in the filter set, and
presence is one vectorised membership test of the candidates' generator keys
(the generator's own dedup key: base-1031 digits of the level codes) against
all 100M filter keys.  `--check c1 c2 c3` recomputes the committed
config_c{1,2,3}.json fixtures (made by the faithful restatement) this way and
asserts they are identical, which pins the method.

Run from the repo root:  python tests/golden/make_config_c5.py [--check c1 c2 c3]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as orc  # noqa: E402

CONFIGS = {  # name: (filters, wildcard_only, topics in the stream)
    "c1": (10_000, False, 1_000_000),
    "c2": (1_000_000, True, 100_000_000),
    "c3": (10_000_000, False, 100_000_000),
    "c5": (100_000_000, False, 100_000_000),
}
SEED, SAMPLE = 1, 2_000
L = orc.LEVELS


def sample_indices(n_stream):  # the same strided sample as make_config_vectors.py
    idx = np.linspace(0, n_stream - 1, SAMPLE).astype(np.int64)
    idx[1:-1] += np.arange(1, SAMPLE - 1) % 7
    return sorted(set(int(i) for i in idx))


def keys_of(codes):
    """The generator's dedup key of each code row (oracle gen_filter_codes)."""
    k = np.zeros(len(codes), np.uint64)
    for lvl in range(L):
        k = k * np.uint64(1031) + (codes[:, lvl].astype(np.int64) + 3).astype(np.uint64)
    return k


def candidates(t):
    """The 63 filter code rows that can match the 5-level topic code row t."""
    out = []
    for m in range(1 << L):  # five levels, each the word or '+'
        out.append([orc.C_PLUS if (m >> lvl) & 1 else int(t[lvl]) for lvl in range(L)])
    for k in range(L):  # k levels (word or '+'), then '#'
        for m in range(1 << k):
            c = [orc.C_PLUS if (m >> lvl) & 1 else int(t[lvl]) for lvl in range(k)] + [orc.C_HASH]
            out.append(c + [orc.C_END] * (L - len(c)))
    return np.array(out, np.int16)


def code_string(c):
    words = []
    for lvl in range(L):
        if c[lvl] == orc.C_END:
            break
        words.append("+" if c[lvl] == orc.C_PLUS else "#" if c[lvl] == orc.C_HASH else f"l{lvl}w{c[lvl]}")
    return "/".join(words)


def rows_for(name, log=print):
    nf, wild, ns = CONFIGS[name]
    t0 = time.time()
    codes = orc.gen_filter_codes(SEED, nf, wildcard_only=wild)
    log(f"[{name}] {nf} filter codes in {time.time() - t0:.1f} s")
    fkeys = np.sort(keys_of(codes))
    ids = sample_indices(ns)
    tc = np.concatenate([orc.gen_topic_codes(SEED, i, 1, codes) for i in ids])
    del codes
    tb, to = orc.render_codes(tc)
    topics = [t.decode() for t in orc.unpack(tb, to)]
    cand = [candidates(t) for t in tc]
    ck = keys_of(np.concatenate(cand))
    pos = np.searchsorted(fkeys, ck)
    hit = (pos < len(fkeys)) & (fkeys[np.minimum(pos, len(fkeys) - 1)] == ck)
    rows, j = [], 0
    for c in cand:
        h = hit[j:j + len(c)]
        j += len(c)
        # Erlang binary order = unsigned bytewise (ASCII here: Python str order)
        rows.append(sorted(code_string(x) for x in c[h]))
    log(f"[{name}] {len(ids)} topics, {sum(len(r) for r in rows)} matches in {time.time() - t0:.1f} s")
    return ids, topics, rows


def main(argv):
    if argv[:1] == ["--check"]:
        for name in argv[1:] or ["c1", "c2", "c3"]:
            ids, topics, rows = rows_for(name)
            with open(os.path.join(ROOT, "tests", "golden", f"config_{name}.json")) as f:
                ref = json.load(f)
            assert ref["topic_index"] == ids and ref["topics"] == topics, name
            assert ref["matches"] == rows, f"{name}: candidate enumeration differs from the faithful restatement"
            print(f"[{name}] identical to the committed fixture (faithful restatement)", flush=True)
        return
    nf, wild, ns = CONFIGS["c5"]
    ids, topics, rows = rows_for("c5")
    out = {"config": "c5", "seed": SEED, "filters": nf, "wildcard_only": wild, "stream_topics": ns,
           "semantics": "match_routes (exact route + wildcard trie matches), rows sorted in Erlang binary order",
           "generated_by": "tests/golden/make_config_c5.py (emqx_topic:match/2 read backwards: candidate "
                           "filters of each topic tested against all 100M generated filters; method pinned "
                           "by --check against the faithful-restatement fixtures c1/c2/c3)",
           "topic_index": ids, "topics": topics, "matches": rows}
    path = os.path.join(ROOT, "tests", "golden", "config_c5.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("c5", len(ids), "topics,", sum(len(x) for x in rows), "matches ->", path, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
