"""The committed config fixtures (tests/golden/config_c{1,2,3}.json, made by
tests/golden/make_config_vectors.py): 2,000 topics strided across each
benchmarked config's publish stream with their match_routes rows as filter
strings (SURVEY.md §8c "large-config vectors").

CPU side: the §8d generator still produces exactly these topics (so every
config test and bench line draws from the pinned stream), and the faithful
restatement and the optimized CPU hash-NFA still give these rows (C1, C2).
The GPU side is checked in test_gpu_parity.py (C1) and test_gpu_scale.py (C2,
C3), against the full config indexes.
"""

import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, f"config_{name}.json")) as f:
        return json.load(f)


def rows_as_strings(filters_sorted, ro, ids):
    return [[filters_sorted[k].decode() for k in ids[ro[i]:ro[i + 1]]] for i in range(len(ro) - 1)]


@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
def test_generator_reproduces_fixture_topics(orc, name):
    fx = load(name)
    codes = orc.gen_filter_codes(fx["seed"], fx["filters"], wildcard_only=fx["wildcard_only"])
    tc = np.concatenate([orc.gen_topic_codes(fx["seed"], i, 1, codes) for i in fx["topic_index"]])
    topics = [t.decode() for t in orc.unpack(*orc.render_codes(tc))]
    assert topics == fx["topics"]
    assert fx["topic_index"][0] == 0 and fx["topic_index"][-1] == fx["stream_topics"] - 1
    assert len(fx["topics"]) == len(fx["matches"]) == 2000


@pytest.mark.parametrize("name", ["c1", "c2"])
def test_oracles_reproduce_fixture_rows(orc, name):
    fx = load(name)
    codes = orc.gen_filter_codes(fx["seed"], fx["filters"], wildcard_only=fx["wildcard_only"])
    fb, fo = orc.render_codes(codes)
    filters = sorted(set(orc.unpack(fb, fo)))
    topics = [t.encode() for t in fx["topics"]]
    r = orc.Router(True)
    r.add_routes((fb, fo))
    ro, ids, _ = r.match_batch(topics, filters, mode=1, nthreads=4)
    assert rows_as_strings(filters, ro, ids) == fx["matches"]
    nro, nids = orc.CpuNfa((fb, fo)).match_batch(orc.pack(topics), nthreads=4)
    assert rows_as_strings(filters, nro, nids) == fx["matches"]
    # every derived-looking topic has a match; a fixture of empty rows would prove nothing
    assert sum(len(m) for m in fx["matches"]) > len(topics)


@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
def test_c5_fixture_method_reproduces_faithful_fixtures(orc, name):
    """The C5 fixture's third method (tests/golden/make_config_c5.py: the 63
    candidate filters of each topic looked up in the filter set) must give the
    faithful restatement's committed rows for C1, C2 and C3 -- so a drift in
    candidates() or keys_of() fails here, not only in a manual --check."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_config_c5", os.path.join(GOLDEN, "make_config_c5.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    fx = load(name)
    ids, topics, rows = mk.rows_for(name, log=lambda *a: None)
    assert ids == fx["topic_index"] and topics == fx["topics"]
    assert rows == fx["matches"]
    c5 = load("c5")
    assert c5["generated_by"].startswith("tests/golden/make_config_c5.py") and len(c5["matches"]) == 2000
