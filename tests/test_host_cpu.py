"""CPU-only checks: the C-ABI library loads and exports every declared symbol,
fails loudly without a device, and its host-side pieces (workload generator,
emqx_topic mirror) agree with the oracle / reference vectors."""

import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    names = set()
    for h in ("emqx_gpu_match.h", "emqx_gm_ext.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(emqx_gm_[a-z0-9_]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    from emqx_amd import _lib
    L = _lib.lib()
    declared = _declared_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert declared == set(_lib.SIGNATURES), "ctypes signatures out of sync with include/*.h"
    assert L.emqx_gm_abi_version() == 1


def test_nif_shim_binds_declared_symbols():
    src = open(os.path.join(ROOT, "nif", "emqx_gpu_match_nif.c")).read()
    used = set(re.findall(r"\b(emqx_gm_[a-z0-9_]+)\s*\(", src))
    assert used and used <= _declared_symbols()


def test_open_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from emqx_amd import Context, GpuMatchError
    with pytest.raises(GpuMatchError):
        Context(0)


def test_workload_generator_matches_oracle(orc):
    from emqx_amd.engine import gen_filter_codes, render_codes
    for wild in (False, True):
        a = gen_filter_codes(3, 5000, wildcard_only=wild)
        b = orc.gen_filter_codes(3, 5000, wildcard_only=wild)
        assert np.array_equal(a, b)
        da, oa = render_codes(a)
        db, ob = orc.render_codes(b)
        assert np.array_equal(oa, ob) and bytes(da[:oa[-1]]) == bytes(db[:ob[-1]])


def test_topic_mirror_golden(golden):
    from emqx_amd import topic as T
    for name, filt, expect in golden["topic_match"]["cases"]:
        assert T.match(name, filt) == expect, (name, filt)
    for t, expect in golden["topic_wildcard"]["cases"]:
        assert T.wildcard(t) == expect
    for case in golden["topic_join"]["cases"]:
        src, expect = case
        if isinstance(src, list):
            assert T.join(src) == expect.encode()
        else:
            assert T.join(T.words(src)) == expect.encode()
    for t, ws, kinds in golden["topic_words"]["cases"]:
        got = T.words(t)
        exp = [w if k == "atom" else w.encode() for w, k in zip(ws, kinds)]
        assert got == exp


def test_topic_mirror_validate():
    from emqx_amd import topic as T
    assert T.validate("a/+/#") and T.validate("x") and T.validate("x//y", "name")
    for bad, why in [("", "empty_topic"), ("abc/#/1", "topic_invalid_#"), ("abc/#xzy/+", "topic_invalid_char"),
                     ("sport+", "topic_invalid_char")]:
        with pytest.raises(T.TopicError, match=re.escape(why)):
            T.validate(bad)
    with pytest.raises(T.TopicError, match="topic_name_error"):
        T.validate("abc/#", "name")
    with pytest.raises(T.TopicError, match="topic_too_long"):
        T.validate(b"a" * 65536, "name")
    assert T.parse("$share/group/topic") == (b"topic", {"share": b"group"})
    assert T.parse("$queue/topic") == (b"topic", {"share": b"$queue"})
    assert T.parse("a/b/+/#") == (b"a/b/+/#", {})
    with pytest.raises(T.TopicError):
        T.parse("$share/t")


def test_topic_mirror_random_vs_oracle(orc):
    import random
    from emqx_amd import topic as T
    rng = random.Random(5)
    alph = ["a", "b", "", "$x", "+", "#"]
    for _ in range(3000):
        n = "/".join(rng.choice(alph[:4]) for _ in range(rng.randint(1, 4)))
        f = "/".join(rng.choice(alph) for _ in range(rng.randint(1, 4)))
        assert T.match(n, f) == orc.topic_match(n, f), (n, f)


def test_broker_bookkeeping_shards():
    """Host bookkeeping only (no device call): the shard indirection keeps every
    subscriber exactly once (emqx_broker_helper.erl:82-86)."""
    from emqx_amd.routing import Broker
    b = Broker(ctx=None, schedulers=2)
    b.router.ctx = object()  # never used: no snapshot is built in this test
    b.ctx = b.router.ctx
    for p in range(1, 2501):
        b.subscribe("hot/t", p)
    b.subscribe("hot/t", 3)  # idempotent
    assert len(b._shards) > 0
    assert sorted(b.subscribers("hot/t")) == list(range(1, 2501))
    assert b.router.has_routes("hot/t")
    for p in range(1, 2501):
        b.unsubscribe("hot/t", p)
    assert not b.router.has_routes("hot/t")


def _compile(filters, subs=None):
    import ctypes as C
    from emqx_amd import _lib
    from emqx_amd.engine import pack
    fb, fo = filters if isinstance(filters, tuple) else pack(filters)
    n = len(fo) - 1
    perm = np.zeros(max(n, 1), np.uint32)
    info = _lib.IndexInfo()
    so = si = None
    if subs is not None:
        so, si = subs
    rc = _lib.lib().emqx_gm_index_compile_host(
        C.c_void_p(fb.ctypes.data), C.c_void_p(fo.ctypes.data), n,
        None if so is None else C.c_void_p(so.ctypes.data), None if si is None else C.c_void_p(si.ctypes.data),
        C.c_void_p(perm.ctypes.data), C.byref(info))
    assert rc == 0
    return info, perm[:n]


def test_knobs_need_the_ab_opt_in(monkeypatch):
    """The shipped library ignores its GM_* A/B knobs unless EMQX_GM_AB opts in
    (gm_internal.h knob(); the default build reads EMQX_GM_AB alone, as
    include/emqx_gpu_match.h lists): a stray GM_NO_MPH on an EMQX host
    must not change a production node's table layout."""
    fs = [f"a/{i}/+/x{i % 7}".encode() for i in range(20000)]
    monkeypatch.delenv("EMQX_GM_AB", raising=False)
    base, _ = _compile(fs)
    monkeypatch.setenv("GM_NO_MPH", "1")  # (with the opt-in: no perfect-hash placement, larger tables)
    assert _compile(fs)[0].device_bytes == base.device_bytes
    monkeypatch.setenv("EMQX_GM_AB", "0")
    assert _compile(fs)[0].device_bytes == base.device_bytes
    monkeypatch.setenv("EMQX_GM_AB", "1")
    assert _compile(fs)[0].device_bytes > base.device_bytes
    # the library's sources read no other variable (the header's list)
    import glob
    names = set()
    for f in glob.glob(os.path.join(ROOT, "emqx_amd", "csrc", "*.*")):
        if f.endswith((".cpp", ".hip", ".h")):
            src = open(f).read()
            names |= set(re.findall(r'getenv\("([A-Z0-9_]+)"', src))
    assert names == {"EMQX_GM_AB"}, names
    # ... and the header lists exactly the knobs the sources read behind it
    knobs = set()
    for f in glob.glob(os.path.join(ROOT, "emqx_amd", "csrc", "*.*")):
        if f.endswith((".cpp", ".hip", ".h")):
            knobs |= set(re.findall(r'(?:knob|env_u64)\("(GM_[A-Z0-9_]+)"', open(f).read()))
    h = open(os.path.join(ROOT, "include", "emqx_gpu_match.h")).read()
    env = h[h.index(" * Environment:"):h.index("*/", h.index(" * Environment:"))]
    assert knobs == set(re.findall(r"\bGM_[A-Z0-9_]+", env))


@pytest.mark.timeout(60)
def test_index_compiler_host_small(golden):
    """The host index compiler (the part of emqx_gm_index_build that runs on
    the CPU) on the reference vectors and edge cases: ids are lexicographic
    ranks, duplicates collapse, trie_empty follows emqx_trie:empty/0."""
    fs = [b"sensor/1/metric/2", b"sensor/+/#", b"sensor/#", b"sensor/#", b"", b"#", b"/+", b"a//b", b"$SYS/#"]
    info, perm = _compile(fs)
    uniq = sorted(set(fs))
    assert info.n_filters == len(uniq)
    assert [uniq[i] for i in perm] == fs
    assert info.n_wildcard == sum(1 for f in uniq if b"+" in f.split(b"/") or b"#" in f.split(b"/"))
    assert not info.trie_empty
    info, _ = _compile([b"a/b", b"c"])
    assert info.trie_empty and info.n_wildcard == 0
    info, _ = _compile([])
    assert info.n_filters == 0 and info.trie_empty and info.n_nodes == 1
    for case in golden["trie_cases"]:
        ins = [a.encode() for op, a in case["ops"] if op == "insert"]
        info, perm = _compile(ins)
        assert info.n_filters == len(set(ins))


@pytest.mark.timeout(120)
def test_index_compiler_host_c2_scale(orc):
    """200k C2-shaped wildcard filters (a fifth of C2, sized for the CPU suite;
    the full 1M index is built and checked on the GPU in test_gpu_scale.py)
    compile in bounded time; node count equals the
    number of distinct word-list prefixes (the non-compact key count of the
    reference trie, emqx_trie.erl:223-232, plus the root)."""
    from emqx_amd.engine import gen_filter_codes, render_codes
    codes = gen_filter_codes(1, 200_000, wildcard_only=True)
    fb, fo = render_codes(codes)
    info, perm = _compile((fb, fo))
    fs = orc.unpack(fb, fo)
    prefixes = set()
    for f in fs:
        ws = f.split(b"/")
        for k in range(1, len(ws) + 1):
            prefixes.add(tuple(ws[:k]))
    assert info.n_nodes == len(prefixes) + 1
    assert info.n_edges == len(prefixes)
    assert info.n_filters == len(set(fs)) == 200_000


def test_nif_shim_type_checks():
    """The NIF shim compiles cleanly (-Wall -Wextra -Werror) against the OTP NIF
    API declarations it uses (tests/nif_stub/erl_nif.h: no Erlang on this
    image) and the library's public header."""
    import subprocess
    p = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "tests", "nif_stub"), "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "nif", "emqx_gpu_match_nif.c")], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


def test_nif_exports_match_erlang_module():
    """Every NIF function/arity the shim registers is declared by the Erlang
    module (nif/emqx_gpu_match.erl) and vice versa for the nif_error stubs."""
    src = open(os.path.join(ROOT, "nif", "emqx_gpu_match_nif.c")).read()
    nif = set(re.findall(r'\{"([a-z_]+)", (\d), [a-z_]+, ', src))
    erl = open(os.path.join(ROOT, "nif", "emqx_gpu_match.erl")).read()
    stubs = set()
    for name, args in re.findall(r"^([a-z_]+)\(([^)]*)\) -> erlang:nif_error", erl, re.M):
        stubs.add((name, str(len([a for a in args.split(",") if a.strip()]))))
    assert nif == stubs, (nif ^ stubs)


@pytest.mark.timeout(300)
def test_index_compiler_parallel_sort_and_dedup_ranks():
    """Above 200k filters the host compiler sorts on all threads (chunk sorts,
    then merges cut along their merge paths) and collapses duplicates per
    thread range (gm_index.cpp par_sort / the dedup pass): every input filter's
    id must still be its rank among the distinct filters in byte order
    (Python's sort of the bytes), duplicates spread over the input included."""
    import ctypes as C
    from emqx_amd import _lib
    from emqx_amd.engine import gen_filter_codes, render_codes
    n, k = 400_000, 60_000
    fb, fo = render_codes(gen_filter_codes(3, n))
    fb2 = np.concatenate([fb[:int(fo[n])], fb[:int(fo[k])], np.zeros(64, np.uint8)])
    fo2 = np.concatenate([fo[:n + 1], fo[1:k + 1] + fo[n]]).astype(np.uint64)
    m = n + k
    perm = np.zeros(m, np.uint32)
    info = _lib.IndexInfo()
    rc = _lib.lib().emqx_gm_index_compile_host(C.c_void_p(fb2.ctypes.data), C.c_void_p(fo2.ctypes.data), m, None,
                                               None, C.c_void_p(perm.ctypes.data), C.byref(info))
    assert rc == 0
    strs = [bytes(fb2[int(fo2[i]):int(fo2[i + 1])]) for i in range(m)]
    rank = {f: r for r, f in enumerate(sorted(set(strs)))}
    assert info.n_filters == len(rank)
    assert np.array_equal(perm, np.array([rank[f] for f in strs], np.uint32))


@pytest.mark.timeout(300)
def test_index_compiler_trie_runs_under_one_root_word(monkeypatch):
    """A set under one root word ("devices/...", one deployment's topic tree)
    above the parallel threshold: the trie is cut into runs below the root
    (gm_index.cpp safe_cut: a run starts from the path it shares with the one
    before) and merged in filter order -- the same ids and the same node,
    edge, word and byte counts as the one-run build (GM_TRIE_RUNS=1); the
    tables themselves are compared byte for byte in the ASan harness."""
    import ctypes as C
    from emqx_amd import _lib
    from emqx_amd.engine import gen_filter_codes, render_codes
    n = 250_000
    fb, fo = render_codes(gen_filter_codes(5, n))
    strs = [b"devices/" + bytes(fb[int(fo[i]):int(fo[i + 1])]) for i in range(n)]
    strs += [b"devices", b"devices-x/a", b"devices/l0w1"]  # the root word as a filter, an interloper, a prefix
    fb2 = np.frombuffer(b"".join(strs) + bytes(64), np.uint8)
    fo2 = np.zeros(len(strs) + 1, np.uint64)
    fo2[1:] = np.cumsum([len(x) for x in strs])

    def compile_(runs):
        if runs:
            monkeypatch.setenv("GM_TRIE_RUNS", runs)
        else:
            monkeypatch.delenv("GM_TRIE_RUNS", raising=False)
        perm = np.zeros(len(strs), np.uint32)
        info = _lib.IndexInfo()
        rc = _lib.lib().emqx_gm_index_compile_host(C.c_void_p(fb2.ctypes.data), C.c_void_p(fo2.ctypes.data),
                                                   len(strs), None, None, C.c_void_p(perm.ctypes.data),
                                                   C.byref(info))
        assert rc == 0
        return perm, (info.n_filters, info.n_wildcard, info.n_nodes, info.n_edges, info.n_words, info.device_bytes,
                      info.max_depth)

    p1, i1 = compile_("1")
    for runs in (None, "97"):
        p2, i2 = compile_(runs)
        assert np.array_equal(p1, p2) and i1 == i2, (runs, i1, i2)


@pytest.mark.parametrize("mph_min", [None, "1"], ids=["default", "mph_all_tables"])
def test_host_compiler_under_asan(mph_min):
    """The host index compiler (gm_index.cpp) and the overlay id mapping
    (gm_overlay.cpp) built with AddressSanitizer + UBSan and fed random,
    empty, NUL-laden, 65,535-byte and 5,000-level filters (SURVEY.md §5;
    tests/asan/asan_host_compiler.cpp): no sanitizer report, every input gets
    a valid id.  Index images (gm_image.cpp validate_image / import_host_part,
    what index_import runs before it touches a device): an exported image cut
    at every section boundary and at random sizes, 3,000 byte flips in its
    header and host sections, and 36 header counts / offsets rewritten and
    resealed -- every cut, flip and oversized value refused with EINVAL, no
    out-of-bounds read."""
    import subprocess
    b = subprocess.run(["make", "-C", os.path.join(ROOT, "emqx_amd", "csrc"), "asan"], capture_output=True, text=True)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               GM_CHAIN="1",  # chain nodes on every index (by default only past 256 MiB of hot tables)
               GM_INDEX_VERIFY="1")  # every Robin Hood hot table checked in order as it is built
    if mph_min:  # every per-depth table placed by hash-and-displace, in-place inserts into its overflow region
        env["GM_MPH_MIN_KEYS"] = mph_min
    p = subprocess.run([os.path.join(ROOT, "tests", "asan", "asan_host_compiler")], capture_output=True, text=True,
                       env=env, timeout=300)
    assert p.returncode == 0 and "ASAN_HOST_CHECK_OK" in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]


def test_c_abi_smoke_program_builds():
    """tests/c_abi_smoke.c -- the boundary driven from plain C, as the NIF or any
    native caller would -- compiles warning-free against include/ and links
    against the library (it runs on the GPU box: test_gpu_parity.py)."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "c_abi_smoke")
        p = subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", "-std=c11", "-I", os.path.join(ROOT, "include"),
                            os.path.join(ROOT, "tests", "c_abi_smoke.c"), "-L", os.path.join(ROOT, "emqx_amd"),
                            "-l:libemqx_gpu_match.so", "-o", out], capture_output=True, text=True)
        assert p.returncode == 0, p.stderr
