"""ctypes wrapper for the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as a checker / baseline.  The product path
(``emqx_amd``) never imports it.

The oracle restates the reference Erlang algorithm (see emqx_oracle.cpp for the
file:line map).  Parity is pinned by the reference's own test vectors in
``tests/golden/suite_vectors.json``.
"""

from __future__ import annotations

import ctypes as C
import os
from typing import List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

LEVELS = 5
VOCAB = (64, 1024, 1024, 64, 16)
C_PLUS, C_HASH, C_END = -1, -2, -3


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run `make -C oracle`)")
        L = C.CDLL(path)
        vp, u64, i64, cp = C.c_void_p, C.c_uint64, C.c_int64, C.c_char_p
        sig = {
            "orc_strlist_len": (i64, [vp]),
            "orc_strlist_get": (vp, [vp, i64, C.POINTER(u64)]),
            "orc_strlist_free": (None, [vp]),
            "orc_u64list_len": (i64, [vp]),
            "orc_u64list_data": (vp, [vp]),
            "orc_u64list_free": (None, [vp]),
            "orc_csr_rows": (u64, [vp]),
            "orc_csr_nnz": (u64, [vp]),
            "orc_csr_row_off": (vp, [vp]),
            "orc_csr_ids": (vp, [vp]),
            "orc_csr_aux": (vp, [vp]),
            "orc_csr_free": (None, [vp]),
            "orc_topic_match": (C.c_int, [cp, u64, cp, u64]),
            "orc_topic_wildcard": (C.c_int, [cp, u64]),
            "orc_topic_words": (vp, [cp, u64, vp, i64]),
            "orc_trie_new": (vp, [C.c_int]),
            "orc_trie_free": (None, [vp]),
            "orc_trie_insert": (None, [vp, cp, u64]),
            "orc_trie_delete": (None, [vp, cp, u64]),
            "orc_trie_empty": (C.c_int, [vp]),
            "orc_trie_match": (vp, [vp, cp, u64, C.POINTER(u64)]),
            "orc_trie_keys": (vp, [vp, vp, vp, i64]),
            "orc_trie_make_prefixes": (vp, [C.c_int, cp, u64]),
            "orc_do_compact": (vp, [cp, u64]),
            "orc_router_new": (vp, [C.c_int]),
            "orc_router_free": (None, [vp]),
            "orc_router_add_route": (None, [vp, cp, u64, cp, u64]),
            "orc_router_delete_route": (None, [vp, cp, u64, cp, u64]),
            "orc_router_add_routes": (None, [vp, vp, vp, u64]),
            "orc_router_trie": (vp, [vp]),
            "orc_router_match_routes": (vp, [vp, cp, u64]),
            "orc_router_topics": (vp, [vp]),
            "orc_broker_new": (vp, [C.c_int, C.c_int]),
            "orc_broker_free": (None, [vp]),
            "orc_broker_router": (vp, [vp]),
            "orc_broker_subscribe": (None, [vp, cp, u64, u64]),
            "orc_broker_subscribers": (vp, [vp, cp, u64]),
            "orc_broker_shard_entries": (i64, [vp, cp, u64]),
            "orc_broker_publish": (vp, [vp, cp, u64]),
            "orc_match_batch": (vp, [vp, C.c_int, vp, vp, u64, vp, vp, u64, C.c_int, C.c_int]),
            "orc_ranker_new": (vp, [vp, vp, u64]),
            "orc_ranker_free": (None, [vp]),
            "orc_match_batch_ranked": (vp, [vp, C.c_int, vp, vp, u64, vp, C.c_int]),
            "orc_bruteforce_batch": (vp, [C.c_int, vp, vp, u64, vp, vp, u64, vp]),
            "orc_fanout": (vp, [vp, vp, u64, vp, vp]),
            "orc_gen_filter_codes": (None, [u64, u64, C.c_int, vp]),
            "orc_gen_topic_codes": (None, [u64, u64, u64, vp, u64, vp]),
            "orc_render_codes": (u64, [vp, u64, vp, vp]),
            "orc_nfa_new": (vp, [vp, vp, u64]),
            "orc_nfa_free": (None, [vp]),
            "orc_nfa_match": (vp, [vp, vp, vp, u64, C.c_int, C.c_int]),
            "orc_nfa_rows_n": (u64, [vp]),
            "orc_nfa_rows_nnz": (u64, [vp]),
            "orc_nfa_rows_off": (vp, [vp]),
            "orc_nfa_rows_ids": (vp, [vp]),
            "orc_nfa_rows_free": (None, [vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def _b(s) -> bytes:
    return s.encode() if isinstance(s, str) else bytes(s)


def _strlist(h) -> List[bytes]:
    L = lib()
    out = []
    n = L.orc_strlist_len(h)
    ln = C.c_uint64()
    for i in range(n):
        p = L.orc_strlist_get(h, i, C.byref(ln))
        out.append(C.string_at(p, ln.value) if ln.value else b"")
    L.orc_strlist_free(h)
    return out


def _u64list(h) -> List[int]:
    L = lib()
    n = L.orc_u64list_len(h)
    p = L.orc_u64list_data(h)
    arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint64)), shape=(n,)).copy() if n else np.zeros(0, np.uint64)
    L.orc_u64list_free(h)
    return [int(x) for x in arr]


def _csr(h) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    L = lib()
    rows = L.orc_csr_rows(h)
    nnz = L.orc_csr_nnz(h)
    ro = np.ctypeslib.as_array(C.cast(L.orc_csr_row_off(h), C.POINTER(C.c_uint64)), shape=(rows + 1,)).copy()
    ids = (np.ctypeslib.as_array(C.cast(L.orc_csr_ids(h), C.POINTER(C.c_uint32)), shape=(nnz,)).copy()
           if nnz else np.zeros(0, np.uint32))
    aux_p = L.orc_csr_aux(h)
    aux = (np.ctypeslib.as_array(C.cast(aux_p, C.POINTER(C.c_uint64)), shape=(rows,)).copy()
           if aux_p and rows else np.zeros(0, np.uint64))
    L.orc_csr_free(h)
    return ro, ids, aux


def pack(strings: Sequence) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate byte strings -> (uint8 bytes, uint64 offsets[n+1])."""
    bs = [_b(s) for s in strings]
    off = np.zeros(len(bs) + 1, np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    data = np.frombuffer(b"".join(bs) + b"\0" * 16, np.uint8).copy()
    return data, off


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


# ---------------------------------------------------------------- emqx_topic
def topic_match(name, filt) -> bool:
    n, f = _b(name), _b(filt)
    return bool(lib().orc_topic_match(n, len(n), f, len(f)))


def wildcard(t) -> bool:
    t = _b(t)
    return bool(lib().orc_topic_wildcard(t, len(t)))


def words(t) -> list:
    """emqx_topic:words/1 -> list of bytes | '' | '+' | '#' (atoms as str)."""
    t = _b(t)
    kinds = np.zeros(len(t) + 2, np.int32)
    ws = _strlist(lib().orc_topic_words(t, len(t), _ptr(kinds), len(kinds)))
    out = []
    for w, k in zip(ws, kinds):
        out.append({0: w, 1: "", 2: "+", 3: "#"}[int(k)])
    return out


# ---------------------------------------------------------------- emqx_trie
class Trie:
    def __init__(self, compact: bool = True, _handle=None):
        self._own = _handle is None
        self.h = lib().orc_trie_new(int(compact)) if _handle is None else _handle

    def __del__(self):
        if getattr(self, "_own", False) and self.h:
            lib().orc_trie_free(self.h)
            self.h = None

    def insert(self, t):
        t = _b(t)
        lib().orc_trie_insert(self.h, t, len(t))

    def delete(self, t):
        t = _b(t)
        lib().orc_trie_delete(self.h, t, len(t))

    def empty(self) -> bool:
        return bool(lib().orc_trie_empty(self.h))

    def match(self, t, with_lookups: bool = False):
        t = _b(t)
        lk = C.c_uint64()
        r = _strlist(lib().orc_trie_match(self.h, t, len(t), C.byref(lk)))
        return (r, lk.value) if with_lookups else r

    def lookup_topic(self, t) -> list:
        t = _b(t)
        for k, kind, cnt in self.keys():
            if k == t and kind == 1 and cnt > 0:
                return [t]
        return []

    def keys(self):
        n = 1 << 20
        kinds = np.zeros(n, np.int64)
        counts = np.zeros(n, np.int64)
        ks = _strlist(lib().orc_trie_keys(self.h, _ptr(kinds), _ptr(counts), n))
        return [(k, int(kinds[i]), int(counts[i])) for i, k in enumerate(ks)]


def make_prefixes(t, compact: bool) -> list:
    t = _b(t)
    return _strlist(lib().orc_trie_make_prefixes(int(compact), t, len(t)))


def do_compact(t) -> list:
    t = _b(t)
    return _strlist(lib().orc_do_compact(t, len(t)))


# ---------------------------------------------------------------- emqx_router
class Router:
    def __init__(self, compact: bool = True, _handle=None):
        self._own = _handle is None
        self.h = lib().orc_router_new(int(compact)) if _handle is None else _handle

    def __del__(self):
        if getattr(self, "_own", False) and self.h:
            lib().orc_router_free(self.h)
            self.h = None

    @property
    def trie(self) -> Trie:
        return Trie(_handle=lib().orc_router_trie(self.h))

    def add_route(self, t, dest=b"node"):
        t, d = _b(t), _b(dest)
        lib().orc_router_add_route(self.h, t, len(t), d, len(d))

    def add_routes(self, packed):
        """add_route/1 for every filter of a packed (bytes, offsets) pair, in one call."""
        fb, fo = packed
        fb = np.ascontiguousarray(fb, np.uint8)
        fo = np.ascontiguousarray(fo, np.uint64)
        lib().orc_router_add_routes(self.h, _ptr(fb), _ptr(fo), len(fo) - 1)

    def delete_route(self, t, dest=b"node"):
        t, d = _b(t), _b(dest)
        lib().orc_router_delete_route(self.h, t, len(t), d, len(d))

    def match_routes(self, t) -> List[Tuple[bytes, bytes]]:
        t = _b(t)
        it = _strlist(lib().orc_router_match_routes(self.h, t, len(t)))
        return [(it[i], it[i + 1]) for i in range(0, len(it), 2)]

    def topics(self) -> List[bytes]:
        return _strlist(lib().orc_router_topics(self.h))

    def match_batch(self, topics, sorted_filters, mode: int = 1, nthreads: int = 1, want_ids: bool = True):
        """Returns (row_off, ids, lookups) with ids = rank in ``sorted_filters``
        (a list, a packed (bytes, offsets) pair, or a :class:`Ranker` built once
        for many batches; None with want_ids=False: counts only)."""
        tb, to = topics if isinstance(topics, tuple) else pack(topics)
        n = len(to) - 1
        if isinstance(sorted_filters, Ranker) or not want_ids:
            k = sorted_filters.h if (want_ids and sorted_filters is not None) else None
            return _csr(lib().orc_match_batch_ranked(self.h, mode, _ptr(tb), _ptr(to), n, k, nthreads))
        fb, fo = sorted_filters if isinstance(sorted_filters, tuple) else pack(sorted_filters)
        nf = len(fo) - 1
        return _csr(lib().orc_match_batch(self.h, mode, _ptr(tb), _ptr(to), n, _ptr(fb), _ptr(fo), nf,
                                          nthreads, int(want_ids)))


class CpuNfa:
    """The optimized CPU hash-NFA (cpu_nfa.cpp): emqx_router:match_routes/1
    rows over flat hash tables, multi-threaded.  The second CPU figure of the
    bench's cpu_baseline leg; checked against the faithful restatement."""

    def __init__(self, filters):
        fb, fo = filters if isinstance(filters, tuple) else pack(filters)
        fb = np.ascontiguousarray(fb, np.uint8)
        fo = np.ascontiguousarray(fo, np.uint64)
        self.h = lib().orc_nfa_new(_ptr(fb), _ptr(fo), len(fo) - 1)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_nfa_free(self.h)
            self.h = None

    def match_batch(self, topics, nthreads: int = 1, want_ids: bool = True):
        """(row_off, ids) with ids = rank among the sorted unique filters;
        want_ids=False: row lengths only (ids empty)."""
        tb, to = topics if isinstance(topics, tuple) else pack(topics)
        tb = np.ascontiguousarray(tb, np.uint8)
        to = np.ascontiguousarray(to, np.uint64)
        L = lib()
        h = L.orc_nfa_match(self.h, _ptr(tb), _ptr(to), len(to) - 1, nthreads, int(want_ids))
        rows, nnz = L.orc_nfa_rows_n(h), L.orc_nfa_rows_nnz(h)
        ro = np.ctypeslib.as_array(C.cast(L.orc_nfa_rows_off(h), C.POINTER(C.c_uint64)), shape=(rows + 1,)).copy()
        ids = (np.ctypeslib.as_array(C.cast(L.orc_nfa_rows_ids(h), C.POINTER(C.c_uint32)), shape=(nnz,)).copy()
               if nnz else np.zeros(0, np.uint32))
        L.orc_nfa_rows_free(h)
        return ro, ids


class Ranker:
    """Filter -> id map (rank among the sorted unique filters), built once."""

    def __init__(self, sorted_filters):
        fb, fo = sorted_filters if isinstance(sorted_filters, tuple) else pack(sorted_filters)
        fb = np.ascontiguousarray(fb, np.uint8)
        fo = np.ascontiguousarray(fo, np.uint64)
        self.h = lib().orc_ranker_new(_ptr(fb), _ptr(fo), len(fo) - 1)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_ranker_free(self.h)
            self.h = None


# ---------------------------------------------------------------- emqx_broker
class Broker:
    def __init__(self, compact: bool = True, schedulers: int = 8):
        self.h = lib().orc_broker_new(int(compact), schedulers)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_broker_free(self.h)
            self.h = None

    @property
    def router(self) -> Router:
        return Router(_handle=lib().orc_broker_router(self.h))

    def subscribe(self, t, pid: int):
        t = _b(t)
        lib().orc_broker_subscribe(self.h, t, len(t), pid)

    def subscribers(self, t) -> List[int]:
        t = _b(t)
        return _u64list(lib().orc_broker_subscribers(self.h, t, len(t)))

    def shard_entries(self, t) -> int:
        t = _b(t)
        return int(lib().orc_broker_shard_entries(self.h, t, len(t)))

    def publish(self, t) -> List[int]:
        t = _b(t)
        return _u64list(lib().orc_broker_publish(self.h, t, len(t)))


# ---------------------------------------------------------------- brute force / fan-out
def bruteforce(topics, sorted_filters, mode: int = 1, in_trie=None):
    tb, to = topics if isinstance(topics, tuple) else pack(topics)
    fb, fo = sorted_filters if isinstance(sorted_filters, tuple) else pack(sorted_filters)
    nf = len(fo) - 1
    it = np.ones(max(nf, 1), np.uint8) if in_trie is None else np.asarray(in_trie, np.uint8)
    ro, ids, _ = _csr(lib().orc_bruteforce_batch(mode, _ptr(tb), _ptr(to), len(to) - 1, _ptr(fb), _ptr(fo), nf,
                                                 _ptr(it)))
    return ro, ids


def fanout(m_off, m_ids, s_off, s_ids):
    m_off = np.ascontiguousarray(m_off, np.uint64)
    m_ids = np.ascontiguousarray(m_ids, np.uint32)
    s_off = np.ascontiguousarray(s_off, np.uint64)
    s_ids = np.ascontiguousarray(s_ids, np.uint32)
    if len(m_ids) == 0:
        m_ids = np.zeros(1, np.uint32)
    if len(s_ids) == 0:
        s_ids = np.zeros(1, np.uint32)
    ro, ids, _ = _csr(lib().orc_fanout(_ptr(m_off), _ptr(m_ids), len(m_off) - 1, _ptr(s_off), _ptr(s_ids)))
    return ro, ids


# ---------------------------------------------------------------- workload generator
def gen_filter_codes(seed: int, n: int, wildcard_only: bool = False) -> np.ndarray:
    out = np.zeros((n, LEVELS), np.int16)
    lib().orc_gen_filter_codes(seed, n, int(wildcard_only), _ptr(out))
    return out


def gen_topic_codes(seed: int, start: int, n: int, fcodes: np.ndarray) -> np.ndarray:
    fcodes = np.ascontiguousarray(fcodes, np.int16)
    out = np.zeros((n, LEVELS), np.int16)
    lib().orc_gen_topic_codes(seed, start, n, _ptr(fcodes), len(fcodes), _ptr(out))
    return out


def render_codes(codes: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    codes = np.ascontiguousarray(codes, np.int16)
    n = len(codes)
    off = np.zeros(n + 1, np.uint64)
    total = lib().orc_render_codes(_ptr(codes), n, None, _ptr(off))
    data = np.zeros(int(total) + 16, np.uint8)
    lib().orc_render_codes(_ptr(codes), n, _ptr(data), _ptr(off))
    return data, off


def unpack(data: np.ndarray, off: np.ndarray) -> List[bytes]:
    raw = data.tobytes()
    return [raw[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
