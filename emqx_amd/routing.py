"""Host mirrors of the reference routing interfaces, served by the GPU engine.

    Trie    <- emqx_trie    (apps/emqx/src/emqx_trie.erl: insert/1, delete/1, match/1, empty/0)
    Router  <- emqx_router  (apps/emqx/src/emqx_router.erl: add_route/1,2, delete_route/1,2,
                             match_routes/1, lookup_routes/1, has_routes/1, topics/0)
    Broker  <- emqx_broker  (apps/emqx/src/emqx_broker.erl: subscribe/1,2, unsubscribe/1,
                             subscribers/1, publish/1 -> dispatch/2)

Writes update host tables with the reference's semantics (insert is idempotent
per topic key, delete only if present, emqx_trie.erl:114-136; a wildcard route
enters the trie with its first dest, emqx_router_utils.erl:33-38).  Reads go to
an immutable index snapshot in HBM; the first read after writes derives a new
snapshot from the previous one with emqx_gm_index_update (tombstones + a delta
index, or a flat rebuild once the delta is large) -- RCU: a reader holding the
old snapshot keeps using it.  The batched
forms (``match_batch``, ``match_routes_batch``, ``publish_batch``) are the hot
path; the single-topic forms are the reference API on a batch of one.
"""

from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import topic as T
from .engine import Context, Index, pack

_DEFAULT_CTX: Optional[Context] = None
_CTX_LOCK = threading.Lock()


def default_context() -> Context:
    global _DEFAULT_CTX
    with _CTX_LOCK:
        if _DEFAULT_CTX is None:
            _DEFAULT_CTX = Context(0)
        return _DEFAULT_CTX


def _b(s) -> bytes:
    return s.encode() if isinstance(s, str) else bytes(s)


class _Snapshot:
    """An index snapshot plus the id -> filter table (sorted filters) it serves."""

    def __init__(self, ctx: Context, filters: List[bytes], subs: Optional[List[List[int]]] = None,
                 index: Optional[Index] = None):
        self.filters = sorted(set(filters))
        self.index: Index = index if index is not None else ctx.build_index(self.filters, subs=subs)


def _refresh(ctx: Context, snap: Optional[_Snapshot], keys, pending: List[Tuple[bytes, bool]]) -> _Snapshot:
    """The snapshot for the current key set: derived from `snap` by the pending
    inserts/deletes when there is one, built from scratch otherwise."""
    if snap is None:
        return _Snapshot(ctx, list(keys))
    return _Snapshot(ctx, list(keys), index=ctx.update_index(snap.index, pending))


class Trie:
    """emqx_trie over the GPU index.  ``compact`` is accepted for API parity
    (broker.perf.trie_compaction); it changes the reference's key layout and
    lookup count, never the result set (emqx_trie_SUITE.erl:25-39)."""

    def __init__(self, ctx: Optional[Context] = None, compact: bool = True):
        self.ctx = ctx
        self.compact = compact
        self._topics: set = set()
        self._snap: Optional[_Snapshot] = None
        self._pending: List[Tuple[bytes, bool]] = []
        self._lock = threading.Lock()

    def _context(self) -> Context:
        if self.ctx is None:
            self.ctx = default_context()
        return self.ctx

    def insert(self, t) -> None:
        with self._lock:
            t = _b(t)
            if t not in self._topics:
                self._topics.add(t)
                self._pending.append((t, True))

    def delete(self, t) -> None:
        with self._lock:
            t = _b(t)
            if t in self._topics:
                self._topics.discard(t)
                self._pending.append((t, False))

    def empty(self) -> bool:
        """emqx_trie:empty/0 (ets:first =:= '$end_of_table')."""
        return not self._topics

    def snapshot(self) -> _Snapshot:
        with self._lock:
            if self._snap is None or self._pending:
                self._snap = _refresh(self._context(), self._snap, self._topics, self._pending)
                self._pending = []
            return self._snap

    def match_batch(self, topics: Sequence) -> List[List[bytes]]:
        snap = self.snapshot()
        ro, ids = self._context().match(snap.index, list(topics), exact=False)
        return [[snap.filters[i] for i in ids[ro[k]:ro[k + 1]]] for k in range(len(ro) - 1)]

    def match(self, t) -> List[bytes]:
        return self.match_batch([t])[0]


class Router:
    """emqx_router: the emqx_route bag plus the wildcard trie, on the GPU."""

    def __init__(self, ctx: Optional[Context] = None, node: bytes = b"node"):
        self.ctx = ctx
        self.node = _b(node)
        self._routes: Dict[bytes, List[object]] = {}
        self._snap: Optional[_Snapshot] = None
        self._pending: List[Tuple[bytes, bool]] = []
        self._lock = threading.Lock()

    def _context(self) -> Context:
        if self.ctx is None:
            self.ctx = default_context()
        return self.ctx

    def add_route(self, t, dest=None) -> None:
        """do_add_route/2 (emqx_router.erl:112-125)."""
        t = _b(t)
        dest = self.node if dest is None else dest
        with self._lock:
            ds = self._routes.setdefault(t, [])
            if dest not in ds:
                ds.append(dest)
                if len(ds) == 1:  # the filter enters the index with its first route
                    self._pending.append((t, True))

    def delete_route(self, t, dest=None) -> None:
        """do_delete_route/2 (emqx_router.erl:164-172)."""
        t = _b(t)
        dest = self.node if dest is None else dest
        with self._lock:
            ds = self._routes.get(t)
            if ds and dest in ds:
                ds.remove(dest)
                if not ds:  # ... and leaves it with its last
                    del self._routes[t]
                    self._pending.append((t, False))

    def lookup_routes(self, t) -> List[Tuple[bytes, object]]:
        t = _b(t)
        return [(t, d) for d in self._routes.get(t, [])]

    def has_routes(self, t) -> bool:
        return _b(t) in self._routes

    def topics(self) -> List[bytes]:
        return list(self._routes)

    def trie_empty(self) -> bool:
        return not any(T.wildcard(f) for f in self._routes)

    def snapshot(self) -> _Snapshot:
        with self._lock:
            if self._snap is None or self._pending:
                self._snap = _refresh(self._context(), self._snap, self._routes, self._pending)
                self._pending = []
            return self._snap

    def match_filters_batch(self, topics: Sequence) -> Tuple[_Snapshot, np.ndarray, np.ndarray]:
        snap = self.snapshot()
        ro, ids = self._context().match(snap.index, list(topics), exact=True)
        return snap, ro, ids

    def match_routes_batch(self, topics: Sequence) -> List[List[Tuple[bytes, object]]]:
        """match_routes/1 (emqx_router.erl:128-134) for each topic."""
        snap, ro, ids = self.match_filters_batch(topics)
        out = []
        for k in range(len(ro) - 1):
            rows = []
            for i in ids[ro[k]:ro[k + 1]]:
                f = snap.filters[i]
                rows.extend((f, d) for d in self._routes.get(f, []))
            out.append(rows)
        return out

    def match_routes(self, t) -> List[Tuple[bytes, object]]:
        return self.match_routes_batch([t])[0]


class SessionRouter(Router):
    """emqx_session_router: the persistent-session routing table
    (apps/emqx/src/emqx_session_router.erl:100-134).  The same algorithm over
    a second trie (emqx_trie:insert_session/1, match_session/1,
    emqx_trie.erl:110-112, 143-145), so it is a second index served by the same
    kernels; a route's dest is a session id instead of a node."""

    def __init__(self, ctx: Optional[Context] = None):
        super().__init__(ctx, node=b"")

    def add_route(self, t, session_id) -> None:
        """do_add_route/2 (emqx_session_router.erl:100-118)."""
        super().add_route(t, session_id)

    def delete_route(self, t, session_id) -> None:
        super().delete_route(t, session_id)


class Broker:
    """emqx_broker subscribe / dispatch over the GPU fan-out.

    Bookkeeping mirrors emqx_broker:do_subscribe/4 and emqx_broker_helper:
    get_sub_shard/2: the first 1,024 subscribers of a topic sit directly under
    the topic, later ones in ``{shard, Topic, I}`` buckets with one
    ``{shard, I}`` marker per bucket (emqx_broker.erl:147-165, 445-454).  The
    snapshot flattens the buckets into one subscriber list per filter, which is
    what do_dispatch/2,3 (emqx_broker.erl:506-530) folds over.

    Snapshots are incremental: the subscribe / unsubscribe calls since the last
    snapshot are applied with one emqx_gm_index_update_subs (a filter's first
    subscriber adds its route, its last one leaving deletes it).  Within a
    filter the incremental list keeps arrival order, so a sharded topic's
    deliveries may come in another order than subscribers/1 lists them; the
    delivery multiset is the same (the reference promises no order either)."""

    SHARD = 1024  # emqx_broker_helper.erl:54

    def __init__(self, ctx: Optional[Context] = None, schedulers: int = 8):
        self.ctx = ctx
        self.router = Router(ctx)
        self.shards_num = schedulers * 32
        self._direct: Dict[bytes, List[int]] = {}
        self._shards: Dict[Tuple[bytes, int], List[int]] = {}
        self._seq: Dict[bytes, int] = {}
        self._subopt: set = set()
        self._snap: Optional[_Snapshot] = None
        self._pending: List[Tuple[bytes, int, bool]] = []  # since the snapshot: (filter, subscriber, subscribe)
        self._lock = threading.Lock()

    def _context(self) -> Context:
        if self.ctx is None:
            self.ctx = self.router._context()
        return self.ctx

    def subscribe(self, t, subpid: int) -> None:
        t = _b(t)
        with self._lock:
            if (subpid, t) in self._subopt:
                return
            self._subopt.add((subpid, t))
            s = self._seq[t] = self._seq.get(t, 0) + 1
            if s <= self.SHARD:
                self._direct.setdefault(t, []).append(subpid)
            else:
                i = (subpid * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF)
                i = ((i ^ (i >> 29)) % self.shards_num) + 1
                self._shards.setdefault((t, i), []).append(subpid)
            self._pending.append((t, subpid, True))
        self.router.add_route(t)

    def unsubscribe(self, t, subpid: int) -> None:
        t = _b(t)
        with self._lock:
            if (subpid, t) not in self._subopt:
                return
            self._subopt.discard((subpid, t))
            if subpid in self._direct.get(t, []):
                self._direct[t].remove(subpid)
            for k in [k for k in self._shards if k[0] == t]:
                if subpid in self._shards[k]:
                    self._shards[k].remove(subpid)
            self._pending.append((t, subpid, False))
            still = bool(self._direct.get(t)) or any(v for k, v in self._shards.items() if k[0] == t)
        if not still:
            self.router.delete_route(t)

    def subscribers(self, t) -> List[int]:
        """subscribers/1 with the shard markers expanded (do_dispatch/3)."""
        t = _b(t)
        out = list(self._direct.get(t, []))
        for (tt, _i), v in sorted(self._shards.items(), key=lambda kv: kv[0][1]):
            if tt == t:
                out.extend(v)
        return out

    def snapshot(self) -> _Snapshot:
        with self._lock:
            filters = sorted(self.router._routes)
            if self._snap is not None and self._pending:
                idx = self._context().update_subs(self._snap.index, self._pending)
                # the filters the library's snapshot holds: the previous ones, each
                # touched filter kept iff it still has a subscriber (its route)
                held = set(self._snap.filters)
                for t in {t for t, _, _ in self._pending}:
                    if self._direct.get(t) or any(v for k, v in self._shards.items() if k[0] == t):
                        held.add(t)
                    else:
                        held.discard(t)
                if idx.n_filters == len(held) and held == set(filters):
                    self._snap = _Snapshot(self._context(), filters, index=idx)
                else:  # routes changed behind the broker's back (router.add_route / a racing
                    # add or delete_route outside the broker lock): rebuild from the lists
                    idx.release()
                    self._snap = None
                self._pending = []
            if self._snap is None:
                subs = [self.subscribers(f) for f in filters]
                self._snap = _Snapshot(self._context(), filters, subs)
                self._pending = []
            return self._snap

    def publish_batch(self, topics: Sequence) -> List[List[int]]:
        """publish/1 for each topic: match_routes -> dispatch; returns each
        topic's deliveries (a multiset of subscriber ids).  An empty row is a
        'messages.dropped.no_subscribers' (emqx_broker.erl:245-248)."""
        snap = self.snapshot()
        ctx = self._context()
        (ro, ids), (fro, fids) = ctx.match_fanout(snap.index, list(topics), exact=True)
        return [fids[fro[k]:fro[k + 1]].astype(np.int64).tolist() for k in range(len(fro) - 1)]

    def publish(self, t) -> List[int]:
        return self.publish_batch([t])[0]
