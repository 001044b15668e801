"""Publish batching aggregator: the host mirror of nif/emqx_gpu_match_batcher.erl.

The reference publishes one message at a time in the publisher's process:
emqx_broker:publish/1 counts 'messages.publish', runs the 'message.publish'
hook, persists the message and then route(aggre(match_routes(Topic))) --
a local route dispatches to the filter's subscribers, a remote one is
forwarded, a shared-group one goes to emqx_shared_sub, and no route at all
runs 'message.dropped' + inc_dropped_cnt (apps/emqx/src/emqx_broker.erl:
204-215, 245-273, 296-322, 506-530).

Here only the MATCH is batched.  ``PublishBatcher`` is the server side: it
collects topics for at most ``window_s`` seconds or ``max_batch`` topics and
answers each with its row -- ``[(filter, subscriber ids)]`` over every matched
route filter -- from ONE groups call (``GpuRoutes.groups``: emqx_gm_match
WITH_EXACT -> emqx_gm_fanout -> each fan-out row cut back into one segment per
filter, the NIF's fanout_batch/2).  ``PublishBatcher.publish`` is the caller
side: it does everything else the reference's publish/1 does, in the caller's
thread, with the local dispatch over the row's subscriber ids and
lookup_routes/1 only for filters that have other destinations (remote nodes,
shared groups).  When the server answers an error (no index, a failed
engine call, a stale snapshot) the caller takes the reference path
(``fallback``: match_routes/1).

``GpuRoutes`` is the server's index maintenance: subscribe / unsubscribe /
subscriber_down / route_add / route_delete queue ops, and the next batch
applies them with ONE emqx_gm_index_update_subs (a new snapshot derived from
the last, never a rebuild by the aggregator).

The window logic takes an injectable clock and groups function, so it is
tested on the CPU; the GPU path is ``GpuRoutes``.
"""

from __future__ import annotations

import threading
import time
from concurrent.futures import Future
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

Group = Tuple[bytes, np.ndarray]  # (filter, subscriber ids)
Row = List[Group]
Result = List[Tuple[object, bytes, Tuple[str, object]]]  # publish_result(): [(node | "share", filter, result)]


def _b(s) -> bytes:
    return s.encode() if isinstance(s, str) else bytes(s)


def is_sys(topic: bytes) -> bool:
    """emqx_message:is_sys/1: a $SYS/ topic (not counted in the publish/drop metrics)."""
    return topic.startswith(b"$SYS/")


class GpuRoutes:
    """The aggregator's index over the route filters, with the local
    subscribers' ids as fan-out lists (mirror of the gen_server state of
    nif/emqx_gpu_match_batcher.erl).  A filter is in the index while it has a
    local subscriber or another destination (route_add)."""

    def __init__(self, ctx, node: bytes = b"node"):
        self.ctx, self.node = ctx, _b(node)
        self.index = ctx.build_index([], subs=[])  # load_index([], []) at init
        self.ops: List[Tuple[bytes, int, str]] = []  # since the snapshot, oldest first
        self.ids: Dict[object, int] = {}       # subscriber -> id
        self._next_id = 0                      # monotonic, as next_id in the Erlang server: a
                                               # subscriber that went down never lends its id
        self.subs: Dict[int, object] = {}      # id -> subscriber (the ?SUBS table)
        self.filters_of: Dict[object, set] = {}
        self.other: Dict[bytes, int] = {}      # filter -> destinations other than node (?OTHER)
        self.updates = 0
        self.builds = 1
        self.stale = False
        self._names: Dict[int, bytes] = {}     # filter id -> bytes of the current snapshot
        self._lock = threading.Lock()

    # ---- maintenance (handle_call subscribe / unsubscribe / route, 'DOWN')
    def subscribe(self, filt, sub) -> None:
        f = _b(filt)
        with self._lock:
            sid = self.ids.get(sub)
            if sid is None:
                sid = self.ids[sub] = self._next_id
                self._next_id += 1
                self.subs[sid] = sub
            self.filters_of.setdefault(sub, set()).add(f)
            self.ops.append((f, sid, "subscribe"))

    def unsubscribe(self, filt, sub) -> None:
        f = _b(filt)
        with self._lock:
            sid = self.ids.get(sub)
            if sid is None:
                return
            self.filters_of.get(sub, set()).discard(f)
            self.ops.append((f, sid, "unsubscribe"))

    def subscriber_down(self, sub) -> None:
        """emqx_broker_helper's subscriber_down: every subscription of the subscriber goes."""
        with self._lock:
            sid = self.ids.pop(sub, None)
            if sid is None:
                return
            for f in sorted(self.filters_of.pop(sub, set())):
                self.ops.append((f, sid, "unsubscribe"))
            self.subs.pop(sid, None)

    def route_add(self, filt, dest) -> None:
        self._route(_b(filt), dest, 1)

    def route_delete(self, filt, dest) -> None:
        self._route(_b(filt), dest, -1)

    def _route(self, f: bytes, dest, d: int) -> None:
        if not isinstance(dest, tuple) and _b(dest) == self.node:  # the local route follows the local subscribers
            return
        with self._lock:
            old = self.other.get(f, 0)
            new = max(0, old + d)
            if new:
                self.other[f] = new
            else:
                self.other.pop(f, None)
            if old == 0 and new > 0:
                self.ops.append((f, 0, "route_add"))
            elif old > 0 and new == 0:
                self.ops.append((f, 0, "route_delete"))

    def refresh(self) -> None:
        """The queued ops applied to the last snapshot with one update_subs; on
        failure they stay queued and the snapshot is stale until a retry works."""
        with self._lock:
            ops, self.ops = self.ops, []
        if not ops:
            self.stale = False
            return
        try:
            new = self.ctx.update_subs(self.index, ops)
        except Exception:
            with self._lock:
                self.ops = ops + self.ops
            self.stale = True
            return
        self.index, self._names = new, {}
        self.updates += 1
        self.stale = False

    # ---- the batch call (fanout_batch/2)
    def groups(self, topics: Sequence[bytes]) -> List[Row]:
        self.refresh()
        if self.stale:
            raise RuntimeError("stale_index")
        idx = self.index
        # (the NIF's fanout_batch/2: emqx_gm_match_fanout, the match and its fan-out in one call)
        (ro, ids), (fro, fids) = self.ctx.match_fanout(idx, list(topics), exact=True)
        out = []
        for k in range(len(ro) - 1):
            row, pos = [], int(fro[k])
            for f in ids[ro[k]:ro[k + 1]].tolist():
                c = idx.subscriber_count(f)
                name = self._names.get(f)
                if name is None:
                    name = self._names[f] = idx.filter(f)
                row.append((name, fids[pos:pos + c]))
                pos += c
            assert pos == int(fro[k + 1])
            out.append(row)
        return out


class PublishBatcher:
    """Size/time-window aggregator over a groups function (server side) plus the
    caller-side publish/1 around it (see the module doc).

    Caller-side collaborators (defaults: inert): ``subscribers`` maps subscriber
    id -> subscriber for ``deliver(sub, filter, msg) -> bool`` (False: not
    alive); ``lookup_routes(filter) -> [dest]`` with ``others`` the filters that
    have non-local destinations; ``forward(node, filter, msg)``;
    ``shared_dispatch(group, filter, msg)``; ``fallback(topic) -> [(filter,
    dest)]`` (match_routes/1) with ``fallback_dispatch(filter, msg)``;
    ``on_dropped(msg)`` (the 'message.dropped' hook); ``persist(topic, msg)``;
    ``metrics`` counts messages.publish / dropped / dropped.no_subscribers.
    A dest is the node name (bytes or str) or a (group, node) tuple.

    ``routes`` (a GpuRoutes) wires the server's own index in one argument:
    ``groups_fn`` defaults to ``routes.groups``, ``others`` to ``routes.other``
    (the ?OTHER table the Erlang caller reads directly) and ``subscribers`` to
    ``routes.subs``.  A ``groups_fn`` that is a bound ``GpuRoutes.groups`` gets
    its ``others`` the same way, so remote and shared routes cannot be dropped
    by forgetting the second argument."""

    def __init__(self, groups_fn: Optional[Callable[[Sequence[bytes]], List[Row]]] = None, max_batch: int = 4096,
                 window_s: float = 0.001, subscribers: Optional[Dict[int, object]] = None,
                 deliver: Optional[Callable[[object, bytes, object], bool]] = None,
                 clock: Callable[[], float] = time.monotonic, timer: bool = True, node: bytes = b"node",
                 lookup_routes: Optional[Callable[[bytes], List[object]]] = None, others=None,
                 forward: Optional[Callable[[bytes, bytes, object], object]] = None,
                 shared_dispatch: Optional[Callable[[object, bytes, object], object]] = None,
                 fallback: Optional[Callable[[bytes], List[Tuple[bytes, object]]]] = None,
                 fallback_dispatch: Optional[Callable[[bytes, object], object]] = None,
                 on_dropped: Optional[Callable[[object], None]] = None,
                 persist: Optional[Callable[[bytes, object], None]] = None,
                 routes: Optional[GpuRoutes] = None):
        if routes is None and isinstance(getattr(groups_fn, "__self__", None), GpuRoutes):
            routes = groups_fn.__self__
        if groups_fn is None:
            if routes is None:
                raise TypeError("PublishBatcher needs groups_fn or routes")
            groups_fn = routes.groups
        if routes is not None:
            if others is None:
                others = routes.other
            if subscribers is None:
                subscribers = routes.subs
        self.groups_fn = groups_fn
        self.max_batch = max_batch
        self.window_s = window_s
        self.subscribers = subscribers if subscribers is not None else {}
        self.deliver = deliver or (lambda sub, filt, msg: sub.append((filt, msg)) or True)
        self.clock = clock
        self.node = _b(node)
        self.lookup_routes = lookup_routes or (lambda f: [])
        self.others = others if others is not None else {}
        self.forward = forward or (lambda node, f, msg: ("error", "badrpc"))
        self.shared_dispatch = shared_dispatch or (lambda group, f, msg: ("error", "no_subscribers"))
        self.fallback = fallback
        self.fallback_dispatch = fallback_dispatch or (lambda f, msg: ("error", "no_subscribers"))
        self.on_dropped = on_dropped or (lambda msg: None)
        self.persist = persist or (lambda topic, msg: None)
        self.metrics = {"messages.publish": 0, "messages.dropped": 0, "messages.dropped.no_subscribers": 0}
        self.batches = 0
        self.messages = 0
        self._mlock = threading.Lock()
        self._pending: List[Tuple[bytes, Future]] = []
        self._deadline: Optional[float] = None
        self._cv = threading.Condition()
        self._closed = False
        self._thread = None
        if timer:
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()

    # ---------------------------------------------------------------- server side
    def submit(self, topic) -> Future:
        """Queue one topic's match; the future resolves to ("ok", row) or
        ("error", reason) once its batch is matched (at most window_s after the
        batch's first topic)."""
        fut: Future = Future()
        flush = None
        with self._cv:
            self._pending.append((_b(topic), fut))
            if len(self._pending) == 1:
                self._deadline = self.clock() + self.window_s  # the window starts with the batch
                self._cv.notify()
            if len(self._pending) >= self.max_batch:
                flush = self._take()
        if flush:
            self._match(flush)
        return fut

    def poll(self) -> int:
        """Flush if the window has expired (the timer thread's step; tests call it
        with a fake clock).  Returns the number of topics matched."""
        with self._cv:
            due = self._pending and self._deadline is not None and self.clock() >= self._deadline
            batch = self._take() if due else []
        if batch:
            self._match(batch)
        return len(batch)

    def flush(self) -> int:
        with self._cv:
            batch = self._take()
        if batch:
            self._match(batch)
        return len(batch)

    def close(self):
        with self._cv:
            self._closed = True
            self._cv.notify()
        if self._thread:
            self._thread.join()
        self.flush()

    def _take(self):
        batch, self._pending, self._deadline = self._pending, [], None
        return batch

    def _run(self):
        while True:
            with self._cv:
                while not self._closed and not self._pending:
                    self._cv.wait()
                if self._closed:
                    return
                wait = self._deadline - self.clock() if self._deadline is not None else 0.0
                if wait > 0:
                    self._cv.wait(timeout=wait)
            self.poll()

    def _rows(self, topics: Sequence[bytes]):
        try:
            return [("ok", r) for r in self.groups_fn(list(topics))]
        except Exception as e:  # the NIF's {error, _}: every caller takes the reference path
            return [("error", str(e))] * len(topics)

    def _match(self, batch):
        rows = self._rows([t for t, _ in batch])
        with self._mlock:
            self.batches += 1
            self.messages += len(batch)
        for (_, fut), row in zip(batch, rows):
            fut.set_result(row)

    # ---------------------------------------------------------------- caller side
    def _inc(self, name: str):
        with self._mlock:
            self.metrics[name] += 1

    def prepare(self, topic, msg):
        """publish/1 before the match: the publish metric (not for $SYS) and
        persist_message/1 (the 'message.publish' hook is the caller's own)."""
        t = _b(topic)
        if not is_sys(t):
            self._inc("messages.publish")
        self.persist(t, msg)
        return t

    def publish(self, topic, msg=None) -> Result:
        """emqx_broker:publish/1 with the match batched: blocks until the batch
        holding the topic is matched, then routes in the calling thread."""
        t = self.prepare(topic, msg)
        return self.route_row(self.submit(t).result(), t, msg)

    def publish_batch(self, items: Sequence[Tuple[object, object]]) -> List[Result]:
        """Messages the caller already holds: one groups call, results in order."""
        topics = [self.prepare(t, m) for t, m in items]
        rows = self._rows(topics)
        with self._mlock:
            self.batches += 1
            self.messages += len(topics)
        return [self.route_row(r, t, m) for r, t, (_, m) in zip(rows, topics, items)]

    def route_row(self, row, topic: bytes, msg) -> Result:
        """route(aggre(Routes)) over a matched row (emqx_broker.erl:245-273)."""
        if row[0] == "ok":
            routes: List[tuple] = [(f, self.node, ids) for f, ids in row[1] if len(ids)]
            other = [(f, d) for f, _ in row[1] if f in self.others for d in self.lookup_routes(f)
                     if isinstance(d, tuple) or _b(d) != self.node]
        else:  # the reference path
            routes, other = [], list(self.fallback(topic)) if self.fallback else []
        routes += self.aggre(other)
        if not routes:  # route([], _): no subscribers anywhere
            self.dropped(topic, msg)
            return []
        out: Result = []
        for r in routes:  # lists:foldl prepending, as route/2
            out.insert(0, self.do_route(r, topic, msg))
        return out

    @staticmethod
    def aggre(routes: Sequence[Tuple[bytes, object]]) -> List[tuple]:
        """aggre/1: (filter, node) per node route, one (filter, group) per shared group."""
        nodes = [(f, _b(d)) for f, d in routes if not isinstance(d, tuple)]
        groups = sorted({(f, ("group", d[0])) for f, d in routes if isinstance(d, tuple)})
        return nodes + groups

    def do_route(self, r, topic: bytes, msg):
        if len(r) == 3:  # a local route with the GPU fan-out's subscriber ids
            f, node, ids = r
            return (node, f, self.dispatch_ids(f, ids, topic, msg))
        f, d = r
        if isinstance(d, tuple):  # ("group", G): emqx_shared_sub:dispatch/3
            return ("share", f, self.shared_dispatch(d[1], f, msg))
        if _b(d) == self.node:
            return (d, f, self.fallback_dispatch(f, msg))
        return (d, f, self.forward(d, f, msg))

    def dispatch_ids(self, f: bytes, ids, topic: bytes, msg):
        """do_dispatch/2,3: one delivery per live subscriber; none live is a drop."""
        n = 0
        for sid in (ids.tolist() if hasattr(ids, "tolist") else ids):
            sub = self.subscribers.get(int(sid))
            if sub is not None and self.deliver(sub, f, msg):
                n += 1
        if n:
            return ("ok", n)
        self.dropped(topic, msg)
        return ("error", "no_subscribers")

    def dropped(self, topic: bytes, msg):
        """'message.dropped' hook + inc_dropped_cnt/1 (emqx_broker.erl:245-248, 309-314)."""
        self.on_dropped(msg)
        if not is_sys(topic):
            self._inc("messages.dropped")
            self._inc("messages.dropped.no_subscribers")
