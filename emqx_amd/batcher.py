"""Publish batching aggregator: the host mirror of nif/emqx_gpu_match_batcher.erl.

The reference publishes one message at a time in the publisher's process
(emqx_broker:publish/1 -> match_routes/1 -> route/2 -> dispatch/2 ->
do_dispatch/2,3; apps/emqx/src/emqx_broker.erl:204-215, 245-260, 296-322,
506-530).  The GPU engine pays off over many topics, so publishes are
collected for at most ``window_s`` seconds or ``max_batch`` messages,
whichever comes first, and the batch goes through the C-ABI sequence the
NIF's fanout_batch/2 makes -- emqx_gm_match (WITH_EXACT) -> emqx_gm_fanout ->
each fan-out row cut back into one (filter, subscriber ids) group per matched
filter (emqx_gm_index_subscriber_count) -- then every subscriber id is
mapped back to its subscriber and sent ``(filter, msg)``, one delivery per
live subscriber, as do_dispatch/3 does.  Each publish gets its own
publish_result back: ``[(filter, ("ok", n) | ("error", "no_subscribers"))]``,
``[]`` when nothing matched (route([], _), a dropped message).

The window logic takes an injectable clock and a groups function, so it is
tested on the CPU; the GPU path is ``FanoutGroups``.
"""

from __future__ import annotations

import threading
import time
from concurrent.futures import Future
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

Group = Tuple[bytes, np.ndarray]  # (filter, subscriber ids)
Result = List[Tuple[bytes, Tuple[str, object]]]


class FanoutGroups:
    """fanout_batch/2 over one index snapshot built with subscriber lists."""

    def __init__(self, ctx, index, filters: Sequence[bytes]):
        self.ctx, self.index, self.filters = ctx, index, list(filters)
        self.counts = np.array([index.subscriber_count(i) for i in range(len(self.filters))], np.int64)

    def __call__(self, topics: Sequence[bytes]) -> List[List[Group]]:
        ro, ids = self.ctx.match(self.index, list(topics), exact=True)
        fro, fids = self.ctx.fanout(self.index, ro, ids)
        out = []
        for k in range(len(ro) - 1):
            row, pos = [], int(fro[k])
            for f in ids[ro[k]:ro[k + 1]]:
                c = int(self.counts[f])
                row.append((self.filters[f], fids[pos:pos + c]))
                pos += c
            assert pos == int(fro[k + 1])
            out.append(row)
        return out


class PublishBatcher:
    """Size/time-window aggregator over a groups function (see module doc)."""

    def __init__(self, groups_fn: Callable[[Sequence[bytes]], List[List[Group]]], max_batch: int = 4096,
                 window_s: float = 0.001, subscribers: Optional[Dict[int, object]] = None,
                 deliver: Optional[Callable[[object, bytes, object], bool]] = None,
                 clock: Callable[[], float] = time.monotonic, timer: bool = True):
        self.groups_fn = groups_fn
        self.max_batch = max_batch
        self.window_s = window_s
        self.subscribers = subscribers if subscribers is not None else {}
        self.deliver = deliver or (lambda sub, filt, msg: sub.append((filt, msg)) or True)
        self.clock = clock
        self.batches = 0
        self.messages = 0
        self._pending: List[Tuple[bytes, object, Future]] = []
        self._deadline: Optional[float] = None
        self._cv = threading.Condition()
        self._closed = False
        self._thread = None
        if timer:
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()

    # ---------------------------------------------------------------- API
    def publish(self, topic, msg=None) -> Future:
        """Queue one publish; the future resolves to its publish_result once
        its batch is dispatched (at most window_s after the batch's first message)."""
        fut: Future = Future()
        t = topic.encode() if isinstance(topic, str) else bytes(topic)
        flush = None
        with self._cv:
            self._pending.append((t, msg, fut))
            if len(self._pending) == 1:
                self._deadline = self.clock() + self.window_s  # the window starts with the batch
                self._cv.notify()
            if len(self._pending) >= self.max_batch:
                flush = self._take()
        if flush:
            self._dispatch(flush)
        return fut

    def publish_batch(self, items: Sequence[Tuple[object, object]]) -> List[Result]:
        """A batch the caller already holds: dispatched at once, results in order."""
        futs = [Future() for _ in items]
        self._dispatch([((t.encode() if isinstance(t, str) else bytes(t)), m, f) for (t, m), f in zip(items, futs)])
        return [f.result() for f in futs]

    def poll(self) -> int:
        """Flush if the window has expired (the timer thread's step; tests call it
        with a fake clock).  Returns the number of messages dispatched."""
        with self._cv:
            due = self._pending and self._deadline is not None and self.clock() >= self._deadline
            batch = self._take() if due else []
        if batch:
            self._dispatch(batch)
        return len(batch)

    def flush(self) -> int:
        with self._cv:
            batch = self._take()
        if batch:
            self._dispatch(batch)
        return len(batch)

    def close(self):
        with self._cv:
            self._closed = True
            self._cv.notify()
        if self._thread:
            self._thread.join()
        self.flush()

    # ---------------------------------------------------------------- internals
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

    def _dispatch(self, batch):
        try:
            rows = self.groups_fn([t for t, _, _ in batch])
        except Exception as e:  # the NIF's {error, _}: every future fails, the caller falls back
            for _, _, f in batch:
                f.set_exception(e)
            return
        self.batches += 1
        self.messages += len(batch)
        for (_, msg, fut), groups in zip(batch, rows):
            res: Result = []
            for filt, sids in groups:
                n = 0
                for sid in sids.tolist():
                    sub = self.subscribers.get(int(sid))
                    if sub is not None and self.deliver(sub, filt, msg):
                        n += 1
                res.append((filt, ("ok", n) if n else ("error", "no_subscribers")))
            fut.set_result(res)
