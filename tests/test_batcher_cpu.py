"""The publish aggregator (emqx_amd/batcher.py, the mirror of
nif/emqx_gpu_match_batcher.erl) on the CPU: a fake clock and a fake groups
function stand in for the GPU call, which tests/test_gpu_mirror.py covers.
Server side: the size/time window.  Caller side: emqx_broker:publish/1's
route/2, do_route/2 and do_dispatch/2 around the batched match
(apps/emqx/src/emqx_broker.erl:204-215, 245-273, 296-322, 506-530)."""

import threading

import numpy as np

from emqx_amd.batcher import PublishBatcher


class Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def groups_table(table):
    """groups_fn from a {topic: [(filter, [sid])]} table; records each batch."""
    calls = []

    def fn(topics):
        calls.append(list(topics))
        return [[(f, np.array(s, np.uint32)) for f, s in table.get(t, [])] for t in topics]
    return fn, calls


def test_window_flushes_on_time_not_before():
    clk = Clock()
    fn, calls = groups_table({b"a/b": [(b"a/+", [1, 2])]})
    b = PublishBatcher(fn, max_batch=100, window_s=0.002, clock=clk, timer=False)
    futs = [b.submit("a/b") for _ in range(3)]
    clk.t = 0.0019
    assert b.poll() == 0 and not calls
    clk.t = 0.002
    assert b.poll() == 3
    assert calls == [[b"a/b"] * 3]  # ONE batch, arrival order
    for f in futs:
        ok, row = f.result()
        assert ok == "ok" and [(g, s.tolist()) for g, s in row] == [(b"a/+", [1, 2])]


def test_size_trigger_and_window_restart():
    clk = Clock()
    fn, calls = groups_table({})
    b = PublishBatcher(fn, max_batch=4, window_s=1.0, clock=clk, timer=False)
    futs = [b.submit(f"t/{i}") for i in range(4)]  # the 4th fills the batch: matched inline
    assert len(calls) == 1 and len(calls[0]) == 4
    assert all(f.done() and f.result() == ("ok", []) for f in futs)
    clk.t = 5.0
    f = b.submit("x")  # a new window starts with the next batch's first topic
    clk.t = 5.9
    assert b.poll() == 0
    clk.t = 6.0
    assert b.poll() == 1 and f.result() == ("ok", [])
    assert b.batches == 2 and b.messages == 5


def test_local_dispatch_follows_do_dispatch():
    """{ok, N} over live subscribers only; {error, no_subscribers} plus a drop
    when none is live (emqx_broker.erl:506-530); a subscriber of two matching
    filters is delivered twice (emqx_persistent_session_SUITE.erl:705)."""
    fn, _ = groups_table({b"s/1": [(b"s/#", [7, 9]), (b"s/+", [7]), (b"+/1", [42])]})
    inbox = {7: [], 9: []}
    dropped = []
    b = PublishBatcher(fn, subscribers=inbox, timer=False, on_dropped=dropped.append)
    (res,) = b.publish_batch([(b"s/1", "m")])
    assert sorted(res) == sorted([(b"node", b"s/#", ("ok", 2)), (b"node", b"s/+", ("ok", 1)),
                                  (b"node", b"+/1", ("error", "no_subscribers"))])
    assert inbox[7] == [(b"s/#", "m"), (b"s/+", "m")] and inbox[9] == [(b"s/#", "m")]
    assert dropped == ["m"]  # do_dispatch's 'message.dropped' for the filter with no live subscriber
    assert b.metrics["messages.dropped.no_subscribers"] == 1 and b.metrics["messages.publish"] == 1


def test_remote_and_shared_routes_come_back_as_route_entries():
    """Filters with other destinations: lookup_routes/1 for those filters only;
    a remote node is forwarded, a shared group dispatched once per group
    (aggre/1's usort), the local subscribers from the fan-out row."""
    fn, _ = groups_table({b"a/b": [(b"a/+", [1]), (b"a/#", []), (b"a/b", [])]})
    routes = {b"a/+": [b"node", b"n2"], b"a/#": [(b"g1", b"node"), (b"g1", b"n3"), b"n3"],
              b"a/b": [(b"g2", b"n2")]}
    looked, fwd, shared = [], [], []

    def lookup(f):
        looked.append(f)
        return routes[f]
    inbox = {1: []}
    b = PublishBatcher(fn, subscribers=inbox, timer=False, lookup_routes=lookup, others={b"a/+", b"a/#", b"a/b"},
                       forward=lambda n, f, m: fwd.append((n, f, m)) or ("ok", 1),
                       shared_dispatch=lambda g, f, m: shared.append((g, f, m)) or ("ok", 1))
    (res,) = b.publish_batch([(b"a/b", "m")])
    assert sorted(looked) == [b"a/#", b"a/+", b"a/b"]
    assert sorted(res, key=repr) == sorted([
        (b"node", b"a/+", ("ok", 1)),          # local, from the fan-out row
        (b"n2", b"a/+", ("ok", 1)),            # forward/4
        (b"n3", b"a/#", ("ok", 1)),
        ("share", b"a/#", ("ok", 1)),          # group g1 once for its two nodes
        ("share", b"a/b", ("ok", 1))], key=repr)
    assert sorted(fwd) == [(b"n2", b"a/+", "m"), (b"n3", b"a/#", "m")]
    assert sorted(shared) == [(b"g1", b"a/#", "m"), (b"g2", b"a/b", "m")]
    assert inbox[1] == [(b"a/+", "m")]


def test_no_route_is_a_drop_and_sys_is_not_counted():
    fn, _ = groups_table({})
    dropped = []
    b = PublishBatcher(fn, timer=False, on_dropped=dropped.append)
    assert b.publish_batch([(b"x/y", ("x", 1)), (b"$SYS/a", ("sys", 2))]) == [[], []]
    assert dropped == [("x", 1), ("sys", 2)]  # the hook runs for both (route([], _))
    assert b.metrics == {"messages.publish": 1, "messages.dropped": 1, "messages.dropped.no_subscribers": 1}


def test_persist_runs_before_the_match():
    order = []

    def fn(topics):
        order.append(("match", list(topics)))
        return [[] for _ in topics]
    b = PublishBatcher(fn, timer=False, persist=lambda t, m: order.append(("persist", t)))
    b.publish_batch([(b"p/1", 1), (b"p/2", 2)])
    assert order == [("persist", b"p/1"), ("persist", b"p/2"), ("match", [b"p/1", b"p/2"])]


def test_engine_error_takes_the_reference_path():
    """{error, _} from the batch: every caller routes with match_routes/1."""
    def boom(topics):
        raise RuntimeError("EDEVICE")
    disp = []
    b = PublishBatcher(boom, timer=False, fallback=lambda t: [(t, b"node"), (t, b"n2")],
                       fallback_dispatch=lambda f, m: disp.append((f, m)) or ("ok", 3),
                       forward=lambda n, f, m: ("ok", 1))
    f = b.submit("a")
    b.flush()
    assert f.result()[0] == "error"
    (res,) = b.publish_batch([(b"a", "m")])
    assert sorted(res, key=repr) == sorted([(b"node", b"a", ("ok", 3)), (b"n2", b"a", ("ok", 1))], key=repr)
    assert disp == [(b"a", "m")]


def test_timer_thread_flushes_a_partial_batch():
    fn, calls = groups_table({b"q": [(b"q", [1])]})
    inbox = {1: []}
    b = PublishBatcher(fn, max_batch=1000, window_s=0.005, subscribers=inbox)
    try:
        res = []
        th = [threading.Thread(target=lambda i=i: res.append(b.publish("q", i))) for i in range(10)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=5)
        assert res == [[(b"node", b"q", ("ok", 1))]] * 10
        assert sum(len(c) for c in calls) == 10 and len(inbox[1]) == 10
    finally:
        b.close()


def test_concurrent_publishers():
    fn, calls = groups_table({})
    b = PublishBatcher(fn, max_batch=64, window_s=0.002)
    out, lock = [], threading.Lock()

    def pub(k):
        for i in range(200):
            r = b.publish(f"p{k}/{i}")
            with lock:
                out.append(r)
    th = [threading.Thread(target=pub, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    b.close()
    assert len(out) == 1600 and all(r == [] for r in out)
    assert b.messages == 1600 and sum(len(c) for c in calls) == 1600
    assert max(len(c) for c in calls) <= 64
    assert b.metrics["messages.dropped"] == 1600


# ---------------------------------------------------------------------------
# GpuRoutes bookkeeping on the CPU: a dict-backed stand-in for the context
# (the real emqx_gm_index_update_subs path is tests/test_gpu_mirror.py)
# ---------------------------------------------------------------------------
class _FakeIndex:
    def __init__(self, lists, marks):
        self.lists, self.marks = lists, marks
        self.names = sorted(f for f in set(lists) | marks if lists.get(f) or f in marks)

    def subscriber_count(self, fid):
        return len(self.lists.get(self.names[fid], []))

    def filter(self, fid):
        return self.names[fid]


class _FakeCtx:
    """build_index / update_subs / match / fanout / match_fanout over Python dicts, ids = rank of
    the filter bytes (the library's id rule), matching by emqx_amd.topic.match."""

    def build_index(self, filters, subs=None):
        return _FakeIndex({}, set())

    def update_subs(self, idx, ops):
        lists = {f: list(v) for f, v in idx.lists.items()}
        marks = set(idx.marks)
        for f, sid, op in ops:
            cur = lists.setdefault(f, [])
            if op == "subscribe" and sid not in cur:
                cur.append(sid)
            elif op == "unsubscribe" and sid in cur:
                cur.remove(sid)
            elif op == "route_add":
                marks.add(f)
            elif op == "route_delete":
                marks.discard(f)
        return _FakeIndex(lists, marks)

    def match(self, idx, topics, exact=True):
        from emqx_amd.topic import match
        rows = [[i for i, f in enumerate(idx.names) if match(t, f)] for t in topics]
        ro = np.zeros(len(rows) + 1, np.uint64)
        ro[1:] = np.cumsum([len(r) for r in rows])
        return ro, np.array([i for r in rows for i in r], np.uint32)

    def fanout(self, idx, ro, ids):
        segs = [idx.lists.get(idx.names[int(i)], []) for i in ids]
        out = np.zeros(len(ro), np.uint64)
        for k in range(len(ro) - 1):
            out[k + 1] = out[k] + sum(len(segs[j]) for j in range(int(ro[k]), int(ro[k + 1])))
        return out, np.array([s for seg in segs for s in seg], np.uint32)

    def match_fanout(self, idx, topics, exact=True):  # (emqx_gm_match_fanout: the two in one call)
        m = self.match(idx, topics, exact)
        return m, self.fanout(idx, *m)


def test_subscriber_ids_are_never_reused_after_down():
    """a subscriber that goes down must not lend its id to the next
    new subscriber (next_id in nif/emqx_gpu_match_batcher.erl is monotonic)."""
    from emqx_amd.batcher import GpuRoutes
    routes = GpuRoutes(_FakeCtx())
    ia, ib = [], []
    routes.subscribe("t/+", "a")
    routes.subscribe("t/#", "b")
    routes.subscriber_down("a")
    routes.subscribe("t/1", "c")
    assert routes.ids["c"] not in (0, 1) and routes.ids["b"] == 1
    inbox = {"b": ib, "c": ia}
    b = PublishBatcher(routes=routes, timer=False,
                       deliver=lambda sub, f, m: inbox[sub].append((f, m)) or True)
    (res,) = b.publish_batch([(b"t/1", "m")])
    assert ib == [(b"t/#", "m")] and ia == [(b"t/1", "m")]
    assert sorted(res) == sorted([(b"node", b"t/#", ("ok", 1)), (b"node", b"t/1", ("ok", 1))])


def test_batcher_takes_the_routes_other_table():
    """groups_fn=routes.groups alone wires routes.other, so a remote
    route is forwarded; a str node name is the local node, not a remote one."""
    from emqx_amd.batcher import GpuRoutes
    routes = GpuRoutes(_FakeCtx(), node="n1")
    routes.subscribe("r/+", "s")
    routes.route_add("r/+", "n1")      # the local node as str: no ?OTHER entry
    routes.route_add("r/+", b"n2")
    assert routes.other == {b"r/+": 1}
    fwd = []
    b = PublishBatcher(routes.groups, timer=False, node="n1", subscribers={0: []},
                       lookup_routes=lambda f: ["n1", b"n2"],
                       forward=lambda n, f, m: fwd.append((n, f)) or ("ok", 1))
    (res,) = b.publish_batch([(b"r/x", "m")])
    assert fwd == [(b"n2", b"r/+")]
    assert sorted(res) == sorted([(b"n1", b"r/+", ("ok", 1)), (b"n2", b"r/+", ("ok", 1))])
