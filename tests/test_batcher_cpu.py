"""The publish aggregator's window logic (emqx_amd/batcher.py, the mirror of
nif/emqx_gpu_match_batcher.erl) on the CPU: a fake clock and a fake groups
function stand in for the GPU call, which tests/test_gpu_mirror.py covers."""

import threading

import numpy as np
import pytest

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
    inbox = {1: [], 2: []}
    b = PublishBatcher(fn, max_batch=100, window_s=0.002, subscribers=inbox, clock=clk, timer=False)
    futs = [b.publish("a/b", m) for m in ("m1", "m2", "m3")]
    clk.t = 0.0019
    assert b.poll() == 0 and not calls
    clk.t = 0.002
    assert b.poll() == 3
    assert calls == [[b"a/b"] * 3]  # ONE batch, arrival order
    assert [f.result() for f in futs] == [[(b"a/+", ("ok", 2))]] * 3
    assert inbox[1] == [(b"a/+", "m1"), (b"a/+", "m2"), (b"a/+", "m3")]


def test_size_trigger_and_window_restart():
    clk = Clock()
    fn, calls = groups_table({})
    b = PublishBatcher(fn, max_batch=4, window_s=1.0, clock=clk, timer=False)
    futs = [b.publish(f"t/{i}") for i in range(4)]  # the 4th fills the batch: dispatched inline
    assert len(calls) == 1 and len(calls[0]) == 4
    assert all(f.done() and f.result() == [] for f in futs)  # no route: dropped, publish_result []
    clk.t = 5.0
    f = b.publish("x")  # a new window starts with the next batch's first message
    clk.t = 5.9
    assert b.poll() == 0
    clk.t = 6.0
    assert b.poll() == 1 and f.result() == []
    assert b.batches == 2 and b.messages == 5


def test_dispatch_results_follow_do_dispatch():
    """{ok, N} over live subscribers only; {error, no_subscribers} when none is
    live (emqx_broker.erl:506-530); a subscriber of two matching filters is
    delivered twice (emqx_persistent_session_SUITE.erl:705)."""
    fn, _ = groups_table({b"s/1": [(b"s/#", [7, 9]), (b"s/+", [7]), (b"+/1", [42])]})
    inbox = {7: [], 9: []}
    b = PublishBatcher(fn, subscribers=inbox, timer=False)
    (res,) = b.publish_batch([(b"s/1", "m")])
    assert res == [(b"s/#", ("ok", 2)), (b"s/+", ("ok", 1)), (b"+/1", ("error", "no_subscribers"))]
    assert inbox[7] == [(b"s/#", "m"), (b"s/+", "m")] and inbox[9] == [(b"s/#", "m")]


def test_engine_error_fails_the_batch():
    def boom(topics):
        raise RuntimeError("EDEVICE")
    b = PublishBatcher(boom, timer=False)
    f = b.publish("a")
    b.flush()
    with pytest.raises(RuntimeError):
        f.result()


def test_timer_thread_flushes_a_partial_batch():
    fn, calls = groups_table({b"q": [(b"q", [1])]})
    inbox = {1: []}
    b = PublishBatcher(fn, max_batch=1000, window_s=0.005, subscribers=inbox)
    try:
        futs = [b.publish("q", i) for i in range(10)]
        assert [f.result(timeout=5) for f in futs] == [[(b"q", ("ok", 1))]] * 10
        assert sum(len(c) for c in calls) == 10 and len(inbox[1]) == 10
    finally:
        b.close()


def test_concurrent_publishers():
    fn, calls = groups_table({})
    b = PublishBatcher(fn, max_batch=64, window_s=0.002)
    futs, lock = [], threading.Lock()

    def pub(k):
        for i in range(200):
            f = b.publish(f"p{k}/{i}")
            with lock:
                futs.append(f)
    th = [threading.Thread(target=pub, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(f.result(timeout=5) == [] for f in futs)
    b.close()
    assert b.messages == 1600 and sum(len(c) for c in calls) == 1600
    assert max(len(c) for c in calls) <= 64
