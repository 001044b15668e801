"""The device-tensor path of PrefixShardedMatcher.match_device on one GPU
(tests/test_gpu_sharded.py::test_prefix_device_path_*).

World 1: route_partition on the device, then -- one shard, so the send order
is the batch order -- the batch walked in place (the permute and un-permute
would be identity copies: aliased).

World W > 1: W ranks run as W threads of this process, each with its own
library context and matcher (own stream) over its own prefix shard, and the
collective is a lock-step stand-in: every rank deposits its send buffer, waits
for the others, and copies out the pieces addressed to it -- what
all_to_all_single does across GPUs (two RCCL ranks cannot share one GPU).
Every rank's rows of its own batch must equal the unsharded index's rows, and
rank 0's first window the oracle's.  torch's device runtime is initialised
before the library, as in bench.py.

usage: _prefix_device_worker.py WORLD N_FILTERS TOPICS_PER_RANK [libfirst | chunks=K]

chunks=K (world > 1): the matcher's step in K chunks (default 2: each chunk's
exchange issued before the previous chunk's walk; 1: unchunked).

libfirst (world 1): the library's Context is made BEFORE anything touches
torch's device (emqx_amd.Context brings torch's runtime up first itself), and
the topics are written by torch ops on torch's default stream with
non-blocking copies -- the matcher's stream must wait for them, and the
caller's stream for the matcher's rows.
"""

import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class LockstepExchange:
    """all_to_all_single among W threads (the ranks) on one device."""

    def __init__(self, world):
        self.world = world
        self.slots = [None] * world
        self.barrier = threading.Barrier(world, timeout=120)
        self.calls = [0] * world

    def rank(self, r):
        ex = self

        class View:
            def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None, group=None,
                                  async_op=False):
                W = ex.world
                torch.cuda.current_stream().synchronize()  # this rank's send buffer is written
                ex.slots[r] = (inp, input_split_sizes)
                ex.calls[r] += 1
                ex.barrier.wait()
                chunks = []
                for p in range(W):
                    t, splits = ex.slots[p]
                    if splits is None:
                        size = t.numel() // W
                        chunks.append(t[r * size:(r + 1) * size])
                    else:
                        off = sum(splits[:r])
                        chunks.append(t[off:off + splits[r]])
                got = torch.cat(chunks) if chunks else out[:0]
                assert got.numel() == out.numel(), (r, got.numel(), out.numel())
                if out.numel():
                    out.copy_(got)
                torch.cuda.current_stream().synchronize()  # copied before a peer reuses its buffer
                ex.barrier.wait()
                if async_op:  # (done already: a completed work handle)
                    class Done:
                        def wait(self):
                            return True
                    return Done()
        return View()


def main():
    W, n_f, n = (int(x) for x in sys.argv[1:4])
    libfirst = len(sys.argv) > 4 and sys.argv[4] == "libfirst"
    chunks = int(sys.argv[4].split("=")[1]) if len(sys.argv) > 4 and sys.argv[4].startswith("chunks=") else 2
    if libfirst:
        from emqx_amd import Context
        Context(0).close()  # the library first: its Context initialises torch's runtime itself
    torch.zeros(1, device="cuda:0")
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    from emqx_amd.sharded import PrefixShardedMatcher, plan_prefix_shard
    codes = gen_filter_codes(1, n_f)
    fb, fo = render_codes(codes)
    ctxs = [Context(0) for _ in range(W)]
    plans = [plan_prefix_shard(fb, fo, W, q) for q in range(W)]
    idxs = [ctxs[q].build_index_shard((plans[q][0], plans[q][1]), plans[q][2]) for q in range(W)]
    batches = [ctxs[q].gen_topics_device(codes, 1, q * n, n) for q in range(W)]
    keep = []
    if libfirst:  # the same topics written by torch ops on the default stream, not yet complete when matched
        from oracle import oracle as orc
        tb, to = orc.render_codes(orc.gen_topic_codes(1, 0, n, codes))
        t_tb = torch.from_numpy(np.concatenate([tb, np.zeros(64, np.uint8)])).pin_memory().to("cuda:0",
                                                                                              non_blocking=True)
        t_to = torch.from_numpy(to.view(np.int64)).pin_memory().to("cuda:0", non_blocking=True)
        t_tb2 = t_tb.clone()  # (more default-stream work in front of the match)
        keep = [t_tb, t_to, t_tb2]
        batches = [(t_tb2.data_ptr(), t_to.data_ptr(), int(to[-1]))]
    ex = LockstepExchange(W)
    results, walked, errors, matchers = [None] * W, [0] * W, [], [None] * W

    def rank_main(q):
        try:
            m = matchers[q] = PrefixShardedMatcher(ctxs[q], idxs[q], plans[q][4], W, q,
                                                   dist=ex.rank(q) if W > 1 else None, chunks=chunks)
            db, do, _ = batches[q]
            for _ in range(2):  # twice: the second step reuses the matcher's stream and buffers
                if results[q] is not None:
                    results[q].free()
                results[q] = m.match_device(db, do, n)
            walked[q] = m.last_topics_walked
            torch.cuda.current_stream().synchronize()
            m.stream.synchronize()
        except BaseException as e:  # noqa: BLE001 (reported by the main thread)
            errors.append((q, repr(e)))
            ex.barrier.abort()

    th = [threading.Thread(target=rank_main, args=(q,)) for q in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    assert sum(walked) == W * n, walked
    if W > 1:
        assert max(walked) < 2 * n, walked  # each rank walks about its share, not the whole job
        K = matchers[0].chunks
        # per step: six collectives unchunked; chunked, one for every chunk's sizes + five per chunk
        assert ex.calls[0] == 2 * (6 if K == 1 else 1 + 5 * K), ex.calls
    full_ctx = Context(0)
    full = full_ctx.build_index((fb, fo))
    for q in range(W):
        db, do, _ = batches[q]
        ref = full_ctx.match_device(full, db, do, n, exact=True)
        fro, fids = ref.to_host()
        ref.free()
        ro, ids = results[q].to_host()
        assert np.array_equal(ro, fro), q
        assert np.array_equal(ids, fids), q
    from oracle import oracle as orc
    import bench
    k = min(n, 20_000)
    tb, to = orc.render_codes(orc.gen_topic_codes(1, 0, k, codes))
    r = orc.Router(True)
    r.add_routes((fb, fo))
    oro, oids, _ = r.match_batch((tb, to), orc.Ranker(bench.sorted_unique(fb, fo)), mode=1, nthreads=8)
    ro, ids = results[0].rows(0, k)
    assert np.array_equal(ro, oro) and np.array_equal(ids, oids)
    for q in range(W):
        results[q].free()
        ctxs[q].set_stream(0)
        if not libfirst:
            ctxs[q].dev_free(batches[q][0])
            ctxs[q].dev_free(batches[q][1])
        idxs[q].release()
        plans[q][4].release()
        ctxs[q].close()
    full.release()
    full_ctx.close()
    del keep
    print(f"PREFIX_DEVICE_PATH_OK world={W} walked={walked} chunks={chunks}{' libfirst' if libfirst else ''}",
          flush=True)


if __name__ == "__main__":
    main()
