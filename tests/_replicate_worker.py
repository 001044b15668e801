"""bench.py's replicated_index on its RCCL branch (device tensors), on one GPU:
W ranks as W threads of this process, each with its own library context, and
a lock-step stand-in for torch.distributed.broadcast (every rank deposits its
tensor; the receivers copy rank 0's) -- two RCCL ranks cannot share one GPU.
Rank 0 compiles the index; every other rank imports the broadcast image and
device tables (emqx_gm_index_export / _device_blob / _import) and must answer
a batch exactly as rank 0's build and the oracle do.  torch's device runtime is
initialised before the library, as in bench.py.

usage: _replicate_worker.py WORLD N_FILTERS N_TOPICS
"""

import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class LockstepBroadcast:
    def __init__(self, world):
        self.world, self.slot = world, None
        self.barrier = threading.Barrier(world, timeout=300)
        self.calls = [0] * world

    def rank(self, r):
        ex = self

        class PG:
            def broadcast(self, t, src):
                assert src == 0
                torch.cuda.current_stream().synchronize()
                if r == 0:
                    ex.slot = t
                ex.calls[r] += 1
                ex.barrier.wait()
                if r != 0:
                    assert ex.slot.numel() == t.numel() and ex.slot.dtype == t.dtype
                    t.copy_(ex.slot.to(t.device))
                    torch.cuda.current_stream().synchronize()
                ex.barrier.wait()
        return PG()


def main():
    W, n_f, n = (int(x) for x in sys.argv[1:4])
    torch.zeros(1, device="cuda:0")
    import bench
    assert bench.BACKEND == "nccl"  # the device-tensor branch
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes

    class A:
        build_each = False
        index_cache = None

    codes = gen_filter_codes(1, n_f)
    fpack = render_codes(codes)
    ctxs = [Context(0) for _ in range(W)]
    ex = LockstepBroadcast(W)
    out, errors = [None] * W, []

    def rank_main(q):
        try:
            out[q] = bench.replicated_index(A, ctxs[q], W, q, 0, ex.rank(q), fpack)
        except BaseException as e:  # noqa: BLE001
            errors.append((q, repr(e)))
            ex.barrier.abort()

    th = [threading.Thread(target=rank_main, args=(q,)) for q in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    assert [s for _, s in out] == ["built"] + ["imported"] * (W - 1), out
    assert ex.calls == [3] * W, ex.calls  # sizes, the image, the device tables
    db, do, _ = ctxs[0].gen_topics_device(codes, 1, 0, n)
    rows = []
    for q in range(W):
        idx = out[q][0]
        assert idx.n_filters == out[0][0].n_filters and idx.info.device_bytes == out[0][0].info.device_bytes
        r = ctxs[q].match_device(idx, db, do, n, exact=True)
        rows.append(r.to_host())
        r.free()
    for q in range(1, W):
        assert np.array_equal(rows[q][0], rows[0][0]) and np.array_equal(rows[q][1], rows[0][1]), q
    from oracle import oracle as orc
    k = min(n, 20_000)
    tb, to = orc.render_codes(orc.gen_topic_codes(1, 0, k, codes))
    r = orc.Router(True)
    r.add_routes(fpack)
    oro, oids, _ = r.match_batch((tb, to), orc.Ranker(bench.sorted_unique(*fpack)), mode=1, nthreads=8)
    ro, ids = rows[W - 1]
    assert np.array_equal(ro[:k + 1], oro) and np.array_equal(ids[:int(oro[-1])], oids)
    # an imported replica keeps its in-place update line (its host copy loads on the first update)
    upd = ctxs[W - 1].update_index(out[W - 1][0], [(b"upd/+/x", True), (b"upd/#", True)])
    assert upd.n_filters == out[0][0].n_filters + 2
    upd.release()
    ctxs[0].dev_free(db)
    ctxs[0].dev_free(do)
    for q in range(W):
        out[q][0].release()
        ctxs[q].close()
    print(f"REPLICATE_OK world={W}", flush=True)


if __name__ == "__main__":
    main()
