"""One rank of the C4 split rehearsal (tests/test_gpu_parity.py::test_fanout_split_two_ranks).

Every rank builds the 1/10-scale C4 index on device 0, matches the hot topics
and produces its part of the delivery range (emqx_gm_fanout_part); the parts
are gathered over gloo and rank 0 checks that they are disjoint, cover every
delivery exactly once and, concatenated in rank order, equal the oracle's
do_dispatch fold (emqx_broker.erl:506-530)."""

import ctypes
import os
import sys

import numpy as np
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def c4_small(K=100, S=100_000):
    filters = [b"hot/#", b"hot/+/x/#"] + [b"hot/%d/x/y/z" % k for k in range(K)]
    subs = [list(range(0, 60_000)), list(range(60_000, S - 10 * K))] + \
           [list(range(S - 10 * K + 10 * k, S - 10 * K + 10 * k + 10)) for k in range(K)]
    topics = [b"hot/%d/x/y/z" % k for k in range(K)]
    return filters, subs, topics


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from emqx_amd import Context
    from emqx_amd.engine import pack
    filters, subs, topics = c4_small()
    ctx = Context(0)
    idx = ctx.build_index(filters, subs=subs)
    tb, to = pack(topics)
    d_tb, d_to = ctx.dev_alloc(len(tb)), ctx.dev_alloc(len(to) * 8)
    ctx.memcpy_h2d(d_tb, tb, len(tb))
    ctx.memcpy_h2d(d_to, to, len(to) * 8)
    m = ctx.match_device(idx, d_tb, d_to, len(topics), exact=True)
    part, first = ctx.fanout_part(idx, m, rank, world)
    g_ro = np.zeros(len(topics) + 1, np.uint64)  # global delivery offsets
    ctx.memcpy_d2h(g_ro, ctypes.cast(part.csr.row_off, ctypes.c_void_p).value, g_ro.nbytes)
    ids = np.zeros(max(part.nnz, 1), np.uint32)
    if part.nnz:
        ctx.memcpy_d2h(ids, ctypes.cast(part.csr.ids, ctypes.c_void_p).value, part.nnz * 4)
    mro, mids = m.to_host()
    got = [None] * world
    dist.all_gather_object(got, (first, ids[:part.nnz], g_ro))
    if rank == 0:
        from oracle import oracle as orc
        order = np.argsort(idx.perm)
        ssorted = [subs[i] for i in order]
        so = np.zeros(len(filters) + 1, np.uint64)
        so[1:] = np.cumsum([len(s) for s in ssorted])
        si = np.array([x for s in ssorted for x in s], np.uint32)
        ero, eids = orc.fanout(mro, mids, so, si)
        pos = 0
        for q, (f, pids, pro) in enumerate(got):
            assert f == pos, (q, f, pos)  # contiguous, disjoint
            assert np.array_equal(pro, ero), q  # every part carries the global row offsets
            pos += len(pids)
        assert pos == len(eids)  # complete
        assert np.array_equal(np.concatenate([g[1] for g in got]), eids)
        assert min(len(g[1]) for g in got) > 0
        print(f"FANOUT_SPLIT_OK world={world} deliveries={pos}", flush=True)
    part.free()
    m.free()
    ctx.dev_free(d_tb)
    ctx.dev_free(d_to)
    idx.release()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
