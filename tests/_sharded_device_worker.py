"""The device-tensor (RCCL) path of ShardedMatcher on one GPU, with the
all-to-all replayed from recorded send buffers (tests/test_gpu_sharded.py::
test_device_tensor_path_with_replayed_exchange).  torch's device runtime is
initialised before the library, as in bench.py."""

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _RecordExchange:
    """A `dist` stand-in that records what one rank sends in each all_to_all_single."""

    def __init__(self):
        self.sends = []

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None, group=None):
        self.sends.append((inp.clone(), input_split_sizes))
        out.zero_()


class _ReplayExchange:
    """Rank `rank`'s receive side of the exchange, assembled from every rank's
    recorded sends: piece p = the part of rank p's send buffer addressed to `rank`."""

    def __init__(self, recorders, rank):
        self.recorders, self.rank, self.k = recorders, rank, 0

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None, group=None):
        import torch
        chunks = []
        for rec in self.recorders:
            t, splits = rec.sends[self.k]
            if splits is None:
                size = t.numel() // len(self.recorders)
                chunks.append(t[self.rank * size:(self.rank + 1) * size])
            else:
                off = sum(splits[:self.rank])
                chunks.append(t[off:off + splits[self.rank]])
        self.k += 1
        out.copy_(torch.cat(chunks).to(out.device))


def main():
    torch.zeros(1, device="cuda:0")  # torch's runtime first, as bench.py's dist_setup
    from emqx_amd import Context
    from emqx_amd.engine import pack
    from oracle import oracle as orc
    from tests.test_gpu_sharded import _oracle_rows, _sets, _to_device
    ctx = Context(0)
    from emqx_amd.sharded import ShardedMatcher, plan_shard, slice_bounds
    fs, ts = _sets("c1")
    fb, fo = pack(fs)
    tb, to = pack(ts)
    d_tb, d_to = _to_device(ctx, tb, to)
    n, W = len(ts), 2
    idxs = []
    for q in range(W):
        sfb, sfo, gids, _ = plan_shard(fb, fo, W, q)
        idxs.append(ctx.build_index_shard((sfb, sfo), gids))
    recs = [_RecordExchange() for _ in range(W)]
    for q in range(W):
        res, _, _ = ShardedMatcher(ctx, idxs[q], W, q, dist=recs[q], device_tensors=True).match_device(d_tb, d_to, n)
        torch.cuda.synchronize()  # the recorded sends were written on that matcher's stream
        res.free()
    out, first, rows = ShardedMatcher(ctx, idxs[0], W, 0, dist=_ReplayExchange(recs, 0),
                                      device_tensors=True).match_device(d_tb, d_to, n)
    torch.cuda.synchronize()
    S, b = slice_bounds(n, W)
    assert (first, rows) == (0, S)
    mro, mids = out.rows(0, rows)
    full = ctx.build_index((fb, fo))
    r = ctx.match_device(full, d_tb, d_to, n, exact=True)
    fro, fids = r.rows(0, rows)
    assert np.array_equal(mro, fro) and np.array_equal(mids, fids)
    oro, oids = _oracle_rows(orc, fs, *pack(ts[:rows]))
    assert np.array_equal(mro, oro) and np.array_equal(mids, oids)
    ctx.set_stream(0)
    for x in (out, r):
        x.free()
    for i in idxs + [full]:
        i.release()
    ctx.dev_free(d_tb)
    ctx.dev_free(d_to)
    ctx.close()
    print("SHARDED_DEVICE_PATH_OK", flush=True)


if __name__ == "__main__":
    main()
