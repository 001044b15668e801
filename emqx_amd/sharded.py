"""Sharded index over ranks (BASELINE.json configs[4] "C5").

When the filter set is too large to replicate, filters are hash-partitioned
over the ranks (``emqx_gm_shard_of``) and each rank builds an index over its
shard whose result rows carry GLOBAL filter ids (the filter's lexicographic
rank in the whole set, ``emqx_gm_filter_ranks``).  Every rank matches the
whole publish batch against its shard; then the rows are exchanged so that
rank q ends with topic slice q from every shard -- one all-to-all of the row
lengths and one all-to-all-v of the ids (RCCL over xGMI: each rank sends each
peer only that peer's slice, a direct mesh exchange rather than a ring
all-gather of everything) -- and the pieces are merged on the device by
global id (``emqx_gm_merge_rows``).

The union over shards is exactly the unsharded result: matching is
independent per filter (emqx_topic:match/2, apps/emqx/src/emqx_topic.erl:65-87)
and the shards' id sets are disjoint, so each merged row is the sorted row an
unsharded emqx_gm_match returns for the same topic.
"""

from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .engine import Context, DeviceCsr, Index, filter_ranks, select_filters, shard_of


def slice_bounds(n_rows: int, world: int) -> Tuple[int, List[int]]:
    """Rows per slice S = ceil(n / world) and the slice bounds [0, S, 2S, ..., n]."""
    s = -(-n_rows // world) if n_rows else 0
    return s, [min(q * s, n_rows) for q in range(world + 1)]


def plan_shard(fb: np.ndarray, fo: np.ndarray, world: int, rank: int):
    """This rank's filters (packed), their global ids, and the global filter count."""
    gids, n_unique = filter_ranks(fb, fo)
    sh = shard_of(fb, fo, world)
    sfb, sfo = select_filters(fb, fo, sh, rank)
    return sfb, sfo, gids[sh == rank], n_unique


def exchange_rows(dist, lens, ids, id_bounds: Sequence[int], world: int, group=None):
    """All-to-all of per-slice rows.

    lens: int32 tensor [world * S], this rank's row lengths for the whole batch
    (zero-padded past the last row); ids: int32 tensor, this rank's ids with
    rows in topic order; id_bounds: world + 1 offsets into ids where each slice
    starts.  Returns (recv_lens [world * S]: piece p = rank p's lengths for this
    rank's slice, recv_ids: the pieces' ids concatenated in rank order).
    """
    import torch
    dev = lens.device
    send_counts = [int(id_bounds[q + 1] - id_bounds[q]) for q in range(world)]
    sc = torch.tensor(send_counts, dtype=torch.int64, device=dev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(x) for x in rc.tolist()]
    # never a NULL buffer, also when nothing is received (the merge takes a device pointer)
    recv_ids = torch.empty(max(sum(recv_counts), 1), dtype=torch.int32, device=dev)[:sum(recv_counts)]
    dist.all_to_all_single(recv_ids, ids, output_split_sizes=recv_counts, input_split_sizes=send_counts,
                           group=group)
    recv_lens = torch.empty_like(lens)
    dist.all_to_all_single(recv_lens, lens, group=group)
    return recv_lens, recv_ids


def _ptr(p) -> int:
    return C.cast(p, C.c_void_p).value or 0


class ShardedMatcher:
    """match_routes over a filter set sharded across ranks (one process per GPU).

    ``device_tensors`` True exchanges device buffers (RCCL, backend "nccl");
    False stages them through host memory (backend "gloo", e.g. several ranks
    sharing one device in tests).  On the device path the library runs on
    torch's current stream (emqx_gm_set_stream), so its kernels, torch's
    tensor ops and the collectives are ordered by one stream: no cross-stream
    race, no device-wide synchronisation between the steps.
    """

    def __init__(self, ctx: Context, index: Index, world: int, rank: int, dist=None, group=None,
                 device_tensors: bool = True):
        self.ctx, self.index, self.world, self.rank = ctx, index, world, rank
        self.dist, self.group, self.device_tensors = dist, group, device_tensors
        self.last_exchange_bytes = 0
        if device_tensors and world > 1:
            import torch
            ctx.set_stream(torch.cuda.current_stream(torch.device("cuda", ctx.device)).cuda_stream)

    def match_device(self, d_tb: int, d_to: int, n: int, exact: bool = True) -> Tuple[DeviceCsr, int, int]:
        """Rows of this rank's topic slice; returns (csr, first_row, n_rows)."""
        ctx = self.ctx
        res = ctx.match_device(self.index, d_tb, d_to, n, exact)
        if self.world == 1:
            return res, 0, n
        import torch
        W, r = self.world, self.rank
        S, b = slice_bounds(n, W)
        nnz = res.nnz
        ids_ptr = _ptr(res.csr.ids)
        if self.device_tensors:
            dev = torch.device("cuda", ctx.device)
            lens = torch.zeros(W * S, dtype=torch.int32, device=dev)  # same stream as the kernel below
            ctx.csr_row_lengths(res, lens.data_ptr())
            ids = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
            ctx.memcpy_d2d(ids.data_ptr(), ids_ptr, nnz * 4)
            # where each peer's slice starts in ids: one device reduction, one D2H of W values
            per = lens.view(W, S).to(torch.int64).sum(1).cumsum(0).cpu().tolist()
            bounds = [0] + [int(x) for x in per]
        else:
            ro_h, ids_h = res.to_host()
            lens = torch.zeros(W * S, dtype=torch.int32)
            lens[:n] = torch.from_numpy(np.diff(ro_h.astype(np.int64)).astype(np.int32))
            ids = torch.from_numpy(ids_h.view(np.int32).copy())
            bounds = [int(ro_h[x]) for x in b]
        res.free()
        rl, ri = exchange_rows(self.dist, lens, ids, bounds, W, self.group)
        self.last_exchange_bytes = 4 * (W * S + int(nnz))
        if self.device_tensors:
            # the storage pointer: a tensor with no elements reports data_ptr() 0
            out = ctx.merge_rows(b[r + 1] - b[r], S, W, rl.data_ptr(), ri.untyped_storage().data_ptr())
        else:
            nl, ni = rl.numel() * 4, max(ri.numel(), 1) * 4
            d_l, d_i = ctx.dev_alloc(nl), ctx.dev_alloc(ni)
            try:
                ctx.memcpy_h2d(d_l, rl.numpy(), nl)
                if ri.numel():
                    ctx.memcpy_h2d(d_i, ri.numpy(), ri.numel() * 4)
                out = ctx.merge_rows(b[r + 1] - b[r], S, W, d_l, d_i)
            finally:
                ctx.dev_free(d_l)
                ctx.dev_free(d_i)
        return out, b[r], b[r + 1] - b[r]
