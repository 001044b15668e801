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


def exchange_rows(dist, lens, ids, id_bounds: Optional[Sequence[int]], world: int, group=None):
    """All-to-all of per-slice rows.

    lens: int32 tensor [world * S], this rank's row lengths for the whole batch
    (zero-padded past the last row); ids: int32 tensor, this rank's ids with
    rows in topic order; id_bounds: world + 1 offsets into ids where each slice
    starts, or None (derived from lens).  Returns (recv_lens [world * S]: piece
    p = rank p's lengths for this rank's slice, recv_ids: the pieces' ids
    concatenated in rank order).

    The row lengths go first (fixed sizes); both the counts this rank sends and
    the counts it receives are then sums over them, so ONE device-to-host copy
    of 2 x world values gives the all-to-all-v its split sizes.
    """
    import torch
    recv_lens = torch.empty_like(lens)
    dist.all_to_all_single(recv_lens, lens, group=group)
    recv_per = recv_lens.view(world, -1).to(torch.int64).sum(1)
    if id_bounds is None:
        send_per = lens.view(world, -1).to(torch.int64).sum(1)
        both = torch.cat([send_per, recv_per]).cpu().tolist()
        send_counts, recv_counts = [int(x) for x in both[:world]], [int(x) for x in both[world:]]
    else:
        send_counts = [int(id_bounds[q + 1] - id_bounds[q]) for q in range(world)]
        recv_counts = [int(x) for x in recv_per.cpu().tolist()]
    dev = lens.device
    # never a NULL buffer, also when nothing is received (the merge takes a device pointer)
    recv_ids = torch.empty(max(sum(recv_counts), 1), dtype=torch.int32, device=dev)[:sum(recv_counts)]
    dist.all_to_all_single(recv_ids, ids, output_split_sizes=recv_counts, input_split_sizes=send_counts,
                           group=group)
    return recv_lens, recv_ids


def _ptr(p) -> int:
    return C.cast(p, C.c_void_p).value or 0


def _own_stream(ctx):
    """A torch stream the library is switched to (emqx_gm_set_stream): the
    library's kernels, torch's tensor ops and the collectives then share one
    ordered stream.  torch's DEFAULT stream cannot serve: its handle is NULL,
    which the library reads as "keep your own (non-blocking) stream", and
    nothing would order the two.

    torch's device runtime must have come up before the library's (DESIGN.md
    §7): emqx_amd.Context initialises it first whenever torch is importable; a
    process that made its HIP context some other way first gets this error
    instead of torch's bare "No HIP GPUs are available"."""
    import torch
    try:
        s = torch.cuda.Stream(device=torch.device("cuda", ctx.device))
    except RuntimeError as e:
        raise RuntimeError(
            "emqx_amd: torch cannot see the device because the HIP runtime was initialised before torch's; "
            "create torch's device state first (emqx_amd.Context does when torch is importable, or call "
            "torch.cuda.init() before any library call)") from e
    ctx.set_stream(s.cuda_stream)
    return s


class _on:
    """``with torch.cuda.stream(s)`` for a stream that may be None (host path),
    ordered against the caller's stream both ways: the matcher's stream first
    waits for the work the caller queued (e.g. the torch ops that wrote its
    input topics), and on exit the caller's stream waits for the matcher's (so
    its consumers of the returned rows run after the kernels that wrote them)."""

    def __init__(self, stream):
        self.stream, self.cm, self.caller = stream, None, None

    def __enter__(self):
        if self.stream is not None:
            import torch
            self.caller = torch.cuda.current_stream(self.stream.device)
            self.stream.wait_stream(self.caller)
            self.cm = torch.cuda.stream(self.stream)
            self.cm.__enter__()

    def __exit__(self, *a):
        if self.cm is not None:
            self.cm.__exit__(*a)
            self.caller.wait_stream(self.stream)


class ShardedMatcher:
    """match_routes over a filter set sharded across ranks (one process per GPU).

    ``device_tensors`` True exchanges device buffers (RCCL, backend "nccl");
    False stages them through host memory (backend "gloo", e.g. several ranks
    sharing one device in tests).  On the device path the library and torch
    run on the matcher's own stream (emqx_gm_set_stream), so its kernels,
    torch's tensor ops and the collectives are ordered by one stream: no
    cross-stream race, no device-wide synchronisation between the steps.
    """

    def __init__(self, ctx: Context, index: Index, world: int, rank: int, dist=None, group=None,
                 device_tensors: bool = True):
        self.ctx, self.index, self.world, self.rank = ctx, index, world, rank
        self.dist, self.group, self.device_tensors = dist, group, device_tensors
        self.last_exchange_bytes = 0
        self.stream = _own_stream(ctx) if device_tensors else None

    def match_device(self, d_tb: int, d_to: int, n: int, exact: bool = True) -> Tuple[DeviceCsr, int, int]:
        """Rows of this rank's topic slice; returns (csr, first_row, n_rows)."""
        with _on(self.stream):
            return self._match_device(d_tb, d_to, n, exact)

    def _match_device(self, d_tb: int, d_to: int, n: int, exact: bool) -> Tuple[DeviceCsr, int, int]:
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
            bounds = None  # (the exchange derives the send and receive counts from the lengths: one D2H)
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


# ---------------------------------------------------------------------------
# Prefix sharding (gm_route.hip): every topic needs exactly one shard
# ---------------------------------------------------------------------------
def plan_prefix_shard(fb: np.ndarray, fo: np.ndarray, world: int, rank: int):
    """This rank's filters under prefix sharding (its first-word partitions plus
    the filters every shard holds), their global ids, the global filter count
    and the route (emqx_gm_prefix_plan)."""
    from .engine import ALL_SHARDS, prefix_plan
    gids, n_unique = filter_ranks(fb, fo)
    sh, route = prefix_plan(fb, fo, world)
    mine = (sh == rank) | (sh == ALL_SHARDS)
    sfb, sfo = select_filters(fb, fo, np.where(mine, 0, 1).astype(np.uint32), 0)
    return sfb, sfo, gids[mine], n_unique, route


class PrefixShardedMatcher:
    """match_routes over a prefix-sharded filter set (one process per GPU).

    Each rank holds its own publish batch.  A step routes every topic to the
    one shard holding all the filters it can match (emqx_gm_route_topics),
    sends the topics there (all-to-all-v of the topic bytes and lengths; RCCL
    over xGMI on the device path), each rank walks only the topics it received
    -- ~1/N of the job, against its shard -- and the rows go back to the
    topics' ranks (all-to-all-v of row lengths and ids), where
    emqx_gm_unpermute_rows puts them in batch order.  Per rank and step the
    exchange moves the batch's topic bytes + 4 B per topic out, and 4 B per
    topic + 4 B per match back; nothing is merged (each row comes from one
    shard whole).

    ``device_tensors`` False runs the same exchange on host tensors (gloo),
    with ``match_fn(tb, to) -> (row_off, ids)`` standing in for the device
    match (tests: the oracle over the rank's shard)."""

    def __init__(self, ctx: Optional[Context], index: Optional[Index], route, world: int, rank: int, dist=None,
                 group=None, device_tensors: bool = True, match_fn=None, chunks: int = 2):
        """``chunks`` (device path, world > 1; the same on every rank): the step
        runs as that many contiguous chunks of the batch, each chunk's outbound
        exchange issued asynchronously before the previous chunk's walk, so the
        all-to-all of chunk k+1 crosses xGMI while chunk k walks, and chunk k's
        return exchange while chunk k+1 walks (1: the unchunked step)."""
        self.ctx, self.index, self.route, self.world, self.rank = ctx, index, route, world, rank
        self.dist, self.group, self.device_tensors, self.match_fn = dist, group, device_tensors, match_fn
        self.chunks = max(1, int(chunks))
        self.last_exchange_bytes = 0
        self.last_topics_walked = 0
        # also at world 1: torch's sort / bincount read what the library's kernels write
        self.stream = _own_stream(ctx) if device_tensors and ctx is not None else None

    def _a2a(self, out, inp, out_splits=None, in_splits=None):
        if self.world == 1:
            out.copy_(inp)
            return
        self.dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits,
                                    group=self.group)

    def match_host(self, tb: np.ndarray, to: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """The exchange on host tensors (gloo): rows of this rank's batch, in order."""
        import torch
        W = self.world
        n = len(to) - 1
        dest = self.route.route_host(tb, to).astype(np.int64)
        perm = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=W).astype(np.int64)
        lens = np.diff(to.astype(np.int64))[perm]
        pb = np.concatenate([tb[int(to[i]):int(to[i + 1])] for i in perm]) if n else np.zeros(0, np.uint8)
        cum = np.r_[0, np.cumsum(lens)]
        bnd = np.r_[0, np.cumsum(counts)]
        bsplit = [int(x) for x in cum[bnd[1:]] - cum[bnd[:-1]]]
        sizes = torch.tensor(np.stack([counts, np.array(bsplit, np.int64)], 1).reshape(-1))
        rsizes = torch.empty_like(sizes)
        self._a2a(rsizes, sizes)
        rc = rsizes.view(W, 2)[:, 0].tolist()
        rb = rsizes.view(W, 2)[:, 1].tolist()
        rbytes = torch.empty(sum(rb), dtype=torch.uint8)
        self._a2a(rbytes, torch.from_numpy(pb.copy()), rb, bsplit)
        rlens = torch.empty(sum(rc), dtype=torch.int64)
        self._a2a(rlens, torch.from_numpy(lens.copy()), rc, [int(c) for c in counts])
        roff = np.zeros(sum(rc) + 1, np.uint64)
        roff[1:] = np.cumsum(rlens.numpy())
        rtb = np.concatenate([rbytes.numpy(), np.zeros(64, np.uint8)])
        ro, ids = self.match_fn(rtb, roff)
        self.last_topics_walked = sum(rc)
        rowlen = np.diff(ro.astype(np.int64))
        # back to the topics' ranks: lengths (per source: the topics it sent) and ids
        rbnd = np.r_[0, np.cumsum(rc)].astype(np.int64)
        idsplit = [int(rowlen[a:b].sum()) for a, b in zip(rbnd[:-1], rbnd[1:])]
        bsz = torch.tensor(idsplit, dtype=torch.int64)
        rbsz = torch.empty_like(bsz)
        self._a2a(rbsz, bsz)
        back_lens = torch.empty(n, dtype=torch.int64)
        self._a2a(back_lens, torch.from_numpy(rowlen), [int(c) for c in counts], rc)
        back_ids = torch.empty(int(rbsz.sum()), dtype=torch.int32)
        self._a2a(back_ids, torch.from_numpy(ids.astype(np.int32)), rbsz.tolist(), idsplit)
        self.last_exchange_bytes = int(len(pb) + 8 * n + 8 * sum(rc) + 4 * int(ro[-1]))
        # unpermute: row perm[k] <- received row k
        bl = back_lens.numpy()
        out_len = np.zeros(n, np.int64)
        out_len[perm] = bl
        out_off = np.zeros(n + 1, np.uint64)
        out_off[1:] = np.cumsum(out_len)
        in_off = np.r_[0, np.cumsum(bl)]
        out_ids = np.zeros(int(out_off[-1]), np.uint32)
        bi = back_ids.numpy().view(np.uint32)
        for k in range(n):
            o = int(out_off[perm[k]])
            out_ids[o:o + int(bl[k])] = bi[in_off[k]:in_off[k + 1]]
        return out_off, out_ids

    def match_device(self, d_tb: int, d_to: int, n: int, exact: bool = True) -> DeviceCsr:
        """The exchange on device tensors: rows of this rank's batch (device
        topics d_tb / d_to, n of them), in batch order, as a DeviceCsr.

        Host round trips per step: ONE device-to-host copy of the outbound
        split sizes (topics and bytes per peer, both directions: the byte total
        is their sum), the match's own read-back (its match total), the
        synchronous device copy of the result ids into the collective's torch
        buffer, and ONE copy of the return split sizes (ids per peer, both
        directions).  The
        library and torch's ops run on the matcher's own stream (set in
        __init__), so route, sort, permute, the collectives and the walk are
        ordered by one stream."""
        with _on(self.stream):
            return self._match_device(d_tb, d_to, n, exact)

    def _xchg(self, inp, out_len=None, out_splits=None, in_splits=None):
        """all_to_all_single into a new tensor of out_len elements (default:
        inp's); at world 1 the input itself -- no self-copy (the
        world-1 step spent 3.1 ms copying buffers to themselves)."""
        if self.world == 1:
            return inp
        import torch
        out = torch.empty(inp.numel() if out_len is None else out_len, dtype=inp.dtype, device=inp.device)
        self.dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits,
                                    group=self.group)
        return out

    def _match_device(self, d_tb: int, d_to: int, n: int, exact: bool) -> DeviceCsr:
        import torch
        ctx, W = self.ctx, self.world
        if W > 1 and self.chunks > 1:
            return self._match_device_chunked(d_tb, d_to, n, exact)
        dev = torch.device("cuda", ctx.device)
        # the send order (emqx_gm_route_partition: a counting sort of the batch by
        # shard, stable in batch order) with the topics' lengths in that order and
        # the topics / bytes per peer -- no per-topic atomics into W bins (index_add_
        # over 10^8 topics serialised on W addresses: ~80 ms of a 120-ms step) and
        # no radix sort of the shard numbers
        perm = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
        plen = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
        sizes = torch.empty(2 * W, dtype=torch.int64, device=dev)
        ctx.route_partition(self.route, d_tb, d_to, n, perm.data_ptr(), plen.data_ptr(), sizes.data_ptr())
        rsizes = self._xchg(sizes)
        both = torch.cat([sizes, rsizes]).cpu().tolist()  # D2H 1: the outbound split sizes
        cs, bs = both[0:2 * W:2], both[1:2 * W:2]
        rc, rb = both[2 * W::2], both[2 * W + 1::2]
        tot, m = sum(bs), sum(rc)
        if W == 1:
            # one shard: the stable send order is the batch order (perm = identity), so the
            # permuted batch IS the batch and the rows come back in order -- both copies alias
            res = ctx.match_device(self.index, d_tb, d_to, n, exact)
            self.last_topics_walked = n
            self.last_exchange_bytes = 0
            return res
        pbytes = torch.empty(tot + 64, dtype=torch.uint8, device=dev)
        poff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        ctx.permute_topics(d_tb, d_to, n, perm.data_ptr(), pbytes.data_ptr(), poff.data_ptr())
        rbytes = torch.empty(sum(rb) + 64, dtype=torch.uint8, device=dev)
        self.dist.all_to_all_single(rbytes[:sum(rb)], pbytes[:tot], output_split_sizes=rb, input_split_sizes=bs,
                                    group=self.group)
        rbytes[sum(rb):].zero_()
        rlens = self._xchg(plen, m, rc, cs)
        roff = torch.zeros(m + 1, dtype=torch.int64, device=dev)
        roff[1:] = rlens.to(torch.int64).cumsum(0)
        res = ctx.match_device(self.index, rbytes.data_ptr(), roff.data_ptr(), m, exact)  # read-back: nnz
        self.last_topics_walked = m
        nnz = res.nnz
        rowlen = torch.empty(max(m, 1), dtype=torch.int32, device=dev)[:m]
        ctx.csr_row_lengths(res, rowlen.data_ptr())
        ids = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
        ctx.memcpy_d2d(ids.data_ptr(), _ptr(res.csr.ids), nnz * 4)
        res.free()
        # ids per peer: the rows' prefix sums at the received runs' boundaries
        rbnd = torch.tensor(np.r_[0, np.cumsum(rc)].astype(np.int64), device=dev)
        rcum = torch.zeros(m + 1, dtype=torch.int64, device=dev)
        torch.cumsum(rowlen, 0, out=rcum[1:])
        idsplit_t = rcum[rbnd[1:]] - rcum[rbnd[:-1]]
        rbsz = self._xchg(idsplit_t)
        both = torch.cat([idsplit_t, rbsz]).cpu().tolist()  # D2H 2: the return split sizes
        idsplit, backsplit = both[:W], both[W:]
        back_lens = self._xchg(rowlen, n, cs, rc)
        back_ids = torch.empty(max(sum(backsplit), 1), dtype=torch.int32, device=dev)
        self.dist.all_to_all_single(back_ids[:sum(backsplit)], ids, output_split_sizes=backsplit,
                                    input_split_sizes=idsplit, group=self.group)
        self.last_exchange_bytes = tot + 4 * n + 4 * m + 4 * nnz
        return ctx.unpermute_rows(n, perm.data_ptr(), back_lens.data_ptr(), back_ids.untyped_storage().data_ptr())

    def _match_device_chunked(self, d_tb: int, d_to: int, n: int, exact: bool) -> DeviceCsr:
        """The step in self.chunks contiguous chunks of the batch (world > 1).
        Every rank issues the same collectives in the same order: the split
        sizes of all chunks in one exchange; then, per chunk, its topic bytes
        and lengths (asynchronous); then per chunk, walk -> return split sizes
        -> row lengths and ids (asynchronous).  So chunk k+1's outbound
        all-to-all runs on the collective's stream while chunk k walks on the
        matcher's, and chunk k's return exchange while chunk k+1 walks.  The
        rows of all chunks are un-permuted in one pass at the end (received row
        j of chunk c is topic start_c + perm_c[j])."""
        import torch
        ctx, W, K = self.ctx, self.world, self.chunks
        dev = torch.device("cuda", ctx.device)
        bounds = [n * c // K for c in range(K + 1)]
        ch = []
        sizes_all = torch.empty((K, 2 * W), dtype=torch.int64, device=dev)
        for c in range(K):
            s0, m = bounds[c], bounds[c + 1] - bounds[c]
            perm = torch.empty(max(m, 1), dtype=torch.int32, device=dev)[:m]
            plen = torch.empty(max(m, 1), dtype=torch.int32, device=dev)[:m]
            # a chunk's topics: the offsets array from topic s0 on (offsets are absolute in d_tb)
            if m:
                ctx.route_partition(self.route, d_tb, d_to + 8 * s0, m, perm.data_ptr(), plen.data_ptr(),
                                    sizes_all[c].data_ptr())
            else:
                sizes_all[c].zero_()
            ch.append({"s": s0, "m": m, "perm": perm, "plen": plen})
        send = sizes_all.view(K, W, 2).permute(1, 0, 2).contiguous().view(-1)  # [peer][chunk][count, bytes]
        recv = self._xchg(send)
        sz = torch.cat([send, recv]).cpu().view(2, W, K, 2).tolist()  # D2H 1: every chunk's split sizes
        for c, C in enumerate(ch):
            C["cs"] = [sz[0][p][c][0] for p in range(W)]
            C["bs"] = [sz[0][p][c][1] for p in range(W)]
            C["rc"] = [sz[1][p][c][0] for p in range(W)]
            C["rb"] = [sz[1][p][c][1] for p in range(W)]
        # outbound: every chunk's permute and its two exchanges, issued now (asynchronous)
        for C in ch:
            tot, rbt, mr = sum(C["bs"]), sum(C["rb"]), sum(C["rc"])
            pbytes = torch.empty(tot + 64, dtype=torch.uint8, device=dev)
            poff = torch.empty(C["m"] + 1, dtype=torch.int64, device=dev)
            if C["m"]:
                ctx.permute_topics(d_tb, d_to + 8 * C["s"], C["m"], C["perm"].data_ptr(), pbytes.data_ptr(),
                                   poff.data_ptr())
            rbytes = torch.empty(rbt + 64, dtype=torch.uint8, device=dev)
            rbytes[rbt:].zero_()
            rlens = torch.empty(mr, dtype=torch.int32, device=dev)
            C["w_in"] = [self.dist.all_to_all_single(rbytes[:rbt], pbytes[:tot], output_split_sizes=C["rb"],
                                                     input_split_sizes=C["bs"], group=self.group, async_op=True),
                         self.dist.all_to_all_single(rlens, C["plen"], output_split_sizes=C["rc"],
                                                     input_split_sizes=C["cs"], group=self.group, async_op=True)]
            C.update(pbytes=pbytes, poff=poff, rbytes=rbytes, rlens=rlens, mr=mr)
        walked = 0
        xbytes = 0
        for C in ch:
            for w in C.pop("w_in"):
                w.wait()  # (the matcher's stream waits for the chunk's inbound exchange)
            mr = C["mr"]
            roff = torch.zeros(mr + 1, dtype=torch.int64, device=dev)
            roff[1:] = C["rlens"].to(torch.int64).cumsum(0)
            res = ctx.match_device(self.index, C["rbytes"].data_ptr(), roff.data_ptr(), mr, exact)  # read-back: nnz
            walked += mr
            nnz = res.nnz
            rowlen = torch.empty(max(mr, 1), dtype=torch.int32, device=dev)[:mr]
            ctx.csr_row_lengths(res, rowlen.data_ptr())
            ids = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
            ctx.memcpy_d2d(ids.data_ptr(), _ptr(res.csr.ids), nnz * 4)
            res.free()
            rbnd = torch.tensor(np.r_[0, np.cumsum(C["rc"])].astype(np.int64), device=dev)
            rcum = torch.zeros(mr + 1, dtype=torch.int64, device=dev)
            torch.cumsum(rowlen, 0, out=rcum[1:])
            idsplit_t = rcum[rbnd[1:]] - rcum[rbnd[:-1]]
            rbsz = self._xchg(idsplit_t)
            b2 = torch.cat([idsplit_t, rbsz]).cpu().tolist()  # D2H: the chunk's return split sizes
            idsplit, backsplit = b2[:W], b2[W:]
            back_lens = torch.empty(C["m"], dtype=torch.int32, device=dev)
            back_ids = torch.empty(max(sum(backsplit), 1), dtype=torch.int32, device=dev)
            C["w_out"] = [self.dist.all_to_all_single(back_lens, rowlen, output_split_sizes=C["cs"],
                                                      input_split_sizes=C["rc"], group=self.group, async_op=True),
                          self.dist.all_to_all_single(back_ids[:sum(backsplit)], ids, output_split_sizes=backsplit,
                                                      input_split_sizes=idsplit, group=self.group, async_op=True)]
            C.update(rowlen=rowlen, ids=ids, back_lens=back_lens, back_ids=back_ids[:sum(backsplit)])
            xbytes += sum(C["bs"]) + 4 * C["m"] + 4 * mr + 4 * nnz
        for C in ch:
            for w in C.pop("w_out"):
                w.wait()
        self.last_topics_walked = walked
        self.last_exchange_bytes = xbytes
        perm_all = torch.cat([C["perm"] + C["s"] for C in ch]).to(torch.int32)
        lens_all = torch.cat([C["back_lens"] for C in ch])
        ids_all = torch.cat([C["back_ids"] for C in ch] + [torch.zeros(1, dtype=torch.int32, device=dev)])
        # (the buffers go back to torch's cache on this stream: later users queue behind the un-permute)
        return ctx.unpermute_rows(n, perm_all.data_ptr(), lens_all.data_ptr(), ids_all.data_ptr())
