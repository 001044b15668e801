"""Sharded index on the CPU: the host sharding helpers of
the C ABI, and the rank-to-rank row exchange of emqx_amd.sharded over gloo
with world_size 2 and 3.  Each rank's local rows come from the oracle over
its shard (the device match is covered by tests/test_gpu_sharded.py); the
merged slices must equal the oracle's unsharded rows."""

import os
import random
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rand_set(seed, n_f=300, n_t=400):
    from tests.test_gpu_parity import _rand_filter, _rand_topic
    rng = random.Random(seed)
    filters = [_rand_filter(rng).encode() for _ in range(n_f)]
    filters += filters[:20]  # duplicates collapse to one global id
    topics = [_rand_topic(rng).encode() for _ in range(n_t)]
    return filters, topics


def test_sharding_helpers():
    from emqx_amd.engine import filter_ranks, pack, select_filters, shard_of
    from emqx_amd.sharded import plan_shard, slice_bounds
    filters, _ = _rand_set(1)
    fb, fo = pack(filters)
    ranks, nu = filter_ranks(fb, fo)
    uniq = sorted(set(filters))
    assert nu == len(uniq)
    assert [uniq[r] for r in ranks] == filters
    for world in (1, 2, 3, 8):
        sh = shard_of(fb, fo, world)
        assert sh.max() < world
        assert np.array_equal(sh, shard_of(fb, fo, world))  # deterministic
        # equal filters land on the same shard
        seen = {}
        for f, s in zip(filters, sh):
            assert seen.setdefault(f, s) == s
        got = []
        for r in range(world):
            sfb, sfo, g, n_unique = plan_shard(fb, fo, world, r)
            part = [bytes(sfb[int(sfo[i]):int(sfo[i + 1])]) for i in range(len(sfo) - 1)]
            assert all(uniq[gid] == f for f, gid in zip(part, g))
            got += part
            assert n_unique == nu
        assert sorted(got) == sorted(filters)
    assert slice_bounds(10, 3) == (4, [0, 4, 8, 10])
    assert slice_bounds(0, 2) == (0, [0, 0, 0])


def _merge_np(rl, ri, world, S, n_rows):
    """Test-side merge of the received pieces (the product merges on the device)."""
    lens = rl.reshape(world, S)
    off = np.concatenate([[0], np.cumsum(lens.reshape(-1))])
    rows = []
    for t in range(n_rows):
        row = []
        for p in range(world):
            k = p * S + t
            row += ri[off[k]:off[k + 1]].tolist()
        rows.append(sorted(row))
    return rows


def _worker(rank, world, port, seed, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from emqx_amd.engine import pack
    from emqx_amd.sharded import exchange_rows, plan_shard, slice_bounds
    from oracle import oracle as orc
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        filters, topics = _rand_set(seed)
        fb, fo = pack(filters)
        sfb, sfo, gids, _ = plan_shard(fb, fo, world, rank)
        part = [bytes(sfb[int(sfo[i]):int(sfo[i + 1])]) for i in range(len(sfo) - 1)]
        local = sorted(set(part))
        gid_of = {f: int(g) for f, g in zip(part, gids)}
        ro, ids = orc.bruteforce(topics, local, mode=1) if local else (np.zeros(len(topics) + 1, np.uint64),
                                                                        np.zeros(0, np.uint32))
        gl = np.array([gid_of[local[i]] for i in ids], np.int32)
        n = len(topics)
        S, b = slice_bounds(n, world)
        lens = torch.zeros(world * S, dtype=torch.int32)
        lens[:n] = torch.from_numpy(np.diff(ro.astype(np.int64)).astype(np.int32))
        bounds = [int(ro[x]) for x in b]
        rl, ri = exchange_rows(dist, lens, torch.from_numpy(gl), bounds, world)
        rows = _merge_np(rl.numpy(), ri.numpy(), world, S, b[rank + 1] - b[rank])
        uniq = sorted(set(filters))
        fro, fids = orc.bruteforce(topics, uniq, mode=1)
        for k, t in enumerate(range(b[rank], b[rank + 1])):
            assert rows[k] == fids[fro[t]:fro[t + 1]].tolist(), (rank, t, topics[t])
        open(os.path.join(out_dir, f"ok{rank}"), "w").write(str(len(rows)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 3])
def test_exchange_rows_gloo(world, tmp_path, orc):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), 7 + world, str(tmp_path)), nprocs=world, join=True)
    assert sorted(os.listdir(tmp_path)) == [f"ok{r}" for r in range(world)]
