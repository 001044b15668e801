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
        # the same exchange with the counts derived from the lengths (the device path: one D2H)
        rl2, ri2 = exchange_rows(dist, lens, torch.from_numpy(gl), None, world)
        assert torch.equal(rl, rl2) and torch.equal(ri, ri2)
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


# ---------------------------------------------------------------------------
# prefix sharding (gm_route.hip): every filter a topic can match is on the
# topic's one shard; the topic-routing exchange over gloo
# ---------------------------------------------------------------------------
def _skewed_set(seed, n_f=400, n_t=500):
    """Mixed filters with one HOT first word (about half the set), so the plan
    splits it by its second word; plus its 'w', 'w/#', 'w/+/..' filters, root
    wildcards and $SYS."""
    from tests.test_gpu_parity import _rand_filter, _rand_topic
    rng = random.Random(seed)
    filters = [_rand_filter(rng).encode() for _ in range(n_f // 2)]
    hot = [b"hot/" + _rand_filter(rng).encode() for _ in range(n_f // 2)]
    filters += hot + [b"hot", b"hot/#", b"hot/+", b"hot/+/x", b"#", b"+/+", b"+", b"$SYS/#", b"", b"/"]
    topics = [_rand_topic(rng).encode() for _ in range(n_t // 2)]
    topics += [b"hot/" + _rand_topic(rng).encode() for _ in range(n_t // 2)]
    topics += [b"hot", b"hot/", b"hot/x", b"/", b"", b"$SYS/a", b"+/x", b"hot/+"]
    return filters, topics


@pytest.mark.parametrize("skew", [False, True], ids=["uniform", "hot_word_split"])
def test_prefix_plan_every_match_on_the_topics_shard(skew, orc):
    """For every topic and every filter emqx_topic:match/2 pairs it with
    (oracle brute force, match_routes semantics: the literal route too), the
    filter is on the topic's routed shard or on every shard."""
    from emqx_amd.engine import ALL_SHARDS, pack, prefix_plan
    filters, topics = _skewed_set(5) if skew else _rand_set(5)
    fb, fo = pack(filters)
    uniq = sorted(set(filters))
    fro, fids = orc.bruteforce(topics, uniq, mode=1)
    tb, to = pack(topics)
    for world in (1, 2, 3, 8):
        sh, route = prefix_plan(fb, fo, world)
        shard_of_f = {}
        for f, s in zip(filters, sh):
            assert shard_of_f.setdefault(f, int(s)) == int(s)  # equal filters, one shard
            assert s == ALL_SHARDS or s < world
        dest = route.route_host(tb, to)
        assert (dest < world).all()
        for t in range(len(topics)):
            for i in fids[fro[t]:fro[t + 1]]:
                s = shard_of_f[uniq[i]]
                assert s == ALL_SHARDS or s == dest[t], (world, topics[t], uniq[i], s, int(dest[t]))
        if skew and world > 1:  # the hot word is split: its filters spread over shards
            hot_sh = {shard_of_f[f] for f in filters if f.startswith(b"hot/") and f not in
                      (b"hot/#", b"hot/+", b"hot/+/x")}
            assert len(hot_sh) > 1
            assert shard_of_f[b"hot/#"] == shard_of_f[b"hot"] == shard_of_f[b"hot/+/x"] == ALL_SHARDS
        route.release()


def _prefix_worker(rank, world, port, seed, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from emqx_amd.engine import pack
    from emqx_amd.sharded import PrefixShardedMatcher, plan_prefix_shard
    from oracle import oracle as orc
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        filters, topics = _skewed_set(seed)
        fb, fo = pack(filters)
        sfb, sfo, gids, _, route = plan_prefix_shard(fb, fo, world, rank)
        part = [bytes(sfb[int(sfo[i]):int(sfo[i + 1])]) for i in range(len(sfo) - 1)]
        local = sorted(set(part))
        gid_of = {f: int(g) for f, g in zip(part, gids)}

        def match_fn(rtb, roff):  # this rank's shard, global ids (the device match in production)
            mine = orc.unpack(rtb, roff)
            if not local:
                return np.zeros(len(mine) + 1, np.uint64), np.zeros(0, np.uint32)
            ro, ids = orc.bruteforce(mine, local, mode=1)
            return ro, np.array([gid_of[local[i]] for i in ids], np.uint32)

        # each rank publishes its own batch: a different slice of the topics
        mine = topics[rank::world]
        m = PrefixShardedMatcher(None, None, route, world, rank, dist=dist, device_tensors=False, match_fn=match_fn)
        tb, to = pack(mine)
        ro, ids = m.match_host(tb, to)
        uniq = sorted(set(filters))
        fro, fids = orc.bruteforce(mine, uniq, mode=1)
        assert np.array_equal(ro, fro) and np.array_equal(ids, fids)
        open(os.path.join(out_dir, f"ok{rank}"), "w").write(f"{len(mine)} {m.last_topics_walked}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 3])
def test_prefix_exchange_gloo(world, tmp_path, orc):
    """The topic-routing exchange of PrefixShardedMatcher over gloo, world 2
    and 3: every rank's rows (its own batch, in order) equal the unsharded
    oracle's; each rank walked only the topics routed to it."""
    import torch.multiprocessing as mp
    mp.spawn(_prefix_worker, args=(world, _free_port(), 11 + world, str(tmp_path)), nprocs=world, join=True)
    assert sorted(os.listdir(tmp_path)) == [f"ok{r}" for r in range(world)]
    walked = [int(open(os.path.join(tmp_path, f"ok{r}")).read().split()[1]) for r in range(world)]
    sent = [int(open(os.path.join(tmp_path, f"ok{r}")).read().split()[0]) for r in range(world)]
    assert sum(walked) == sum(sent)  # every topic walked exactly once, on one rank
