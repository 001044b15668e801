"""Index images (emqx_gm_index_export / _device_blob / _import) and the lazy
host mirror (EMQX_GM_OPEN_MIRROR_*): one snapshot compiled once and replicated
-- the reference replicates ONE routing table to every node through mria
(apps/emqx/src/emqx_router.erl:75-84, 136) rather than recomputing it.

Bar: an imported snapshot matches (rows, fan-out, filter names) bit-exactly
like the exported one; its in-place update line goes on (the host mirror is
downloaded on the first update) and gives what the same update of the
original gives; images from another layout or truncated are refused."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from emqx_amd import Context
    c = Context(0)
    yield c
    c.close()


def _workload(n_f=20_000, n_t=50_000):
    from emqx_amd.engine import gen_filter_codes, render_codes
    from oracle import oracle as orc
    codes = gen_filter_codes(3, n_f)
    fb, fo = render_codes(codes)
    tb, to = orc.render_codes(orc.gen_topic_codes(3, 0, n_t, codes))
    return (fb, fo), (tb, to)


def _same_rows(ctx_a, ia, ctx_b, ib, topics):
    ra = ctx_a.match(ia, topics, exact=True)
    rb = ctx_b.match(ib, topics, exact=True)
    assert np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1], rb[1])
    assert int(ra[0][-1]) > len(topics[1]) // 2  # the batch matches something
    return ra


def test_export_import_roundtrip_host_image(ctx):
    from emqx_amd import Context
    fp, tp = _workload()
    idx = ctx.build_index(fp)
    img = idx.export()
    assert img.nbytes > idx.info.device_bytes
    with Context(0) as other:
        imp = other.import_index(img)
        assert imp.n_filters == idx.n_filters and imp.info.device_bytes == idx.info.device_bytes
        assert [imp.filter(i) for i in (0, 7, idx.n_filters - 1)] == [idx.filter(i) for i in (0, 7, idx.n_filters - 1)]
        _same_rows(ctx, idx, other, imp, tp)
        ro, ids = ctx.match(idx, tp, exact=False)  # emqx_trie:match/1 mode too
        ro2, ids2 = other.match(imp, tp, exact=False)
        assert np.array_equal(ro, ro2) and np.array_equal(ids, ids2)
        imp.release()
    idx.release()


def test_import_from_device_blob(ctx):
    """The RCCL form: the image without the device tables, which come from a
    device pointer (here the exported snapshot's own blob on the same GPU)."""
    fp, tp = _workload()
    idx = ctx.build_index(fp)
    img = idx.export(with_blob=False)
    ptr, nb = idx.device_blob()
    assert nb == idx.info.device_bytes and img.nbytes < nb
    imp = ctx.import_index(img, d_blob=ptr)
    _same_rows(ctx, idx, ctx, imp, tp)
    from emqx_amd import GpuMatchError
    with pytest.raises(GpuMatchError, match="EINVAL"):
        ctx.import_index(img)  # no blob in the image and none given
    imp.release()
    idx.release()


def test_import_with_subscribers_fanout(ctx):
    fp, tp = _workload(5_000, 5_000)
    from oracle import oracle as orc
    n = len(orc.unpack(*fp))
    subs = [[i % 97, 1000 + i] for i in range(n)]
    idx = ctx.build_index(fp, subs=subs)
    imp = ctx.import_index(idx.export())
    ro, ids = _same_rows(ctx, idx, ctx, imp, tp)
    fa = ctx.fanout(idx, ro, ids)
    fb = ctx.fanout(imp, ro, ids)
    assert np.array_equal(fa[0], fb[0]) and np.array_equal(fa[1], fb[1]) and int(fa[0][-1]) > 0
    assert imp.subscriber_count(3) == idx.subscriber_count(3)
    imp.release()
    idx.release()


def test_import_shard_index(ctx):
    from emqx_amd.sharded import plan_shard
    fp, tp = _workload()
    sfb, sfo, gids, _ = plan_shard(*fp, 3, 1)
    idx = ctx.build_index_shard((sfb, sfo), gids)
    imp = ctx.import_index(idx.export())
    _same_rows(ctx, idx, ctx, imp, tp)
    assert imp.filter(int(gids[5])) == idx.filter(int(gids[5]))
    imp.release()
    idx.release()


@pytest.mark.parametrize("policy", ["lazy", "eager"])
def test_update_after_import_and_lazy_mirror(policy):
    """A lazily mirrored index (and an imported one) downloads its host copy on
    the first in-place update; the result equals the same update of an eagerly
    mirrored build, and a rebuild of the updated set."""
    from emqx_amd import Context
    fp, tp = _workload()
    from oracle import oracle as orc
    fl = orc.unpack(*fp)
    ops = [(f, False) for f in fl[:300:3]] + [(b"upd/%d/+/#" % i, True) for i in range(100)] + \
          [(b"l0w1/upd/%d" % i, True) for i in range(50)]
    with Context(0, mirror=policy) as c, Context(0, mirror="eager") as ref:
        a = c.build_index(fp)
        b = ref.build_index(fp)
        imp = c.import_index(a.export())
        ua, ub, ui = c.update_index(a, ops), ref.update_index(b, ops), c.update_index(imp, ops)
        want = sorted(set(fl) - {f for f, ins in ops if not ins} | {f for f, ins in ops if ins})
        rebuilt = ref.build_index(want)
        for x, cx in ((ua, c), (ui, c)):
            _same_rows(cx, x, ref, ub, tp)
            _same_rows(cx, x, ref, rebuilt, tp)
        # a second update continues the line (the mirror moved on with the snapshot)
        ua2 = c.update_index(ua, [(b"upd/1/+/#", False)])
        ub2 = ref.update_index(ub, [(b"upd/1/+/#", False)])
        _same_rows(c, ua2, ref, ub2, tp)
        for x in (a, b, imp, ua, ub, ui, rebuilt, ua2, ub2):
            x.release()


def test_bad_images_are_refused(ctx):
    from emqx_amd import GpuMatchError
    fp, _ = _workload(2_000, 10)
    idx = ctx.build_index(fp)
    img = idx.export().copy()
    bad = img.copy()
    bad[0] ^= 0xFF
    with pytest.raises(GpuMatchError, match="EINVAL"):
        ctx.import_index(bad)
    with pytest.raises(GpuMatchError, match="EINVAL"):
        ctx.import_index(img[:1000])
    bad = img.copy()
    bad[16] ^= 0x01  # the layout signature
    with pytest.raises(GpuMatchError, match="layout"):
        ctx.import_index(bad)
    idx.release()
