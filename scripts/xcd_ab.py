"""XCD-locality A/B (DESIGN §9 "Next" 3): does a batch whose tiles are dealt to
the 8 XCDs by a topic word class walk faster?  Blocks b and b + 8 share an XCD
(MI355X_MICROARCH.md, workgroup dispatch), so a batch laid out as
  tile b <- 256 topics of class (b % 8)
gives each XCD's L2 only the subtrees of one class.  Variants (same topics,
reordered on the device with emqx_gm_permute_topics):
  base     the generated order
  w0_xcd   class = level-0 word % 8, tile b <- class b % 8
  w1_xcd   class = level-1 word % 8, tile b <- class b % 8
  w0_ctrl  class = level-0 word % 8, tile b <- class (b // 8) % 8 (same tiles, every
           XCD sees every class: separates XCD locality from in-tile locality)
  w0_seg8  stable sort by level-0 word % 8: 8 contiguous segments, no XCD mapping (all
           XCDs walk one class at a time)
  w0_seg   stable sort by level-0 word: 64 contiguous segments
  sorted   sorted by (w0, w1): the locality bound
Prints the main pass's kernel time per variant (several rounds, interleaved).

usage: xcd_ab.py [--config c2|c3] [--topics N] [--rounds R] [--index-cache PATH]
"""

import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def words01(tb: torch.Tensor, off: torch.Tensor):
    """Level-0 and level-1 word numbers of topics 'l0wA/l1wB/...'."""
    n = off.numel() - 1
    o = off[:n]
    idx = o.unsqueeze(1) + torch.arange(16, device=tb.device)
    r = tb[idx].to(torch.int64)  # (n, 16)
    dig = lambda c: (c >= 48) & (c <= 57)  # noqa: E731
    two = dig(r[:, 4])
    w0 = torch.where(two, (r[:, 3] - 48) * 10 + (r[:, 4] - 48), r[:, 3] - 48)
    s = torch.where(two, 5, 4) + 4  # first digit of the level-1 word
    w1 = torch.zeros(n, dtype=torch.int64, device=tb.device)
    alive = torch.ones(n, dtype=torch.bool, device=tb.device)
    for k in range(4):
        c = r.gather(1, (s + k).unsqueeze(1)).squeeze(1)
        alive &= dig(c)
        w1 = torch.where(alive, w1 * 10 + (c - 48), w1)
    return w0, w1


def xcd_perm(cls: torch.Tensor, ctrl: bool = False) -> torch.Tensor:
    """perm[i] = the topic at position i: tile b gets 256 topics of class b % 8
    (ctrl: (b // 8) % 8); what does not fill whole rounds goes last."""
    n = cls.numel()
    order = torch.sort(cls, stable=True).indices
    counts = torch.bincount(cls, minlength=8)
    start = torch.cumsum(counts, 0) - counts
    sc = cls[order]
    k = torch.arange(n, device=cls.device) - start[sc]  # rank within its class
    R = int((counts // 256).min().item())
    if ctrl:
        R = R // 8 * 8  # whole 64-tile blocks
    tile_r, within = k // 256, k % 256
    full = tile_r < R
    if ctrl:  # round r, slot c -> tile index r*8 + c with the class sequence transposed per 64 tiles
        q = tile_r * 8 + sc
        blk = q // 64
        in_blk = q % 64
        q = blk * 64 + (in_blk % 8) * 8 + in_blk // 8
        pos = q * 256 + within
    else:
        pos = (tile_r * 8 + sc) * 256 + within
    m = R * 8 * 256
    rest = ~full
    pos = torch.where(full, pos, torch.zeros_like(pos))
    pos[rest] = m + torch.arange(int(rest.sum().item()), device=cls.device)
    perm = torch.empty(n, dtype=torch.int64, device=cls.device)
    perm[pos] = order
    return perm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--topics", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--index-cache", default=None)
    ap.add_argument("--variants", default="base,w0_xcd,w1_xcd,w0_ctrl,sorted")
    a = ap.parse_args()
    torch.zeros(1, device="cuda:0")
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    n_f = {"c2": 1_000_000, "c3": 10_000_000}[a.config]
    ctx = Context(0)
    codes = gen_filter_codes(a.seed, n_f, wildcard_only=a.config == "c2")
    t = time.time()
    if a.index_cache and os.path.exists(a.index_cache):
        import numpy as np
        idx = ctx.import_index(np.fromfile(a.index_cache, np.uint8))
    else:
        idx = ctx.build_index(render_codes(codes))
        if a.index_cache:
            idx.export().tofile(a.index_cache)
    print(f"index {a.config}: {idx.n_filters} filters, {idx.info.device_bytes / 1e6:.0f} MB, {time.time() - t:.1f} s",
          flush=True)
    n = a.topics
    db, do, tot = ctx.gen_topics_device(codes, a.seed, 0, n)
    dev = torch.device("cuda", 0)
    # views of the library's buffers (synchronous: gen_topics_device returned after its sync)
    tb = torch.empty(tot + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.memcpy_d2d(tb.data_ptr(), db, tot + 64)
    ctx.memcpy_d2d(off.data_ptr(), do, 8 * (n + 1))
    w0, w1 = [], []
    for s in range(0, n, 10_000_000):
        e = min(n, s + 10_000_000)
        a0, a1 = words01(tb, off[s:e + 1])
        w0.append(a0)
        w1.append(a1)
    w0, w1 = torch.cat(w0), torch.cat(w1)
    print("w0 range", int(w0.min()), int(w0.max()), "w1 range", int(w1.min()), int(w1.max()), flush=True)
    perms = {}
    vs = a.variants.split(",")
    if "w0_xcd" in vs:
        perms["w0_xcd"] = xcd_perm(w0 % 8)
    if "w1_xcd" in vs:
        perms["w1_xcd"] = xcd_perm(w1 % 8)
    if "w0_ctrl" in vs:
        perms["w0_ctrl"] = xcd_perm(w0 % 8, ctrl=True)
    if "w0_seg8" in vs:
        perms["w0_seg8"] = torch.sort(w0 % 8, stable=True).indices
    if "w0_seg" in vs:
        perms["w0_seg"] = torch.sort(w0, stable=True).indices
    if "sorted" in vs:
        perms["sorted"] = torch.sort(w0 * 4096 + w1, stable=True).indices
    batches = {"base": (tb, off)} if "base" in vs else {}
    del w0, w1
    for name, p in perms.items():
        p32 = p.to(torch.int32)
        assert torch.equal(torch.sort(p).values, torch.arange(n, device=dev)), name
        pb = torch.empty(tot + 64, dtype=torch.uint8, device=dev)
        po = torch.empty(n + 1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        ctx.permute_topics(tb.data_ptr(), off.data_ptr(), n, p32.data_ptr(), pb.data_ptr(), po.data_ptr())
        ctx.synchronize()
        pb[tot:].zero_()
        batches[name] = (pb, po)
        del p32
    perms.clear()
    torch.cuda.synchronize()
    nnz = {}
    res_ms = {k: [] for k in batches}
    for r in range(a.rounds):
        for name, (b, o) in batches.items():
            ks = []
            for _ in range(a.reps):
                res = ctx.match_device(idx, b.data_ptr(), o.data_ptr(), n, exact=True)
                ks.append(ctx.last_kernel_ms())
                nnz.setdefault(name, res.nnz)
                assert res.nnz == nnz[name]
                res.free()
            res_ms[name].append(min(ks))
            print(f"round {r} {name:8s} kernel {min(ks):.3f} ms (reps {', '.join(f'{k:.3f}' for k in ks)}) "
                  f"nnz {nnz[name]}", flush=True)
    assert len(set(nnz.values())) == 1, nnz
    for name, v in res_ms.items():
        print(f"{a.config} {name:8s} best {min(v):.3f} ms  median {sorted(v)[len(v) // 2]:.3f} ms", flush=True)
    ctx.dev_free(db)
    ctx.dev_free(do)
    idx.release()
    ctx.close()


if __name__ == "__main__":
    main()
