#!/usr/bin/env python3
"""Headline benchmark: publish topics matched/sec at 1M wildcard subscriptions.

Workload (BASELINE.json configs[1], SURVEY.md §8d "C2"): 1M wildcard filters
(seeded generator, exact share 0), a 100M-topic publish batch per GPU generated
on the device, matched with emqx_router:match_routes/1 semantics into a CSR of
sorted filter ids.  A step = one emqx_gm_match call over the whole batch (every
kernel, the overflow check and the CSR assembly).  Inputs are resident in HBM
before the timed region; the CSR stays in HBM (DEVICE_IO).

Multi-GPU (weak scaling): one process per GPU, replicated index, each rank
matches its own 100M-topic slice; no collective on the data path.  `value` is
the topics of all ranks / the max-over-ranks wall time.

Also reported: a roofline object for the dominant kernel (k_match_fused:
tokenizer + trie walk, algorithmic bytes per SURVEY.md §8d ÷ its HIP-event time), a CPU
baseline (the oracle's faithful emqx_trie restatement -- compact mode, ordered
key table, fresh prefix strings -- on every core of the process's affinity
mask over a bounded sample of the same topic stream) and `parity_sample`: the
last timed step's CSR, still in HBM, compared row for row with the oracle on
strided windows of the batch (outside the timed region).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "publish topics matched/sec at 1M wildcard subs (1/2/4/8 GPU); achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
RANDOM_LINE_CEILING = 52.9e9  # random 128-B line requests/s, 2 GiB table (scripts/randread.hip, profiles/r02_randread)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None,
                   help="timed steps (default 5; C1's 0.13-ms step: 200, so the timed region is not noise)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (default 2; C1: 20)")
    p.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5"])
    p.add_argument("--plan", default="replicated", choices=["replicated", "prefix", "hash"],
                   help="C5: the unsharded index replicated on every GPU with the batch partitioned (north_star: "
                        "replicate while the index fits 288 GB; 100M filters = 38 GB); filters prefix-sharded "
                        "(first word) with each topic routed to its one shard (all-to-all of topics, rows back); "
                        "or filters hash-sharded, every rank walking every topic, rows exchanged and merged")
    p.add_argument("--filters", type=int, default=None)
    p.add_argument("--topics", type=int, default=None, help="topics per GPU per step")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--cpu-threads", type=int, default=None)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-parity", action="store_true", help="skip the oracle check of the last step's sample")
    p.add_argument("--traffic-json", default=None,
                   help="PMC traffic of this build (scripts/traffic.py); default profiles/traffic.json for C2, "
                        "profiles/traffic_<config>.json for the others")
    p.add_argument("--no-update", action="store_true", help="skip the incremental-update detail")
    p.add_argument("--time-every", type=int, default=None,
                   help="time the main pass (HIP events) on every N-th call of the timed region "
                        "(default: every call; C1, whose step is ~0.1 ms: every 8th)")
    p.add_argument("--no-pipeline", action="store_true",
                   help="one call at a time (emqx_gm_match) instead of two in flight (submit / wait)")
    p.add_argument("--build-each", action="store_true",
                   help="replicated configs at N>1: every rank compiles the index itself (the default: rank 0 "
                        "compiles it once and the others import its image, the device tables broadcast over RCCL)")
    p.add_argument("--index-cache", default=None,
                   help="replicated configs: an index image file (emqx_gm_index_export); imported when it exists, "
                        "written after the build otherwise (profiling passes of C3/C5 skip the host build)")
    p.add_argument("--subs-update", action="store_true",
                   help="C5: also measure subscriber updates on a 100M-filter index with subscriber lists")
    p.add_argument("--replicas", type=int, default=2,
                   help="N=1: the multi-device context's rehearsal lists this GPU this many times (0: skip); "
                        "N>1: rank 0 opens one context over all N GPUs instead (the drop-in NIF's form)")
    p.add_argument("--multi-child", default=None, help=argparse.SUPPRESS)  # (internal: run_multi_child)
    p.add_argument("--multi-single", default=None, help=argparse.SUPPRESS)
    p.add_argument("--no-multi", action="store_true",
                   help="skip the multi-device context (one library context over the GPUs: replication, "
                        "host-buffer match spread over the devices, replicated updates)")
    p.add_argument("--no-host-io", action="store_true",
                   help="skip the host-buffer call (PCIe-inclusive rate, reported in detail, never `value`)")
    a = p.parse_args()
    a.no_pipeline = a.no_pipeline or bool(os.environ.get("GM_BENCH_NO_PIPELINE"))  # (A/B scripts set env knobs)
    if a.traffic_json is None:
        a.traffic_json = os.path.join(ROOT, "profiles", "traffic.json" if a.config == "c2" else
                                      f"traffic_{a.config}.json")
    if a.steps is None:
        a.steps = 200 if a.config == "c1" else 5
    if a.warmup is None:
        a.warmup = 20 if a.config == "c1" else 2
    return a


# Rehearsal knobs (tests/test_gpu_bench.py): GM_BENCH_BACKEND=gloo runs the
# rank plumbing over gloo and GM_BENCH_DEVICE pins every rank to one device, so
# the N>1 path of this script runs on a one-GPU box.  The driver's runs use
# neither: one rank per GPU over RCCL ("nccl").
BACKEND = os.environ.get("GM_BENCH_BACKEND", "nccl")


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "GM_BENCH_DEVICE" in os.environ:
        local = int(os.environ["GM_BENCH_DEVICE"])
    pg = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if BACKEND == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(BACKEND)
        pg = dist
        global HOST_GROUP
        # a CPU-side group: ranks waiting while rank 0 works on their GPUs (the
        # multi-device context) wait on the host, not in a collective kernel
        HOST_GROUP = dist.new_group(backend="gloo") if BACKEND == "nccl" else None
    return world, rank, local, pg


HOST_GROUP = None


def host_barrier(pg):
    if pg is not None:
        pg.barrier(group=HOST_GROUP) if HOST_GROUP is not None else pg.barrier()


def torch_first(local):
    """The device-tensor exchange paths use torch on the GPU: its device runtime
    must be initialised before the library's (DESIGN.md §7 "Process order with
    torch"; at N>1 dist_setup has done it, at N=1 this does)."""
    if BACKEND == "nccl":
        import torch
        torch.zeros(1, device=f"cuda:{local}")


def _reduce_tensor(local, x: float):
    import torch
    return torch.tensor([x], dtype=torch.float64, device=f"cuda:{local}" if BACKEND == "nccl" else "cpu")


def barrier_max(pg, local, x: float) -> float:
    if pg is None:
        return x
    t = _reduce_tensor(local, x)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def gather_floats(pg, local, world, x: float):
    """x from every rank, in rank order (an all-gather of one value each)."""
    t = _reduce_tensor(local, x)
    out = [t.clone() for _ in range(world)]
    pg.all_gather(out, t)
    return [float(v.item()) for v in out]


def barrier(pg):
    if pg is not None:
        pg.barrier()


def physical_cores() -> int:
    """Distinct (physical id, core id) pairs in /proc/cpuinfo."""
    seen, phys, core = set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                elif not line.strip() and phys is not None:
                    seen.add((phys, core))
    except OSError:
        pass
    return len(seen) or (os.cpu_count() or 1)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """The cgroup v2 CPU quota of this process (cores), or None when unlimited:
    the file of its own cgroup, else the namespace root's (a container sees its
    own cgroup as /sys/fs/cgroup)."""
    paths = ["/sys/fs/cgroup/cpu.max"]
    try:
        with open("/proc/self/cgroup") as f:
            rel = f.read().strip().split("::", 1)[-1]
        paths.insert(0, os.path.join("/sys/fs/cgroup", rel.lstrip("/"), "cpu.max"))
    except OSError:
        pass
    for p in paths:
        try:
            with open(p) as f:
                q, per = f.read().split()
            return None if q == "max" else float(q) / float(per)
        except (OSError, ValueError):
            continue
    return None


def oracle_router(filters_packed):
    """The oracle's emqx_router over the index's filters (cpu_baseline leg only)."""
    from oracle import oracle as orc
    r = orc.Router(True)
    r.add_routes(filters_packed)
    return r


def sorted_unique(fb, fo):
    """(bytes, offsets) of the unique filters in Erlang binary order, computed
    independently of the product (fixed-width byte rows: no NUL in generated filters)."""
    import numpy as np
    n = len(fo) - 1
    lens = np.diff(fo.astype(np.int64))
    width = max(1, int(lens.max()) if n else 1)
    rows = np.zeros((n, width), np.uint8)
    rid = np.repeat(np.arange(n), lens)
    col = np.arange(int(fo[-1])) - np.repeat(fo[:-1].astype(np.int64), lens)
    rows[rid, col] = fb[:int(fo[-1])]
    u = np.unique(rows.view(f"S{width}").ravel())
    ul = np.char.str_len(u).astype(np.uint64)
    off = np.zeros(len(u) + 1, np.uint64)
    off[1:] = np.cumsum(ul)
    return np.frombuffer(b"".join(u.tolist()) + b"\0" * 64, np.uint8).copy(), off


def cpu_baseline(r, codes, seed, target_s, threads):
    """The oracle's faithful emqx_trie walk (compact) + route lookup on all host cores."""
    from oracle import oracle as orc
    # calibrate on a small slice, then time a sample sized for ~target_s
    probe_n = 20_000 * threads
    tb, to = orc.render_codes(orc.gen_topic_codes(seed, 0, probe_n, codes))
    t0 = time.perf_counter()
    r.match_batch((tb, to), None, mode=1, nthreads=threads, want_ids=False)
    dt = time.perf_counter() - t0
    rate = probe_n / max(dt, 1e-6)
    n = int(min(max(rate * target_s, probe_n), 40_000_000))
    tb, to = orc.render_codes(orc.gen_topic_codes(seed, 0, n, codes))
    t0 = time.perf_counter()
    ro, _, lk = r.match_batch((tb, to), None, mode=1, nthreads=threads, want_ids=False)
    dt = time.perf_counter() - t0
    # single-thread rate on a slice of the same stream (reported beside the all-core one)
    n1 = max(1000, min(n, int(rate / threads * 3)))
    t1 = time.perf_counter()
    r.match_batch((tb, to[:n1 + 1]), None, mode=1, nthreads=1, want_ids=False)
    single = n1 / (time.perf_counter() - t1)
    quota = cpu_quota()
    phys = physical_cores()
    opt = optimized_cpu(codes, seed, max(2.0, target_s / 3), threads)
    return {"value": n / dt, "unit": "topics/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "optimized": opt,
            "cpu_quota_cores": quota, "single_thread_value": single,
            # measured value is capped by the cgroup quota when one is set; this is the
            # single-thread rate scaled to every physical core (an estimate, not a measurement)
            "linear_estimate_all_physical_cores": {"value": single * phys, "physical_cores": phys},
            "sample": f"first {n} topics of the same seeded stream (seed {seed}), emqx_trie compact walk + "
                      f"lookup_routes restated in C++ (oracle/emqx_oracle.cpp), {threads} std::threads = every "
                      f"core in this process's affinity mask (cgroup CPU quota: {quota} cores), {dt:.1f} s; "
                      f"{float(ro[-1]) / n:.3f} matches/topic; "
                      f"{float(lk.mean()) if len(lk) else 0:.1f} ordered-set lookups/topic"}


def optimized_cpu(codes, seed, target_s, threads):
    """The optimized CPU hash-NFA (oracle/cpu_nfa.cpp: flat hash tables, the same
    match_routes rows, checked against the faithful restatement by the tests) on the
    same cores: an honest CPU figure beside the faithful one."""
    from oracle import oracle as orc
    fb, fo = orc.render_codes(codes)
    t0 = time.perf_counter()
    nfa = orc.CpuNfa((fb, fo))
    build_s = time.perf_counter() - t0
    probe_n = 50_000 * threads
    tb, to = orc.render_codes(orc.gen_topic_codes(seed, 0, probe_n, codes))
    t0 = time.perf_counter()
    nfa.match_batch((tb, to), nthreads=threads, want_ids=False)
    rate = probe_n / max(time.perf_counter() - t0, 1e-6)
    n = int(min(max(rate * target_s, probe_n), 60_000_000))
    tb, to = orc.render_codes(orc.gen_topic_codes(seed, 0, n, codes))
    t0 = time.perf_counter()
    ro, _ = nfa.match_batch((tb, to), nthreads=threads, want_ids=False)
    dt = time.perf_counter() - t0
    n1 = max(1000, min(n, int(rate / threads * 2)))
    t1 = time.perf_counter()
    nfa.match_batch((tb, to[:n1 + 1]), nthreads=1, want_ids=False)
    single = n1 / (time.perf_counter() - t1)
    return {"value": n / dt, "unit": "topics/s", "cores": threads, "kind": "port-optimized",
            "single_thread_value": single, "index_build_s": build_s,
            "sample": f"first {n} topics of the same seeded stream, optimized hash-NFA (oracle/cpu_nfa.cpp: "
                      f"flat open-addressing level trie, words resolved once per topic), {threads} std::threads, "
                      f"{dt:.1f} s; {float(ro[-1]) / n:.3f} matches/topic"}


def parity_sample(ctx, r, res, codes, fpack_sorted, seed, first_topic, n_topics, threads, windows=20, width=50_000):
    """A strided sample of one step's CSR (still in HBM: a DeviceCsr; or a host
    (row_off, ids) pair) against the oracle: `windows` windows of `width`
    topics spread over the batch, the last window included."""
    import numpy as np
    from oracle import oracle as orc
    ranker = orc.Ranker(fpack_sorted)
    width = min(width, n_topics)
    starts = sorted({int(x) for x in np.linspace(0, n_topics - width, windows)})
    if isinstance(res, tuple):
        hro, hids = res

        def rows(s):
            ro = hro[s:s + width + 1].astype(np.uint64)
            return ro, hids[int(ro[0]):int(ro[-1])]
    else:
        ro_ptr = ctypes_ptr(res.csr.row_off)
        ids_ptr = ctypes_ptr(res.csr.ids)

        def rows(s):
            ro = np.zeros(width + 1, np.uint64)
            ctx.memcpy_d2h(ro, ro_ptr + 8 * s, (width + 1) * 8)
            nnz = int(ro[-1] - ro[0])
            ids = np.zeros(max(nnz, 1), np.uint32)
            if nnz:
                ctx.memcpy_d2h(ids, ids_ptr + 4 * int(ro[0]), nnz * 4)
            return ro, ids[:nnz]
    checked, ok, bad = 0, True, []
    for s in starts:
        ro, ids = rows(s)
        tb, to = orc.render_codes(orc.gen_topic_codes(seed, first_topic + s, width, codes))
        oro, oids, _ = r.match_batch((tb, to), ranker, mode=1, nthreads=threads)
        good = np.array_equal(ro - ro[0], oro) and np.array_equal(ids, oids)
        checked += width
        if not good:
            ok = False
            bad.append(s)
    return {"topics": checked, "windows": len(starts), "window_topics": width, "ok": ok,
            "mismatched_windows": bad[:8]}


def fixture_check(ctx, idx, name):
    """The committed config fixture (tests/golden/config_<name>.json: strided
    topics of the config's stream, their match_routes rows as filter strings)
    matched through the host-buffer call against this index."""
    with open(os.path.join(ROOT, "tests", "golden", f"config_{name}.json")) as f:
        fx = json.load(f)
    ro, ids = ctx.match(idx, [t.encode() for t in fx["topics"]], exact=True)
    got = [[idx.filter(int(k)).decode() for k in ids[ro[i]:ro[i + 1]]] for i in range(len(fx["topics"]))]
    bad = [i for i, (g, w) in enumerate(zip(got, fx["matches"])) if g != w]
    return {"topics": len(got), "fixture": f"tests/golden/config_{name}.json", "ok": not bad,
            "mismatched_topics": bad[:8]}


def host_peak_rss_gb() -> float:
    """This process's peak resident host memory (ru_maxrss, KiB) in GB."""
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024 / 1e9


def replicated_index(a, ctx, world, rank, local, pg, fpack):
    """The replicated configs' index ("the index is broadcast once
    at build time"; the reference replicates one routing table to every node,
    emqx_router.erl:75-84): rank 0 compiles the filter set, the other ranks
    import its image (emqx_gm_index_export / _import).  Over RCCL the host part
    of the image (filter table, layout) and the device tables are broadcast as
    device tensors -- the tables GPU to GPU over xGMI, never through the host;
    over gloo (rehearsals) the whole image goes as one host tensor.  Returns
    (index, "built" | "imported")."""
    if a.index_cache and world == 1:
        import numpy as np
        if os.path.exists(a.index_cache):
            return ctx.import_index(np.memmap(a.index_cache, np.uint8, "r")), "imported (cache)"
        idx = ctx.build_index(fpack)
        img = np.memmap(a.index_cache, np.uint8, "w+", shape=(idx.export_size(),))
        idx.export(out=img)
        img.flush()
        del img
        return idx, "built"
    if world == 1 or a.build_each:
        return ctx.build_index(fpack), "built"
    import numpy as np
    import torch
    dev = BACKEND == "nccl"
    tdev = torch.device("cuda", local) if dev else torch.device("cpu")
    idx = img = None
    sizes = torch.zeros(2, dtype=torch.int64, device=tdev)
    if rank == 0:
        idx = ctx.build_index(fpack)
        img = idx.export(with_blob=not dev)
        sizes[0], sizes[1] = img.nbytes, (idx.device_blob()[1] if dev else 0)
    pg.broadcast(sizes, 0)
    n_img, n_blob = (int(x) for x in sizes.tolist())
    timg = torch.from_numpy(img).to(tdev) if rank == 0 else torch.empty(n_img, dtype=torch.uint8, device=tdev)
    pg.broadcast(timg, 0)
    if not dev:
        out = idx if rank == 0 else ctx.import_index(timg.numpy())
        return out, "built" if rank == 0 else "imported"
    blob = torch.empty(n_blob, dtype=torch.uint8, device=tdev)
    if rank == 0:
        ptr, nb = idx.device_blob()
        ctx.memcpy_d2d(blob.data_ptr(), ptr, nb)  # (synchronous on the library's stream)
    pg.broadcast(blob, 0)
    torch.cuda.synchronize(tdev)
    if rank == 0:
        return idx, "built"
    out = ctx.import_index(timg.cpu().numpy(), d_blob=blob.data_ptr())
    del blob, timg
    torch.cuda.empty_cache()
    return out, "imported"


def replicas_agree(ctx, idx, codes, seed, pg, local, n=65_536) -> bool:
    """Every rank matches the same probe batch (the stream's first n topics) on
    its replica and the rows' digest must be the same on all ranks (min == max
    over the ranks): an imported replica answers exactly as rank 0's build."""
    import numpy as np
    db, do, _ = ctx.gen_topics_device(codes, seed, 0, n)
    r = ctx.match_device(idx, db, do, n, exact=True)
    ro, ids = r.to_host()
    r.free()
    ctx.dev_free(db)
    ctx.dev_free(do)
    h = np.uint64(1469598103934665603)
    for part in (ro.astype(np.uint64), ids.astype(np.uint64)):
        w = np.arange(1, len(part) + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        h = np.uint64((int(h) * 1099511628211 + int(np.bitwise_xor.reduce(part * w ^ (part >> np.uint64(7)))))
                      % (1 << 64))
    d = float(int(h) % (1 << 52))
    lo = -barrier_max(pg, local, -d)
    return lo == barrier_max(pg, local, d)


def ctypes_ptr(p) -> int:
    import ctypes
    return ctypes.cast(p, ctypes.c_void_p).value or 0


def heartbeat(every_s: float = 60.0):
    """A line on stderr every minute while the bench runs (the 100M-filter C5
    index alone builds for ~2.5 min in one library call)."""
    import threading
    t0 = time.perf_counter()

    def beat():
        while True:
            time.sleep(every_s)
            print(f"[bench] running, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def subs_update(ctx, fpack, n_ops=100, batches=7):
    """Subscriber maintenance at this config's filter count (emqx_broker:
    subscribe/unsubscribe, apps/emqx/src/emqx_broker.erl:147-165), outside the
    timed region: an index over the same filters built with one subscriber
    each, then batches of n_ops subscriber-only ops (a new subscriber joins a
    filter, its old one leaves: no route changes) through
    emqx_gm_index_update_subs -- the O(delta) path (gm_subs.cpp, SubTable).
    Wall time of each call (host work + the new subscriber CSR's device copy)."""
    import numpy as np
    fb, fo = fpack
    n = len(fo) - 1
    t0 = time.perf_counter()
    sidx = ctx.build_index(fpack, subs=(np.arange(n + 1, dtype=np.uint64), np.arange(n, dtype=np.uint32)))
    build_s = time.perf_counter() - t0
    rng = np.random.default_rng(3)
    ms = []
    cur = sidx
    for b in range(batches):
        ops = []
        for k, i in enumerate(rng.choice(n, n_ops // 2, replace=False).tolist()):
            f = bytes(fb[int(fo[i]):int(fo[i + 1])])
            ops += [(f, 1_000_000_000 + b * n_ops + k, "subscribe"), (f, i, "unsubscribe")]
        t0 = time.perf_counter()
        nxt = ctx.update_subs(cur, ops)
        ms.append((time.perf_counter() - t0) * 1e3)
        cur.release()
        cur = nxt
    ok = cur.n_filters == n
    cur.release()
    ms_sorted = sorted(ms[1:])  # (the first call warms the pools)
    return {"filters": n, "ops_per_batch": n_ops, "batches": batches, "ms_median": ms_sorted[len(ms_sorted) // 2],
            "ms_max": ms_sorted[-1], "ms_first": ms[0], "build_with_subscribers_s": build_s, "filters_unchanged": ok}


def link_peaks(ctx, nbytes=1 << 30):
    """This box's measured PCIe copy rates, one pinned buffer to / from this
    GPU (hipMemcpy, best of 3): the link roofline of the host-buffer path."""
    import numpy as np
    hb = ctx.host_alloc(nbytes)
    hb[:] = 1
    d = ctx.dev_alloc(nbytes)
    out = {}
    for name, fn in (("h2d", lambda: ctx.memcpy_h2d(d, hb, nbytes)), ("d2h", lambda: ctx.memcpy_d2h(hb, d, nbytes))):
        fn()
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            fn()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        out[name + "_peak_gbs"] = nbytes / best / 1e9
    ctx.dev_free(d)
    ctx.host_free(hb)
    del np
    return out


def host_io(ctx, idx, db, do, tbytes, n_topics, nnz, reps=2):
    """The host-buffer emqx_gm_match (the NIF's call, gm_host.cpp), best of
    ``reps`` after a warm-up: topics from page-locked memory (emqx_gm_host_alloc:
    what the NIF packs into, sent by DMA with no staging copy) and from plain
    pageable memory.  Against the link: the bytes that cross PCIe per topic each
    way (in: the text + a u16 length; out: the u64 row offset + 4 B per match)
    and the rates they reach beside this box's measured hipMemcpy peaks.
    Returns (detail, the page-locked batch and its offsets for later calls)."""
    import numpy as np
    d = {}
    ho = np.zeros(n_topics + 1, np.uint64)
    ctx.memcpy_d2h(ho, do, (n_topics + 1) * 8)
    pb = ctx.host_alloc(tbytes + 64)
    ctx.memcpy_d2h(pb, db, tbytes)
    pb[tbytes:] = 0

    cpu = {}

    def timed(c, ix, buf, name):
        c.match_host(ix, (buf, ho), exact=True).free()  # pinned staging, result pool and workers warm
        best, ok = None, True
        for _ in range(reps):
            c0, t0 = time.process_time(), time.perf_counter()
            h = c.match_host(ix, (buf, ho), exact=True)
            dt = time.perf_counter() - t0
            # host CPU seconds of the call (every thread of the process): the copies it makes
            cpu[name] = min(cpu.get(name, 1e9), time.process_time() - c0)
            ok = ok and h.nnz == nnz
            h.free()
            best = dt if best is None else min(best, dt)
        return best, ok

    best, ok = timed(ctx, idx, pb, "page-locked")
    d["host_io_topics_per_s"] = n_topics / best
    d["host_io_ms"] = best * 1e3
    d["host_io_input"] = "page-locked (emqx_gm_host_alloc)"
    hb = np.array(pb)  # the same bytes in pageable memory
    best_p, ok_p = timed(ctx, idx, hb, "pageable")
    del hb
    d["host_io_pageable_topics_per_s"] = n_topics / best_p
    d["host_io_nnz_matches_device"] = ok and ok_p
    d["host_io_cpu_s_per_call"] = cpu
    # the link: PCIe bytes per topic each way (gm_host.cpp: the text and a u16 length in, the
    # u64 row offsets -- DMA'd into the caller's CSR -- and the 4-B ids out) and the rates
    h2d = (tbytes + 2 * n_topics) / n_topics
    d2h = (8 * n_topics + 4 * nnz) / n_topics
    peaks = link_peaks(ctx)
    link = {"h2d_bytes_per_topic": h2d, "d2h_bytes_per_topic": d2h,
            "h2d_gbs": h2d * n_topics / best / 1e9, "d2h_gbs": d2h * n_topics / best / 1e9, **peaks}
    link["h2d_frac_of_peak"] = link["h2d_gbs"] / peaks["h2d_peak_gbs"]
    link["d2h_frac_of_peak"] = link["d2h_gbs"] / peaks["d2h_peak_gbs"]
    link["bound"] = "h2d" if link["h2d_frac_of_peak"] >= link["d2h_frac_of_peak"] else "d2h"
    link["note"] = ("the host-buffer call's ceiling is the PCIe link, not the kernel: "
                    "topics/s <= h2d_peak_gbs / h2d_bytes_per_topic")
    link["topics_per_s_link_ceiling"] = peaks["h2d_peak_gbs"] * 1e9 / h2d
    d["host_io_link"] = link
    return d, pb, ho


def update_chain(ctx, idx, n_rounds=2, n_ops=200, seed=7, own=False):
    """n_rounds in-place updates of n_ops (half deletes of present filters,
    half inserts), each on the previous result; wall time and what the library
    says each call did (emqx_gm_last_update_stats).  Returns (rounds, last).
    own: idx is released once the first update has replaced it."""
    import numpy as np
    rng = np.random.default_rng(seed)
    out, cur = [], idx
    for rnd in range(n_rounds):
        dels = [cur.filter(int(i)) for i in rng.choice(cur.n_filters, n_ops // 2, replace=False)]
        ins = [b"upd%d/%d/+/#" % (rnd, i) for i in range(n_ops // 2)]
        t0 = time.perf_counter()
        new = ctx.update_index(cur, [(f, False) for f in dels] + [(f, True) for f in ins])
        ms = (time.perf_counter() - t0) * 1e3
        out.append({"ms": ms, **{k: v for k, v in ctx.update_stats().items()
                                 if k in ("kind", "replica_mode", "replicas", "mirror_loaded", "mirror_bytes",
                                          "mirror_ms", "device_ms", "blobs_reused", "blobs_fresh")}})
        if cur is not idx or own:
            cur.release()
        cur = new
    return out, cur


def small_calls(c, ix, pb, ho, threads=8, calls=32, batch=16_384):
    """A NIF-sized workload: `threads` callers (dirty schedulers), each issuing
    `calls` host-buffer calls of `batch` topics (publish windows) from the
    page-locked batch, all at once on one context.  Topics/s over the wall time
    of the whole set (a multi-device context runs each small call whole on one
    of its GPUs, round-robin; a single-device context queues them on one)."""
    import threading
    n = len(ho) - 1
    errs = []

    def run(t):
        try:
            for k in range(calls):
                s0 = ((t * calls + k) * batch) % max(1, n - batch)
                c.match_host(ix, (pb, ho[s0:s0 + batch + 1]), exact=True).free()
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    warm = [threading.Thread(target=run, args=(t,)) for t in range(threads)]  # (every caller's pinned staging)
    for x in warm:
        x.start()
    for x in warm:
        x.join()
    th = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    if errs:
        raise RuntimeError(errs[0])
    return {"threads": threads, "calls_per_thread": calls, "topics_per_call": batch,
            "topics_per_s": threads * calls * batch / dt, "ms_per_call_avg": dt * 1e3 / calls}


def multi_measure(c, ix, devices, pb, ho, n_topics, nnz, single, d):
    """On a multi-device context c holding snapshot ix (replicated on every
    device): one host-buffer emqx_gm_match of the whole page-locked batch spread
    over every device (gm_host.cpp), the NIF-sized concurrent small calls, and
    200-op updates applied on every replica at once (O(delta), each from its own
    predecessor replica).  ix is released."""
    c.match_host(ix, (pb, ho), exact=True).free()  # (warm: pinned staging, pools, workers on every device)
    best, ok = None, True
    for _ in range(2):
        t0 = time.perf_counter()
        h = c.match_host(ix, (pb, ho), exact=True)
        dt = time.perf_counter() - t0
        ok = ok and h.nnz == nnz
        h.free()
        best = dt if best is None else min(best, dt)
    d["host_io_multi_topics_per_s"] = n_topics / best
    d["host_io_multi_ms"] = best * 1e3
    d["host_io_multi_nnz_matches_device"] = ok
    if single.get("host_io_topics_per_s"):
        d["host_io_multi_vs_single_device"] = d["host_io_multi_topics_per_s"] / single["host_io_topics_per_s"]
    d["small_calls"] = small_calls(c, ix, pb, ho)
    if single.get("small_calls"):
        d["small_calls"]["vs_single_device"] = d["small_calls"]["topics_per_s"] / single["small_calls"]["topics_per_s"]
    rounds, last = update_chain(c, ix, own=True)
    d["index_update_replicas"] = {"ops": 200, "update_ms": rounds[-1]["ms"], "rounds": rounds}
    if single.get("update_ms"):
        d["index_update_replicas"]["vs_single_device"] = rounds[-1]["ms"] / single["update_ms"]
    if len(set(devices)) == 1:
        d["note"] = (f"one-GPU rehearsal: {len(devices)} replicas share this GPU's HBM, CUs and PCIe link "
                     "(an update's device passes run side by side on one GPU)")
    last.release()
    return d


def multi_device(ctx, idx, img, devices, pb, ho, n_topics, nnz, single):
    """The drop-in path's multi-GPU form, rehearsed in this process (N=1):
    ONE library context over ``devices`` (what the NIF opens on a node:
    emqx_gm_opts.n_devices), outside the timed region.  The index goes in once
    (an import of this rank's snapshot) and is replicated device to device in a
    tree; then multi_measure.  ``single``: this rank's single-device figures."""
    from emqx_amd import Context
    d = {"devices": list(devices), "process": "in-process"}
    ctx.pool_trim()  # (this rank's cached buffers and spare tables: C5's replicas need the room)
    with Context(devices=list(devices)) as c:
        t0 = time.perf_counter()
        ix = c.import_index(img, d_blob=idx.device_blob()[0])
        st = c.update_stats()
        idx.release()  # (the replicas are copies: this rank's snapshot is no longer needed)
        d["import_and_replicate_ms"] = (time.perf_counter() - t0) * 1e3
        d["replicate_ms"] = st["replicate_ms"]
        d["replica_mode"] = st["replica_mode"]
        d["replicated_bytes"] = int(ix.info.device_bytes) * (len(devices) - 1)
        d["import_mirror_loaded"] = st["mirror_loaded"]
        del img
        multi_measure(c, ix, devices, pb, ho, n_topics, nnz, single, d)
    return d


def multi_device_child(a):
    """`--multi-child DEVICES`: the multi-device measurement in a process of its
    own (rank 0 at N>1 starts it while the other ranks wait on the host): a
    fault on the 8-GPU node then costs this detail, not the bench line.  Builds
    the config's index through ONE context over the devices (compiled once,
    replicated in a tree), generates the same topic stream and prints one JSON
    line."""
    import numpy as np
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    devices = [int(x) for x in a.multi_child.split(",")]
    single = json.loads(a.multi_single) if a.multi_single else {}
    n_filters = a.filters or {"c1": 10_000, "c2": 1_000_000, "c3": 10_000_000, "c5": 100_000_000}[a.config]
    n_topics = a.topics or {"c1": 1_000_000, "c2": 100_000_000, "c3": 100_000_000, "c5": 100_000_000}[a.config]
    codes = gen_filter_codes(a.seed, n_filters, wildcard_only=a.config == "c2")
    fpack = render_codes(codes)
    d = {"devices": devices, "process": "child"}
    with Context(devices=devices) as c:
        t0 = time.perf_counter()
        ix = c.build_index(fpack)
        st = c.update_stats()
        d["build_and_replicate_ms"] = (time.perf_counter() - t0) * 1e3
        d["replicate_ms"] = st["replicate_ms"]
        d["replica_mode"] = st["replica_mode"]
        d["replicated_bytes"] = int(ix.info.device_bytes) * (len(devices) - 1)
        del fpack
        db, do, tbytes = c.gen_topics_device(codes, a.seed, 0, n_topics)
        r = c.match_device(ix, db, do, n_topics, exact=True)
        nnz = r.nnz
        r.free()
        ho = np.zeros(n_topics + 1, np.uint64)
        c.memcpy_d2h(ho, do, (n_topics + 1) * 8)
        pb = c.host_alloc(tbytes + 64)
        c.memcpy_d2h(pb, db, tbytes)
        pb[tbytes:] = 0
        c.dev_free(db)
        c.dev_free(do)
        multi_measure(c, ix, devices, pb, ho, n_topics, nnz, single, d)
        c.host_free(pb)
    print(json.dumps(d), flush=True)


def run_multi_child(a, devices, single):
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "GM_BENCH_DEVICE", "GM_BENCH_BACKEND")}
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--multi-child", ",".join(map(str, devices)),
           "--config", a.config, "--seed", str(a.seed), "--multi-single", json.dumps(single)]
    if a.filters:
        cmd += ["--filters", str(a.filters)]
    if a.topics:
        cmd += ["--topics", str(a.topics)]
    try:
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    except subprocess.TimeoutExpired:
        return {"devices": devices, "error": "timed out (900 s)"}
    lines = [l for l in p.stdout.splitlines() if l.startswith('{"devices"')]
    if p.returncode != 0 or not lines:
        return {"devices": devices, "error": f"exit {p.returncode}", "stderr_tail": p.stderr[-2000:]}
    return json.loads(lines[-1])


def main():
    a = parse()
    heartbeat()
    if a.multi_child:
        return multi_device_child(a)
    world, rank, local, pg = dist_setup(a.gpus)
    import numpy as np
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes

    cfg = a.config
    if cfg == "c4":
        return bench_c4(a, world, rank, local, pg)
    if cfg == "c5" and a.plan == "hash":
        return bench_c5(a, world, rank, local, pg)
    if cfg == "c5" and a.plan == "prefix":
        return bench_c5_prefix(a, world, rank, local, pg)
    n_filters = a.filters or {"c1": 10_000, "c2": 1_000_000, "c3": 10_000_000, "c5": 100_000_000}[cfg]
    n_topics = a.topics or {"c1": 1_000_000, "c2": 100_000_000, "c3": 100_000_000, "c5": 100_000_000}[cfg]
    wildcard_only = cfg == "c2"

    ctx = Context(local)
    t_build0 = time.perf_counter()
    codes = gen_filter_codes(a.seed, n_filters, wildcard_only=wildcard_only)
    # only a compiling rank renders the filter strings (C5: 100M filters, ~2.6 GB of text
    # plus offsets); the others import rank 0's image and need just the codes, which
    # generate their topics
    compiles = world == 1 or rank == 0 or a.build_each
    fpack = render_codes(codes) if compiles else None
    t_gen = time.perf_counter() - t_build0  # the synthetic filter set (codes, rendered strings): bench-side
    idx, source = replicated_index(a, ctx, world, rank, local, pg, fpack)
    t_build = time.perf_counter() - t_build0
    # index_build_s: filter generation + the index (compile, or import); index_compile_s: the
    # library's part alone (emqx_gm_index_build, or the image broadcast and import)
    build_info = {"index_source": source, "index_build_s": t_build, "filters_gen_s": t_gen,
                  "index_compile_s": t_build - t_gen}
    if source.startswith("imported"):
        # the mirror policy at an import (gm_image.cpp): the build's -- kept up to 8 GiB of
        # tables (from the image's own bytes), lazy above -- as the library observed it
        ust = ctx.update_stats()
        build_info.update(index_import_mirror_loaded=ust["mirror_loaded"],
                          index_import_mirror_bytes=ust["mirror_bytes"], index_import_mirror_ms=ust["mirror_ms"])
    if pg is not None:  # how many ranks compiled, the slowest rank's build, the largest host RSS
        n_built = _reduce_tensor(local, float(source == "built"))
        pg.all_reduce(n_built)
        build_info.update(ranks_compiled=int(n_built.item()), index_build_s_max=barrier_max(pg, local, t_build),
                          host_peak_rss_gb_max=barrier_max(pg, local, host_peak_rss_gb()),
                          host_peak_rss_gb_per_rank=gather_floats(pg, local, world, host_peak_rss_gb()),
                          replicas_agree=replicas_agree(ctx, idx, codes, a.seed, pg, local))
    db, do, tbytes = ctx.gen_topics_device(codes, a.seed, rank * n_topics, n_topics)

    # warmup (also yields the per-batch constants for the roofline)
    res = None
    for _ in range(max(a.warmup, 1)):
        if res is not None:
            res.free()
        res = ctx.match_device(idx, db, do, n_topics, exact=True)
    st = ctx.stats()
    fbytes_matched = ctx.matched_filter_bytes(idx, res)
    nnz = res.nnz
    res.free()

    barrier(pg)
    ctx.synchronize()
    kern_ms = []
    last = None
    t0 = time.perf_counter()
    if a.no_pipeline:
        for _ in range(a.steps):
            if last is not None:
                last.free()
            last = ctx.match_device(idx, db, do, n_topics, exact=True)
            kern_ms.append(ctx.last_kernel_ms())
    else:
        # two calls in flight (emqx_gm_match_submit / _wait): step i+1's kernels
        # are queued before the host finishes step i, as a serving loop does
        # The main pass is timed (HIP events on its stream) on every te-th call
        # of the timed region: a timed call's two timestamps each leave the
        # device ~5 us idle, which a 0.1-ms C1 step notices (EMQX_GM_NO_TIMING)
        te = a.time_every or (8 if cfg == "c1" else 1)
        cur = ctx.match_submit(idx, db, do, n_topics, exact=True, timed=True)
        for i in range(a.steps):
            nxt = (ctx.match_submit(idx, db, do, n_topics, exact=True, timed=(i + 1) % te == 0)
                   if i + 1 < a.steps else None)
            r = cur.wait()
            if i % te == 0:
                kern_ms.append(ctx.last_kernel_ms())
            if last is not None:
                last.free()
            last, cur = r, nxt
    ctx.synchronize()
    barrier(pg)
    elapsed = time.perf_counter() - t0
    elapsed = barrier_max(pg, local, elapsed)

    ms_per_step = elapsed * 1000.0 / a.steps
    value = world * n_topics * a.steps / elapsed
    # algorithmic bytes of one match call's main pass, k_match_fused:
    #   B = Σ len(topic) + 8·n (offsets) + 16·P + Σ_matches (4 + len f) + 8·n (row offsets)
    algo = tbytes + 8 * n_topics + 16 * st["probes"] + 4 * nnz + fbytes_matched + 8 * n_topics
    kern_ms = [k for k in kern_ms if k > 0]  # (an untimed call reports 0)
    if not kern_ms:
        raise SystemExit("bench: no timed k_match_fused launch in the timed region (--time-every > --steps?)")
    kavg = sum(kern_ms) / len(kern_ms)
    achieved = algo / (kavg / 1e3) / 1e9
    # roofline.traffic: the PMC bytes of this very build (scripts/profile.sh ->
    # scripts/traffic.py stamps the library's hash); a stale file gives null
    traffic, lines, traffic_note = None, None, "no profile of this build (scripts/gpu_full.sh)"
    pmc = {}  # the same profile's L2 hit rate and wave occupancy
    try:
        import hashlib
        with open(a.traffic_json) as f:
            tj = json.load(f)
        with open(os.path.join(ROOT, "emqx_amd", "libemqx_gpu_match.so"), "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()[:16]
        if tj.get("config") == cfg and tj.get("n_topics") == n_topics and tj.get("lib_sha16") == sha:
            traffic, lines = tj.get("hbm_bytes_per_launch"), tj.get("lines_per_topic")
            pmc = {k: tj[k] for k in ("l2_hit_rate", "l2_requests_per_topic", "occupancy_waves_per_cu",
                                      "occupancy_frac") if tj.get(k) is not None}
            traffic_note = f"PMC of this build ({os.path.relpath(a.traffic_json, ROOT)}, lib {sha})"
    except (OSError, ValueError):
        pass

    out = {
        "metric": METRIC, "value": value, "unit": "topics/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (seeded §8d generator, topics generated on device)",
        "config": {"workload": {"c1": "C1: 10k mixed filters, 1M topics", "c2": "C2: 1M wildcard filters, "
                                "100M-topic publish batch per GPU", "c3": "C3: 10M mixed filters, replicated index, "
                                "100M topics per GPU", "c5": "C5: 100M mixed filters, replicated index (the "
                                "unsharded index fits one GPU), 100M topics per GPU"}[cfg]
                   + " (match_routes semantics, CSR of sorted filter ids)",
                   "filters": int(idx.n_filters), "topics_per_gpu": n_topics,
                   "parallelism": f"replicated index, batch partitioned over {world} GPU(s)"},
        "matches_per_sec": world * nnz * a.steps / elapsed,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_note,
                     "lines_per_topic": lines, **pmc,
                     # the SURVEY §8d formula credits Σ len(f) of the matched filters, bytes no kernel reads
                     "frac_without_filter_bytes": (algo - fbytes_matched) / (kavg / 1e3) / 1e9 / HBM_PEAK_GBS,
                     "kernel": "k_match_fused", "kernel_ms": kavg, "timed_launches": len(kern_ms),
                     # SURVEY §8d asks for the median of the runs too (the mean is what frac uses)
                     "kernel_ms_median": sorted(kern_ms)[len(kern_ms) // 2],
                     "algo_bytes_per_launch": algo,
                     # the walk's physical bound: random 128-B fabric line requests (PMC TCC_EA0_RDREQ per
                     # topic) against the calibrated ceiling of this access pattern (scripts/randread.hip:
                     # 52.9 G random lines/s beyond the Infinity Cache, profiles/r02_randread/)
                     "fabric_lines_per_s": None if lines is None else lines * n_topics / (kavg / 1e3),
                     "frac_of_random_line_ceiling": None if lines is None else
                     lines * n_topics / (kavg / 1e3) / RANDOM_LINE_CEILING},
        "detail": {"nnz_per_step": nnz, "matches_per_topic": nnz / n_topics, "probes_per_topic": st["probes"] /
                   n_topics, "overflow_rows": st["n_overflow"], "topic_bytes": tbytes,
                   "index_device_bytes": int(idx.info.device_bytes), "index_nodes": int(idx.info.n_nodes),
                   **build_info, "host_peak_rss_gb": host_peak_rss_gb(),
                   "device_ms_per_call": st["total_device_ms"],
                   "calls_in_flight": 1 if a.no_pipeline else 2},
    }
    pb = ho = None
    multi = not a.no_multi and not a.no_host_io and (world > 1 or a.replicas > 1)
    mimg = None
    if multi and rank == 0 and world == 1:
        # the image (host part; the tables are copied from this rank's device blob) that
        # the multi-device context imports, taken before this rank's own updates move the
        # snapshot line's host mirror on (an image carries the line's mirror metadata)
        mimg = idx.export(with_blob=False)
    if not a.no_host_io and rank == 0:
        # PCIe-inclusive, outside the timed region: the same batch handed over in host
        # memory and its CSR returned in host memory (the NIF's call, gm_host.cpp)
        hd, pb, ho = host_io(ctx, idx, db, do, tbytes, n_topics, nnz)
        out["detail"].update(hd)
    if rank == 0 and world == 1 and not a.no_update:
        # incremental maintenance, outside the timed region: 100 deletes +
        # 100 inserts patched into this index, three times in a row, and a match of the same batch on
        # the result.  The first update of an index whose host mirror is lazy (C5: 53 GB of
        # tables) downloads the mirror -- the library reports whether it did
        # (emqx_gm_last_update_stats); the last is the steady state.
        # (three rounds: the third takes the blob the first result released -- the steady
        # state of a broker applying windows of updates; the second, with the original
        # snapshot still held, may take a fresh allocation, whose cost is box dependent)
        rounds, cur = update_chain(ctx, idx, n_rounds=3)
        ks = []
        for _ in range(3):
            r = ctx.match_device(cur, db, do, n_topics, exact=True)
            ks.append(ctx.stats()["match_kernel_ms"])
            r.free()
        f0 = rounds[0]
        out["detail"]["index_update"] = {"ops": 200, "update_ms": rounds[-1]["ms"], "first_update_ms": f0["ms"],
                                         "first_includes_mirror_download": f0["mirror_loaded"],
                                         "first_mirror_bytes": f0["mirror_bytes"], "first_mirror_ms": f0["mirror_ms"],
                                         "index_source": source, "rounds": rounds,
                                         "match_kernel_ms_after": min(ks), "vs_flat": min(ks) / min(kern_ms)}
        cur.release()
    if rank == 0 and world == 1 and not a.no_update and (cfg != "c5" or a.subs_update):
        out["detail"]["subs_update"] = subs_update(ctx, fpack)
    big = cfg == "c5" and n_filters >= 50_000_000  # the oracle over this many keys does not fit the box
    if big and rank == 0 and not a.no_parity:
        # the oracle over 100M keys does not fit the box's memory: the committed C5
        # fixture (2,000 strided topics of the stream, rows as filter strings) instead
        out["parity_sample"] = fixture_check(ctx, idx, "c5")
    # the cpu_baseline leg (oracle): timed on all host cores at N=1, and, outside the
    # timed region, the last step's CSR checked against it on a strided sample
    want_cpu = rank == 0 and world == 1 and not a.no_cpu and not big
    want_parity = rank == 0 and not a.no_parity and not big
    if want_cpu or want_parity:
        threads = a.cpu_threads or len(os.sched_getaffinity(0))
        r = oracle_router(fpack)
        if want_parity:
            # C3's 10M-filter oracle runs ~0.5 M topics/s on the box's quota: a 200k-topic sample
            out["parity_sample"] = parity_sample(ctx, r, last, codes, sorted_unique(*fpack), a.seed,
                                                 rank * n_topics, n_topics, threads,
                                                 width=50_000 if n_filters <= 2_000_000 else 10_000)
        if want_cpu:
            out["cpu_baseline"] = cpu_baseline(r, codes, a.seed, a.cpu_seconds, threads)
            out["vs_cpu"] = value / out["cpu_baseline"]["value"]
            out["vs_cpu_optimized"] = value / out["cpu_baseline"]["optimized"]["value"]
        del r
    last.free()
    ctx.dev_free(db)
    ctx.dev_free(do)
    # the drop-in path's multi-GPU form (one context over the GPUs), rank 0, while the
    # other ranks wait on the host
    host_barrier(pg)
    if multi and rank == 0:
        single = {"host_io_topics_per_s": out["detail"].get("host_io_topics_per_s"),
                  "update_ms": out["detail"].get("index_update", {}).get("update_ms"),
                  "small_calls": small_calls(ctx, idx, pb, ho)}
        out["detail"]["small_calls_single_device"] = single["small_calls"]
        if world == 1:
            out["detail"]["multi_device"] = multi_device(ctx, idx, mimg, [local] * a.replicas, pb, ho, n_topics,
                                                         nnz, single)
            idx = mimg = None
        else:
            # N>1: one context over all the node's GPUs, in a process of its own
            devices = [local] * world if "GM_BENCH_DEVICE" in os.environ else list(range(world))
            out["detail"]["multi_device"] = run_multi_child(a, devices, single)
    host_barrier(pg)
    if pb is not None:
        ctx.host_free(pb)
    if idx is not None:
        idx.release()
    ctx.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.destroy_process_group()


def bench_c5(a, world, rank, local, pg):
    """C5: filters hash-sharded over the ranks (global ids), every rank matches
    the whole batch against its shard, rows exchanged by all-to-all (RCCL) and
    merged on the device by global id; rank q ends with topic slice q."""
    import numpy as np
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    from emqx_amd.sharded import ShardedMatcher, plan_shard
    n_filters = a.filters or 100_000_000
    n_topics = a.topics or 100_000_000
    torch_first(local)
    ctx = Context(local)
    t0 = time.perf_counter()
    codes = gen_filter_codes(a.seed, n_filters)
    fb, fo = render_codes(codes)
    sfb, sfo, gids, n_unique = plan_shard(fb, fo, world, rank)
    del fb, fo
    idx = ctx.build_index_shard((sfb, sfo), gids)
    t_build = time.perf_counter() - t0
    db, do, tbytes = ctx.gen_topics_device(codes, a.seed, 0, n_topics)  # same batch on every rank
    m = ShardedMatcher(ctx, idx, world, rank, dist=pg, device_tensors=BACKEND == "nccl")
    for _ in range(max(a.warmup, 1)):
        res, first, rows = m.match_device(db, do, n_topics)
        res.free()
    barrier(pg)
    ctx.synchronize()
    t0 = time.perf_counter()
    nnz, res = 0, None
    for _ in range(a.steps):
        if res is not None:
            res.free()
        res, first, rows = m.match_device(db, do, n_topics)
        nnz = res.nnz
    ctx.synchronize()
    barrier(pg)
    elapsed = barrier_max(pg, local, time.perf_counter() - t0)
    if pg is not None:
        t = _reduce_tensor(local, float(nnz))
        pg.all_reduce(t)
        nnz = int(t.item())
    out = {"metric": "publish topics matched/sec, filters sharded over GPUs (C5)",
           "value": n_topics * a.steps / elapsed, "unit": "topics/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": elapsed * 1e3 / a.steps, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (seeded §8d generator, mixed filters; topics generated on device)",
           "config": {"workload": f"C5: {n_unique} filters hash-sharded over {world} GPU(s), {n_topics}-topic batch, "
                                  "all-to-all row exchange + device merge by global id",
                      "filters": n_unique, "topics": n_topics, "parallelism": f"filter shards x{world}"},
           "matches_per_sec": nnz * a.steps / elapsed,
           "detail": {"index_build_s": t_build, "shard_filters": int(len(gids)),
                      "exchange_bytes_per_step_rank0": m.last_exchange_bytes}}
    if rank == 0 and not a.no_parity and n_filters < 50_000_000:
        # rank 0's merged rows (its slice of the batch: every shard's piece merged
        # by global id) against the oracle over the whole filter set
        threads = a.cpu_threads or len(os.sched_getaffinity(0))
        fpack = render_codes(codes)
        out["parity_sample"] = parity_sample(ctx, oracle_router(fpack), res, codes, sorted_unique(*fpack), a.seed,
                                             first, rows, threads, width=min(50_000, rows // 4 or 1))
    res.free()
    ctx.dev_free(db)
    ctx.dev_free(do)
    idx.release()
    ctx.close()
    if rank == 0:
        print(json.dumps(out), flush=True)


def bench_c5_prefix(a, world, rank, local, pg):
    """C5 prefix-sharded (gm_route.hip): filters partitioned by first word
    over the ranks (root wildcards on every shard), each rank publishes its own
    batch, every topic is routed to the one shard that holds all the filters it
    can match and walked there (all-to-all of topics, rows back in batch order):
    a rank walks ~1/N of the job, so topic throughput grows with N ("weak":
    each rank publishes n topics per step)."""
    import numpy as np
    from emqx_amd import Context
    from emqx_amd.engine import gen_filter_codes, render_codes
    from emqx_amd.sharded import PrefixShardedMatcher, plan_prefix_shard
    n_filters = a.filters or 100_000_000
    n_topics = a.topics or 100_000_000
    torch_first(local)
    ctx = Context(local)
    t0 = time.perf_counter()
    codes = gen_filter_codes(a.seed, n_filters)
    fb, fo = render_codes(codes)
    sfb, sfo, gids, n_unique, route = plan_prefix_shard(fb, fo, world, rank)
    del fb, fo
    idx = ctx.build_index_shard((sfb, sfo), gids)
    t_build = time.perf_counter() - t0
    db, do, tbytes = ctx.gen_topics_device(codes, a.seed, rank * n_topics, n_topics)
    dev = BACKEND == "nccl"
    if dev:
        m = PrefixShardedMatcher(ctx, idx, route, world, rank, dist=pg)
        step = lambda: m.match_device(db, do, n_topics)  # noqa: E731
    else:  # rehearsal (gloo, ranks sharing a device): the exchange on host tensors, the match on the device
        hb = np.zeros(tbytes + 64, np.uint8)
        ho = np.zeros(n_topics + 1, np.uint64)
        ctx.memcpy_d2h(hb, db, tbytes)
        ctx.memcpy_d2h(ho, do, (n_topics + 1) * 8)
        m = PrefixShardedMatcher(ctx, idx, route, world, rank, dist=pg, device_tensors=False,
                                 match_fn=lambda tb, to: ctx.match(idx, (tb, to), exact=True))
        step = lambda: m.match_host(hb, ho)  # noqa: E731
    for _ in range(max(a.warmup, 1)):
        r = step()
        if dev:
            r.free()
    barrier(pg)
    ctx.synchronize()
    t0 = time.perf_counter()
    nnz, last = 0, None
    for _ in range(a.steps):
        if dev and last is not None:
            last.free()
        last = step()
        nnz = last.nnz if dev else int(last[0][-1])
    ctx.synchronize()
    barrier(pg)
    elapsed = barrier_max(pg, local, time.perf_counter() - t0)
    walked = [m.last_topics_walked]
    if pg is not None:
        import torch
        t = torch.zeros(world + 1, dtype=torch.float64, device=f"cuda:{local}" if dev else "cpu")
        t[rank] = float(m.last_topics_walked)
        t[world] = float(nnz)
        pg.all_reduce(t)
        walked = [int(x) for x in t[:world].tolist()]
        nnz = int(t[world].item())
    out = {"metric": "publish topics matched/sec, filters prefix-sharded over GPUs (C5)",
           "value": world * n_topics * a.steps / elapsed, "unit": "topics/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": elapsed * 1e3 / a.steps, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (seeded §8d generator, mixed filters; topics generated on device)",
           "config": {"workload": f"C5: {n_unique} filters prefix-sharded over {world} GPU(s) (first word; root "
                                  f"wildcards on every shard), {n_topics} topics per GPU routed to their shard",
                      "filters": n_unique, "topics_per_gpu": n_topics, "parallelism": f"prefix shards x{world}"},
           "matches_per_sec": nnz * a.steps / elapsed,
           "detail": {"index_build_s": t_build, "shard_filters": int(len(gids)), "topics_walked_per_rank": walked,
                      "exchange_bytes_per_step_rank0": m.last_exchange_bytes,
                      "device_exchange": dev}}
    if rank == 0 and not a.no_parity and n_filters < 50_000_000:
        # rank 0's rows of its own batch (walked on every shard they were routed to,
        # back in batch order) against the oracle over the whole filter set
        threads = a.cpu_threads or len(os.sched_getaffinity(0))
        fpack = render_codes(codes)
        out["parity_sample"] = parity_sample(ctx, oracle_router(fpack), last, codes, sorted_unique(*fpack), a.seed,
                                             0, n_topics, threads, width=min(50_000, n_topics // 4 or 1))
    if dev:
        last.free()
    ctx.dev_free(db)
    ctx.dev_free(do)
    idx.release()
    route.release()
    ctx.close()
    if rank == 0:
        print(json.dumps(out), flush=True)


def bench_c4(a, world, rank, local, pg):
    """C4 hot fan-out: 1k topics x 1M subscribers each (10^9 deliveries),
    split across the ranks: the deliveries are numbered in
    emqx_gm_fanout order and rank r produces the contiguous range
    [T*r/N, T*(r+1)/N) (emqx_gm_fanout_part), so rows and 1M-wide rows alike
    are cut across GPUs; the parts are disjoint and sum to T ("strong"
    scaling: the job is fixed, N GPUs share it)."""
    import numpy as np
    from emqx_amd import Context
    K, S = 1000, 1_000_000
    filters = [b"hot/#", b"hot/+/x/#"] + [b"hot/%d/x/y/z" % k for k in range(K)]
    # hot/# -> 0..599,999; hot/+/x/# -> 600,000..999,899; each exact topic -> 999,900..999,999
    lists = [np.arange(0, 600_000), np.arange(600_000, 999_900)] + [np.arange(999_900, S)] * K
    so = np.zeros(len(lists) + 1, np.uint64)
    so[1:] = np.cumsum([len(x) for x in lists])
    si = np.concatenate(lists).astype(np.uint32)
    ctx = Context(local)
    idx = ctx.build_index(filters, subs=(so, si))
    topics = [b"hot/%d/x/y/z" % k for k in range(K)]
    from emqx_amd.engine import pack
    tb, to = pack(topics)
    d_tb = ctx.dev_alloc(len(tb))
    d_to = ctx.dev_alloc(len(to) * 8)
    ctx.memcpy_h2d(d_tb, tb, len(tb))
    ctx.memcpy_h2d(d_to, to, len(to) * 8)
    m = ctx.match_device(idx, d_tb, d_to, K, exact=True)
    for _ in range(max(a.warmup, 1)):
        r, first = ctx.fanout_part(idx, m, rank, world)
        r.free()
    barrier(pg)
    ctx.synchronize()
    kms = []
    t0 = time.perf_counter()
    part = 0
    for _ in range(a.steps):
        r, first = ctx.fanout_part(idx, m, rank, world)
        part = r.nnz
        kms.append(ctx.stats()["match_kernel_ms"])
        r.free()
    ctx.synchronize()
    barrier(pg)
    elapsed = barrier_max(pg, local, time.perf_counter() - t0)
    parts = [part]
    if pg is not None:
        import torch
        t = torch.zeros(world, dtype=torch.float64, device=f"cuda:{local}" if BACKEND == "nccl" else "cpu")
        t[rank] = float(part)
        pg.all_reduce(t)
        parts = [int(x) for x in t.tolist()]
    pairs = sum(parts)
    # algorithmic bytes of this rank's k_fanout_copy launch: its deliveries
    # written (4 B each), the row offsets, and the distinct subscriber lists read once
    algo = 4 * part + 8 * (K + 1) + 4 * S
    kavg = sum(kms) / len(kms)
    achieved = algo / (kavg / 1e3) / 1e9
    # roofline.traffic: the PMC bytes of k_fanout_copy from a profile of this very build
    # (scripts/profile.sh CONFIG=c4 -> scripts/traffic.py --kernel k_fanout_copy), else null
    traffic, traffic_note, pmc = None, "no profile of this build", {}
    try:
        import hashlib
        with open(a.traffic_json) as f:
            tj = json.load(f)
        with open(os.path.join(ROOT, "emqx_amd", "libemqx_gpu_match.so"), "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()[:16]
        if tj.get("config") == "c4" and tj.get("kernel") == "k_fanout_copy" and tj.get("lib_sha16") == sha \
                and world == 1:
            traffic = tj.get("hbm_bytes_per_launch")
            pmc = {k: tj[k] for k in ("l2_hit_rate", "occupancy_waves_per_cu", "occupancy_frac")
                   if tj.get(k) is not None}
            traffic_note = f"PMC of this build ({os.path.relpath(a.traffic_json, ROOT)}, lib {sha})"
    except (OSError, ValueError):
        pass
    out = {"metric": "hot-topic fan-out deliveries/sec (C4: 1k topics x 1M subscribers)",
           "value": pairs * a.steps / elapsed, "unit": "deliveries/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": elapsed * 1e3 / a.steps, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "u32", "data": "synthetic (C4 layout, SURVEY.md §8d)",
           "config": {"workload": "C4: 1k hot topics x 1M subscribers, CSR subscriber lists, delivery range "
                                  f"split over {world} GPU(s)", "pairs": pairs, "pairs_per_rank": parts},
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_note,
                        "kernel": "k_fanout_copy", "kernel_ms": kavg, "algo_bytes_per_launch": algo, **pmc}}
    m.free()
    ctx.dev_free(d_tb)
    ctx.dev_free(d_to)
    idx.release()
    ctx.close()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
