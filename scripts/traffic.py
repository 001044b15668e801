#!/usr/bin/env python3
"""HBM traffic per launch of the dominant kernel from rocprofv3 PMC passes.

Reads the separate FETCH_SIZE and WRITE_SIZE passes that scripts/profile.sh
writes (gpurun_out/prof/pmc_fetch, pmc_write; one counter group per run) and
writes profiles/traffic.json, which bench.py reports as roofline.traffic.

Units and corrections (MI355X_MICROARCH.md § HBM): FETCH_SIZE / WRITE_SIZE are
KB (1024 B).  On gfx950 FETCH_SIZE = TCC_EA0_RDREQ x 64 B while a request moves
128 B, so the fetch figure is doubled.  The counters sit on the L2's fabric
side: Infinity-Cache hits are included, so this is L2-miss traffic (an upper
bound on HBM bytes).  Only launches over the whole batch (Grid_Size >= the
batch's topics) are averaged.

usage: traffic.py [prof_dir] [--kernel k_match_reg] [--topics N] [--config c2] [--out path]
"""
import argparse
import csv
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel, min_grid, counter=None):
    vals = []
    if not os.path.exists(path):
        return vals
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"] and int(r["Grid_Size"]) >= min_grid and \
                    (counter is None or r["Counter_Name"] == counter):
                vals.append(float(r["Counter_Value"]))
    return vals


def per_launch_sum(path, kernels, min_grid, counter=None):
    """Per-launch average of each kernel, summed over the kernels of one match call."""
    total, counts = 0.0, []
    for k in kernels:
        v = per_launch(path, k, min_grid, counter)
        if not v:
            return None, counts
        total += statistics.mean(v)
        counts.append(len(v))
    return total, counts


def main():
    p = argparse.ArgumentParser()
    p.add_argument("prof", nargs="?", default=os.path.join(ROOT, "gpurun_out", "prof"))
    p.add_argument("--kernel", default="k_match_fused", help="comma-separated kernels of one match call")
    p.add_argument("--topics", type=int, default=100_000_000)
    p.add_argument("--config", default="c2")
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "traffic.json"))
    a = p.parse_args()
    ks = a.kernel.split(",")
    fetch, nf = per_launch_sum(os.path.join(a.prof, "pmc_fetch", "run_counter_collection.csv"), ks, a.topics)
    write, nw = per_launch_sum(os.path.join(a.prof, "pmc_write", "run_counter_collection.csv"), ks, a.topics)
    if fetch is None or write is None:
        raise SystemExit(f"no full-batch {a.kernel} launches in {a.prof}")
    fetch_b = fetch * 1024 * 2  # KB -> B, gfx950 x2 correction
    write_b = write * 1024
    rdreq, _ = per_launch_sum(os.path.join(a.prof, "pmc_ea", "run_counter_collection.csv"), ks, a.topics, "TCC_EA0_RDREQ_sum")
    # L2 hit rate and requests (SURVEY §8d "L2 hit %"), from the pmc_l2 pass
    l2 = os.path.join(a.prof, "pmc_l2", "run_counter_collection.csv")
    hit, _ = per_launch_sum(l2, ks, a.topics, "TCC_HIT_sum")
    miss, _ = per_launch_sum(l2, ks, a.topics, "TCC_MISS_sum")
    # wave occupancy (§8d) from the pmc_sq pass: SQ_WAVE_CYCLES counts quad-cycles
    # summed over waves (MI355X_MICROARCH.md, s_memtime vs SQ units); SQ_BUSY_CYCLES
    # is summed over the 32 shader engines (8 XCDs x 4), so the kernel's cycles are
    # SQ_BUSY_CYCLES / 32 and the mean resident waves per CU is
    # 4 * SQ_WAVE_CYCLES / (256 CUs * kernel cycles) (of at most 32)
    sq = os.path.join(a.prof, "pmc_sq", "run_counter_collection.csv")
    wcyc, _ = per_launch_sum(sq, ks, a.topics, "SQ_WAVE_CYCLES")
    busy, _ = per_launch_sum(sq, ks, a.topics, "SQ_BUSY_CYCLES")
    waves, _ = per_launch_sum(sq, ks, a.topics, "SQ_WAVES")
    occ = 4 * wcyc / (256 * busy / 32) if wcyc and busy else None
    import hashlib
    with open(os.path.join(ROOT, "emqx_amd", "libemqx_gpu_match.so"), "rb") as f:
        lib_sha = hashlib.sha256(f.read()).hexdigest()[:16]
    out = {"config": a.config, "n_topics": a.topics, "kernel": a.kernel,
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": fetch_b + write_b, "launches": [nf, nw],
           "lines_per_topic": None if rdreq is None else rdreq / a.topics,
           "l2_hit_rate": hit / (hit + miss) if hit is not None and miss is not None else None,
           "l2_requests_per_topic": (hit + miss) / a.topics if hit is not None and miss is not None else None,
           "occupancy_waves_per_cu": occ,
           "occupancy_frac": None if occ is None else occ / 32,
           "wave_lifetime_cycles": 4 * wcyc / waves if wcyc and waves else None,
           "lib_sha16": lib_sha,
           "note": "FETCH_SIZE x1024 x2 (gfx950 correction) + WRITE_SIZE x1024 per launch; L2 fabric side, "
                   "Infinity-Cache hits included"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
