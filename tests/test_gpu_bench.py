"""The N>1 path of bench.py, rehearsed on one GPU: two ranks under
torch.distributed.run with the rank plumbing over gloo and both ranks pinned to
device 0 (GM_BENCH_BACKEND / GM_BENCH_DEVICE).  The driver's 2/4/8-GPU runs use
the same code with one rank per GPU over RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(args, world=2):
    env = dict(os.environ, GM_BENCH_BACKEND="gloo", GM_BENCH_DEVICE="0", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-cpu"] + args
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-3000:]  # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_c2():
    one = _run_ranks(["--filters", "20000", "--topics", "1000000"], world=1)
    two = _run_ranks(["--filters", "20000", "--topics", "1000000"], world=2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["detail"]["ranks_compiled"] == 1 and two["detail"]["replicas_agree"] is True
    # weak scaling: each rank matches its own slice, same per-rank work
    assert two["config"]["topics_per_gpu"] == one["config"]["topics_per_gpu"] == 1_000_000
    assert two["value"] > 0 and two["roofline"]["frac"] > 0
    # the two slices are different windows of the same stream: same matches/topic within noise
    assert abs(two["detail"]["matches_per_topic"] - one["detail"]["matches_per_topic"]) < 0.1
    # the drop-in path's multi-GPU form: rank 0 opens ONE context over the ranks' devices (here
    # device 0 twice), replicates the index in a tree, spreads one host-buffer call over both
    # and applies 200-op updates on both replicas at once
    for out, devs in ((one, [0, 0]), (two, [0, 0])):
        m = out["detail"]["multi_device"]
        assert m["devices"] == devs and m["replica_mode"] == "copied", m
        assert m["host_io_multi_topics_per_s"] > 0 and m["host_io_multi_nnz_matches_device"] is True, m
        u = m["index_update_replicas"]
        assert all(r["replica_mode"] == "patched" and r["replicas"] == 1 for r in u["rounds"]), u
    assert one["detail"]["multi_device"]["index_update_replicas"]["vs_single_device"] > 0
    # the host path against its link: bytes per topic each way and the measured peaks
    link = one["detail"]["host_io_link"]
    assert link["h2d_bytes_per_topic"] > 2 and link["h2d_peak_gbs"] > 0 and 0 < link["h2d_frac_of_peak"] < 1.5
    # the first update says what it did (an index built here keeps its mirror: no download)
    assert one["detail"]["index_update"]["first_includes_mirror_download"] is False


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_c5_exchange():
    out = _run_ranks(["--config", "c5", "--plan", "hash", "--filters", "50000", "--topics", "200000"], world=2)
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["detail"]["exchange_bytes_per_step_rank0"] > 0
    assert out["matches_per_sec"] > 0
    # rank 0's merged rows (slice 0: the shards' pieces merged by global id) = the oracle
    assert out["parity_sample"]["ok"] and out["parity_sample"]["topics"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_c5_replicated():
    """C5's default plan (north_star: replicate while the index fits): the
    unsharded index on every rank, the batch partitioned, weak scaling."""
    out = _run_ranks(["--config", "c5", "--filters", "2000000", "--topics", "200000"], world=2)
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["config"]["topics_per_gpu"] == 200_000 and "replicated" in out["config"]["workload"]
    assert out["parity_sample"]["ok"]
    # the index is compiled ONCE (rank 0) and the other rank imports its image
    d = out["detail"]
    assert d["index_source"] == "built" and d["ranks_compiled"] == 1, d
    assert d["replicas_agree"] is True and d["host_peak_rss_gb_max"] > 0
    # the importing rank neither renders the filter strings nor compiles: less host memory
    rss = d["host_peak_rss_gb_per_rank"]
    assert len(rss) == 2 and rss[1] < rss[0], rss


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_c5_prefix():
    """C5 prefix-sharded: each rank walks about half of the two ranks' topics."""
    out = _run_ranks(["--config", "c5", "--plan", "prefix", "--filters", "200000", "--topics", "200000"], world=2)
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    walked = out["detail"]["topics_walked_per_rank"]
    assert sum(walked) == 400_000 and min(walked) > 0.35 * 400_000
    assert out["detail"]["exchange_bytes_per_step_rank0"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_c4():
    out = _run_ranks(["--config", "c4"], world=2)
    assert out["n_gpus"] == 2 and out["config"]["pairs"] == 10**9


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_c5_prefix_one_gpu_device_path():
    """bench.py --config c5 --plan prefix --gpus 1 on its default (nccl) path:
    PrefixShardedMatcher on device tensors, the exchange's copy path at world 1,
    and the oracle parity sample over rank 0's rows."""
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    env.pop("GM_BENCH_BACKEND", None)
    env.pop("GM_BENCH_DEVICE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c5", "--plan", "prefix", "--gpus", "1",
           "--filters", "4000000", "--topics", "2000000", "--steps", "3", "--warmup", "1", "--no-cpu"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=380)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith('{"metric"')][-1])
    assert out["detail"]["device_exchange"] is True
    assert out["detail"]["topics_walked_per_rank"] == [2_000_000]
    assert out["parity_sample"]["ok"], out["parity_sample"]


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_replicated_index_rccl_branch_lockstep():
    """bench.replicated_index on its device-tensor (RCCL) branch, 3 ranks as
    threads on one GPU with a lock-step broadcast: rank 0 compiles, ranks 1-2
    import the broadcast image + device tables; every replica's rows equal rank
    0's and the oracle's, and an imported replica takes an in-place update
    (tests/_replicate_worker.py)."""
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "_replicate_worker.py"), "3", "200000",
                        "100000"], cwd=ROOT, capture_output=True, text=True, timeout=380,
                       env={k: v for k, v in os.environ.items() if k not in ("GM_BENCH_BACKEND", "GM_BENCH_DEVICE")})
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "REPLICATE_OK world=3" in p.stdout
