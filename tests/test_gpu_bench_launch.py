"""bench.py's multi-GPU entry point as the driver can run it: `python bench.py --gpus 2` with
no external launcher starts torch.distributed.run itself (a child process, before any GPU call), and its line carries
the configs[4] strong-scaling leg (shard1200: one global batch split across the ranks) beside the weak-scaling
headline. Both ranks run on cuda:0 over gloo (PTLS_BENCH_ONE_DEVICE=1), the one-GPU rehearsal of the nccl path.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=240):
    env = dict(os.environ, PTLS_BENCH_ONE_DEVICE="1", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert lines, r.stderr[-3000:]
    return json.loads(lines[-1])  # the result line is the last stdout line


def test_bench_self_launches_two_ranks_with_shard1200_leg():
    records = 2048
    out = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--records", str(records), "--extra", "shard1200",
                "--no-cpu-baseline"])
    assert out["n_gpus"] == 2
    assert out["scaling"] == "weak"
    assert out["verified"]["roundtrip"] is True
    assert out["value"] > 0 and out["config"]["records_per_gpu"] == records
    sh = out["extra"]["shard1200"]
    assert sh["n_gpus"] == 2 and sh["scaling"] == "strong"
    assert sh["verified"]["roundtrip"] is True
    want_total = records * 16384 // 1200  # --records scales the extra legs by bytes (bench.py)
    assert sh["records_total"] == want_total
    assert sh["records_per_gpu"] in (want_total // 2, want_total - want_total // 2)
    assert sh["value"] > 0
    assert out["cpu_baseline"] is None  # rank 0 at N = 1 only


def test_bench_eight_ranks_shard_the_configs4_index_space_once():
    """The driver's N = 8 run rehearsed on one GPU: `bench.py --gpus 8` through the
    self-launcher, eight gloo ranks on cuda:0. The configs[4] leg's global batch is split into eight contiguous shards
    that cover its record index space exactly once, every rank's shard round-trips, and the line reports all ranks."""
    records = 1024
    out = _run(["--gpus", "8", "--steps", "1", "--warmup", "1", "--records", str(records), "--extra", "shard1200",
                "--no-cpu-baseline", "--no-e2e"], timeout=600)
    assert out["n_gpus"] == 8 and out["config"]["dist_backend"] == "gloo"
    assert out["verified"]["roundtrip"] is True
    sh = out["extra"]["shard1200"]
    assert sh["n_gpus"] == 8 and sh["scaling"] == "strong" and sh["verified"]["roundtrip"] is True
    total = records * 16384 // 1200
    assert sh["records_total"] == total
    shards = sh["shards"]
    assert len(shards) == 8
    assert shards[0][0] == 0 and shards[-1][1] == total
    assert all(shards[i][1] == shards[i + 1][0] for i in range(7))  # contiguous: every index exactly once
    assert all(z - a in (total // 8, total - 7 * (total // 8)) for a, z in shards)
    assert sh["value"] > 0 and out["value"] > 0
    # every rank's seal / open / wall times, and the slowest rank named
    for leg in (out, sh):
        pr = leg["per_rank"]
        assert len(pr["seal_ms"]) == len(pr["open_ms"]) == len(pr["wall_s"]) == 8
        assert all(t > 0 for t in pr["seal_ms"] + pr["open_ms"] + pr["wall_s"])
        assert pr["wall_s"][pr["slowest_rank"]] == pr["max_wall_s"] and pr["min_wall_s"] <= pr["max_wall_s"]


def test_bench_single_gpu_line_has_shard1200_by_default():
    """The default --extra list includes configs[4] (N = 1 anchor of the scaling curve)."""
    out = _run(["--steps", "1", "--warmup", "1", "--records", "1024", "--no-cpu-baseline", "--extra", "shard1200"])
    assert out["n_gpus"] == 1
    sh = out["extra"]["shard1200"]
    assert sh["scaling"] == "strong" and sh["n_gpus"] == 1 and sh["verified"]["roundtrip"] is True
    # XCD 0's shader clock over each timed leg: a plausible MI355X clock
    for leg in (out, sh):
        assert leg["sclk_mhz"] is not None and 500 < leg["sclk_mhz"] < 3000, leg["sclk_mhz"]
    # ... sampled inside the kernels (ptls_mi355x_debug_kernel_clock: workgroup 0 of every chunked launch)
    assert out["clock_probe"]["in_kernel_launches"] >= 2 and out["clock_probe"]["in_kernel_mhz"] == out["sclk_mhz"]


def test_bench_nccl_process_group_on_one_gpu():
    """The nccl branch of the rank setup (RankContext.from_env: init_process_group("nccl", device_id), the barriers and
    the device-side max / sum reductions of the timings), which the 8-GPU driver run takes: one rank under
    torch.distributed.run, made to join its process group (PTLS_BENCH_PROCESS_GROUP=1; two nccl ranks cannot share
    one GPU)."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PTLS_BENCH_PROCESS_GROUP="1")
    env.pop("PTLS_BENCH_ONE_DEVICE", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
                        "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup",
                        "1", "--records", "1024", "--extra", "shard1200", "--no-cpu-baseline"], capture_output=True,
                       text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert out["config"]["dist_backend"] == "nccl"
    assert out["n_gpus"] == 1 and out["verified"]["roundtrip"] is True
    sh = out["extra"]["shard1200"]
    assert sh["verified"]["roundtrip"] is True and sh["records_total"] == 1024 * 16384 // 1200
