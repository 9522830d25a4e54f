"""bench.py's command line on the CPU: the default legs (every BASELINE config, configs[4] included) and when the
self-launcher starts ranks (never for N = 1 or inside torch.distributed.run)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_default_legs_cover_every_baseline_config(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.gpus == 1 and a.workload == "tls16k"
    assert set(a.extra.split(",")) == {"quic1200", "mixed", "mixedrand", "shard1200", "ptlsbench", "quic64k", "tls64k"}
    assert a.e2e is None  # on for N = 1 at full size (main), off with --no-e2e
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-e2e"])
    assert bench.parse().e2e is False


def test_self_launch_only_outside_a_launcher(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.self_launch(1) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.self_launch(2) is None  # already a rank of torch.distributed.run
