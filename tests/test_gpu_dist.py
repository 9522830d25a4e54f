"""Multi-GPU rehearsal on one GPU with the real engine (BASELINE configs[4] and the per-GPU shards of
configs[3]): two fresh rank processes started by torch.distributed.run, both on cuda:0 over gloo
(PTLS_BENCH_ONE_DEVICE=1, the path bench.py rehearses), shard the batch with picotls_amd.dist and seal / open their
shards with the HIP kernels. The concatenated shards equal lib/fusion.c on the whole batch, every shard's records open,
and the aggregate throughput every rank reports is the same number (sum of bytes / max wall over ranks).
The 8-GPU node run itself is the driver's (bench.py --gpus 8); tests/test_dist.py covers the sharding arithmetic on CPU.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import FusionRef  # noqa: E402
from picotls_amd.workloads import WORKLOADS, payload_np  # noqa: E402

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("workload,records,ranks", [("shard1200", 65536, 2), ("mixed", 12000, 2), ("mixedrand", 9000, 3)])
def test_ranks_on_one_gpu_shards_equal_fusion(tmp_path, workload, records, ranks):
    if not os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libfusion_ref.so")):
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    env = dict(os.environ, PTLS_BENCH_ONE_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "gpu_dist_worker.py"), "--workload", workload,
           "--records", str(records), "--out", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    info = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(ranks)]
    assert [x["world"] for x in info] == [ranks] * ranks
    assert all(x["ok"] and x["roundtrip"] for x in info)
    assert info[0]["begin"] == 0 and info[-1]["end"] == records
    assert all(info[i]["end"] == info[i + 1]["begin"] for i in range(ranks - 1))
    assert len({round(x["value"], 6) for x in info}) == 1  # one aggregate, computed by the reductions
    assert sum(x["bytes"] for x in info) * 2 / info[0]["maxwall"] / 2**30 == pytest.approx(info[0]["value"], rel=1e-9)
    sealed = np.concatenate([np.load(tmp_path / f"rank{i}.npy") for i in range(ranks)])

    wl = WORKLOADS[workload].scaled(records)
    g = wl.descriptors(0, records)
    keys, ivs = wl.keys()
    pt = payload_np(wl.seed, 0, g.pt_bytes).copy()  # the workers zero their slot padding; fusion reads record bytes only
    want = np.zeros(g.sealed_bytes, np.uint8)
    FusionRef().run_batch(True, keys, ivs, wl.key_size, g.seal, pt, wl.aad_arena(g, 0), want, nthreads=8)
    assert sealed.size == want.size
    assert np.array_equal(sealed, want)
