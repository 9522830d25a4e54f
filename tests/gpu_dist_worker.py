"""One rank of the multi-GPU rehearsal (tests/test_gpu_dist.py), started by torch.distributed.run.

Every rank takes its contiguous shard of a BASELINE workload (picotls_amd.dist.shard_for_rank, balanced by bytes for
mixed lengths), seals it with the HIP engine on its device (cuda:LOCAL_RANK, or cuda:0 for every rank with
PTLS_BENCH_ONE_DEVICE=1 on a one-GPU box), opens it again, and writes its sealed arena to <out>/rank<r>.npy; the
barrier + max/sum reductions of bench.py's timing run over the process group (gloo here). The parent test concatenates
the shards and compares them with lib/fusion.c on the whole batch.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", required=True)
    p.add_argument("--records", type=int, required=True)
    p.add_argument("--out", required=True)
    a = p.parse_args()

    import torch

    import picotls_amd as pa
    from picotls_amd.dist import RankContext, aggregate_throughput, shard_for_rank, shard_weights
    from picotls_amd.workloads import WORKLOADS, payload_np

    one_device = os.environ.get("PTLS_BENCH_ONE_DEVICE") == "1"
    local = 0 if one_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    R = RankContext.from_env("gloo" if one_device else "nccl", device=dev)
    wl = WORKLOADS[a.workload].scaled(a.records)
    weights = None if wl.rec_len is not None else shard_weights(wl.lens(0, wl.nrecs))
    begin, end = shard_for_rank(wl.nrecs, R.rank, R.world, weights)
    g = wl.descriptors(0, wl.nrecs)  # the global layout: this shard's arenas are slices of it
    b = wl.descriptors(begin, end)
    p0 = int(g.seal["in_off"][begin]) if end > begin else 0
    keys, ivs = wl.keys()
    ks = pa.Keyset(keys, ivs, wl.key_size)
    pt = payload_np(wl.seed, p0, b.pt_bytes).copy()
    pad = np.ones(b.pt_bytes, bool)  # slot padding is zero (the opened arena only gets record bytes)
    for o, ln in zip(b.seal["in_off"], b.seal["len"]):
        pad[int(o):int(o) + int(ln)] = False
    pt[pad] = 0
    d_seal = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    d_pt = torch.from_numpy(pt).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, begin)).to(dev)
    d_sealed = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device=dev)
    d_back = torch.zeros(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(max(b.n, 1), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    torch.cuda.synchronize(dev)
    R.barrier()
    t0 = time.perf_counter()
    pa.seal_batch(ks, d_seal.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), s)
    pa.open_batch(ks, d_open.data_ptr(), b.n, d_sealed.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    torch.cuda.synchronize(dev)
    R.barrier()
    wall = time.perf_counter() - t0
    value, maxwall = aggregate_throughput(R, b.payload_bytes, wall, 1)
    ok = bool(d_ok[:b.n].min().item() == 1) if b.n else True
    roundtrip = bool(torch.equal(d_back, d_pt))
    np.save(os.path.join(a.out, f"rank{R.rank}.npy"), d_sealed.cpu().numpy())
    with open(os.path.join(a.out, f"rank{R.rank}.json"), "w") as f:
        json.dump({"rank": R.rank, "world": R.world, "begin": begin, "end": end, "ok": ok, "roundtrip": roundtrip,
                   "value": value, "maxwall": maxwall, "wall": wall, "bytes": b.payload_bytes}, f)
    ks.free()
    R.close()


if __name__ == "__main__":
    main()
