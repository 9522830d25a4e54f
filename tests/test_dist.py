"""World-size-2 gloo runs of the multi-GPU plumbing (CPU only; the GPU box runs the same code over RCCL).

Each rank seals its contiguous shard of one global batch independently -- here with the CPU oracle standing in for the
per-GPU engine launch -- and the shards together must reproduce the single-process result bit for bit; the throughput
aggregation must be sum(bytes) / max(wall)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, workload, nrecs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import GcmOracle
    from picotls_amd.dist import RankContext, aggregate_throughput, shard_for_rank, shard_weights
    from picotls_amd.workloads import WORKLOADS, payload_np

    ctx = RankContext.from_env("gloo")
    wl = WORKLOADS[workload].scaled(nrecs)
    weights = None if wl.rec_len is not None else shard_weights(wl.lens(0, wl.nrecs))
    begin, end = shard_for_rank(wl.nrecs, ctx.rank, ctx.world, weights)
    b = wl.descriptors(begin, end)
    keys, ivs = wl.keys()
    # the shard's plaintext is the slice of the global stream: offsets of the global layout
    gb = wl.descriptors(0, wl.nrecs)
    pt_global = payload_np(wl.seed, 0, gb.pt_bytes)
    pt = np.zeros(max(b.pt_bytes, 1), np.uint8)
    for i in range(b.n):
        go = int(gb.seal["in_off"][begin + i])
        ln = int(b.seal["len"][i])
        pt[int(b.seal["in_off"][i]):int(b.seal["in_off"][i]) + ln] = pt_global[go:go + ln]
    aad_g = wl.aad_arena(gb, 0)
    aad = np.zeros(max(b.aad_bytes, 1), np.uint8)
    for i in range(b.n):
        go, al = int(gb.seal["aad_off"][begin + i]), int(b.seal["aad_len"][i])
        aad[int(b.seal["aad_off"][i]):int(b.seal["aad_off"][i]) + al] = aad_g[go:go + al]
    out = np.zeros(max(b.sealed_bytes, 1), np.uint8)
    GcmOracle().seal_batch(keys, ivs, wl.key_size, b.seal, pt, aad, out)
    sealed_records = [bytes(out[int(o):int(o) + int(ln) + 16]) for o, ln in zip(b.seal["out_off"], b.seal["len"])]
    ctx.barrier()
    # fake per-rank timings: rank r took (r + 1) seconds
    value, wall = aggregate_throughput(ctx, b.payload_bytes, float(ctx.rank + 1), 1)
    gathered = [None] * ctx.world
    ctx.dist.all_gather_object(gathered, (begin, end, sealed_records, b.payload_bytes))
    ranges = ctx.gather([begin, end])  # what bench.py reports as "shards"
    if ctx.rank == 0:
        q.put((gathered, value, wall, ranges))
    ctx.close()


def _ranges_worker(rank, world, port, nrecs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from picotls_amd.dist import RankContext, shard_for_rank

    ctx = RankContext.from_env("gloo")
    begin, end = shard_for_rank(nrecs, ctx.rank, ctx.world)
    ranges = ctx.gather([begin, end])
    total = ctx.sum(float(end - begin))
    if ctx.rank == 0:
        q.put((ranges, total))
    ctx.close()


@pytest.mark.parametrize("workload,nrecs", [("shard1200", 97), ("mixed", 41)])
def test_two_rank_shards_reproduce_single_process(workload, nrecs):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import GcmOracle
    from picotls_amd.workloads import WORKLOADS, payload_np

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, workload, nrecs, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, value, wall, ranges = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # shards are disjoint, ordered and cover the batch
    assert gathered[0][0] == 0 and gathered[0][1] == gathered[1][0] and gathered[1][1] == nrecs
    assert [[int(a), int(z)] for a, z in ranges] == [[g[0], g[1]] for g in gathered]
    # bit-identical to the single-process batch
    wl = WORKLOADS[workload].scaled(nrecs)
    gb = wl.descriptors(0, nrecs)
    keys, ivs = wl.keys()
    pt = payload_np(wl.seed, 0, gb.pt_bytes).copy()
    out = np.zeros(gb.sealed_bytes, np.uint8)
    GcmOracle().seal_batch(keys, ivs, wl.key_size, gb.seal, pt, wl.aad_arena(gb, 0), out)
    single = [bytes(out[int(o):int(o) + int(ln) + 16]) for o, ln in zip(gb.seal["out_off"], gb.seal["len"])]
    assert gathered[0][2] + gathered[1][2] == single
    # throughput = 2 * sum(bytes) / max(wall) (the slowest rank took 2 s)
    total = gathered[0][3] + gathered[1][3]
    assert wall == 2.0
    assert value == pytest.approx(2 * total / 2.0 / 2**30)


def test_eight_rank_shards_cover_configs4_once():
    """configs[4]'s record index space (here 32M / 2^10 records) over eight gloo ranks: contiguous shards, each index
    exactly once, gathered on rank 0 as bench.py reports them (the 8-GPU line's "shards")."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    nrecs = (32 << 20) >> 10
    procs = [ctx.Process(target=_ranges_worker, args=(r, 8, port, nrecs, q)) for r in range(8)]
    for p in procs:
        p.start()
    ranges, total = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranges = [[int(a), int(z)] for a, z in ranges]
    assert ranges[0][0] == 0 and ranges[-1][1] == nrecs and total == nrecs
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(7))
