#!/usr/bin/env python3
"""AES-GCM seal+open throughput of the MI355X record engine (BASELINE.json metric), device-resident.

    python bench.py [--gpus N --steps K --warmup W] [--workload tls16k]
                    [--extra quic1200,mixed,mixedrand,shard1200,ptlsbench,quic64k,tls64k] [--no-cpu-baseline] [--no-e2e]

One step = seal the whole batch, then open the sealed batch again (one launch each), inputs already in HBM.
value = (sum L sealed + sum L opened) over all ranks / max-over-ranks wall time of the K timed steps, in GiB/s
(2^30 bytes). Multi-GPU: one process per GPU. Under torch.distributed.run (the driver's N > 1 form) every rank is one
of its processes; `python bench.py --gpus N` on its own starts torch.distributed.run with N ranks as a child process
and relays rank 0's line. The headline workload is weak scaling (every rank seals/opens its own full batch); the
shard1200 leg (configs[4]: 32M x 1200 B split across the ranks) is strong scaling. Independent record shards, no
collective on the data path; a barrier + max/sum reductions of the timings only.

Also reported:
  roofline      dominant kernel (seal), algorithmic bytes per launch / average launch time (HIP events on the
                launch stream) against the 8 TB/s HBM peak of MI355X; traffic (PMC) from profiles/ when committed
  cpu_baseline  picotls' own lib/fusion.c (oracle/_ref, compiled from the reference) sealing+opening a bounded sample
                of each workload on this host's cores (rank 0, N=1 only): ptls_fusion_aes{128,256}gcm (the ptlsbench
                path, primary) and ptls_non_temporal_aes128gcm (the TLS path, secondary), median of reps with the
                spread; t/ptlsbench.c's own loop for configs[0]. The same leg checks records sampled from every GPU leg
                bit for bit against fusion (verified.fusion_spot_check).
  e2e_host_buffers  (N = 1) the headline records starting and ending in pinned host memory (north_star): serial,
                pipelined and in-place (kernels on the device-mapped host arenas) seal+open rates beside the PCIe link's
                own rate (both directions busy); never `value`
  extra         the other BASELINE configs at full size: quic1200 (configs[2]), mixed / mixedrand (configs[3], keys
                grouped by connection / in random order as SURVEY §8(d) writes it), ptlsbench (configs[0]: 1000-record
                batches under t/ptlsbench.c's conventions, on the GPU; fusion beside it in cpu_baseline), and two
                many-connection shapes: quic64k (4M x 1200 B over 64K connections, the
                multi-key runs of round 6) and tls64k (1M x 16 KiB over 64K connections)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s spec)
METRIC = "AES-GCM seal+open GiB/s (device-resident), 16KiB & 1200B record batches"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="tls16k")
    p.add_argument("--extra", default="quic1200,mixed,mixedrand,shard1200,ptlsbench,quic64k,tls64k",
                   help="comma list of extra workloads to report ('' for none)")
    p.add_argument("--records", type=int, default=0, help="override record count (smaller runs)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=3.0, help="wall budget of each cpu_baseline leg")
    p.add_argument("--e2e", dest="e2e", action="store_true", default=None,
                   help="time records that start and end in pinned host memory (DESIGN.md); default: on for N = 1")
    p.add_argument("--no-e2e", dest="e2e", action="store_false")
    p.add_argument("--e2e-chunks", type=int, default=256,
                   help="--e2e: chunks of the pipelined mode (16 MiB at the default 4 GiB: 34.4 GiB/s vs 31.6-31.8 with 64-16)")
    p.add_argument("--schedule", default="auto", choices=["auto", "lockstep", "chunked"],
                   help="batch schedule (ptls_mi355x_keyset_set_schedule)")
    p.add_argument("--verify", type=int, default=1, help="verify round trip + fusion spot checks after timing")
    return p.parse_args()


def self_launch(gpus: int):
    """`bench.py --gpus N` (N > 1) outside torch.distributed.run: start the N ranks as ONE child process
    (`python -m torch.distributed.run --nproc-per-node N bench.py <same args>`, rendezvous on 127.0.0.1), relay rank 0's
    JSON line as this process's last stdout line and return the child's exit code. Called before anything touches the
    GPU (this process never initialises HIP; the ranks do, in their own processes). None when there is nothing to
    launch (N = 1, or already a rank)."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    line = None
    with subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env) as p:
        for out in p.stdout:  # progress and warnings pass through on stderr; the result line is printed last
            if out.startswith("{") and '"metric"' in out:
                line = out
            else:
                sys.stderr.write(out)
        rc = p.wait()
    if line is not None:
        sys.stdout.write(line)
        sys.stdout.flush()
    return rc if line is not None or rc != 0 else 1


def make_rank(gpus: int):
    import torch

    from picotls_amd.dist import RankContext

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if gpus > 1 and world != gpus:
        raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}: one rank per GPU")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a one-GPU box: every rank on cuda:0, gloo for the barrier/reductions
    one_device = os.environ.get("PTLS_BENCH_ONE_DEVICE") == "1"
    if one_device:
        local = 0
    torch.cuda.set_device(local)
    # PTLS_BENCH_PROCESS_GROUP=1: join the process group even as the only rank (exercises the nccl branch on one GPU)
    return RankContext.from_env("gloo" if one_device else "nccl", device=torch.device("cuda", local),
                                always=os.environ.get("PTLS_BENCH_PROCESS_GROUP") == "1")


def run_workload(R, wl, steps: int, warmup: int, verify: int, shard_global: bool, schedule: str = "auto"):
    import torch
    import picotls_amd as pa
    from picotls_amd.records import algorithmic_bytes
    from picotls_amd.workloads import payload_torch

    from picotls_amd.dist import shard_for_rank, shard_weights

    if shard_global:  # strong scaling: the global batch is split across ranks (by bytes for mixed lengths)
        weights = None if wl.rec_len is not None else shard_weights(wl.lens(0, wl.nrecs))
        begin, end = shard_for_rank(wl.nrecs, R.rank, R.world, weights)
    else:  # weak scaling: every rank processes a full batch (its own records)
        begin, end = 0, wl.nrecs
    b = wl.descriptors(begin, end)
    keys, ivs = wl.keys()
    ks = pa.Keyset(keys, ivs, wl.key_size)
    ks.set_schedule(schedule, allow_variable_time=True)
    dev = R.device
    d_seal = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, begin)).to(dev)
    d_pt = payload_torch(wl.seed + 7919 * (R.rank if not shard_global else 0), b.pt_bytes, dev)
    zero_slot_padding(d_pt, b.seal, dev)  # so the round-trip check can compare whole arenas
    d_sealed = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    d_back = torch.zeros(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def seal():
        pa.seal_batch(ks, d_seal.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), sp)

    def open_():
        pa.open_batch(ks, d_open.data_ptr(), b.n, d_sealed.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(),
                      d_ok.data_ptr(), sp)

    for _ in range(warmup):
        seal()
        open_()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    clk = torch.zeros(8, dtype=torch.int64, device=dev)  # two (s_memtime, s_memrealtime, XCD) samples of XCD 0
    kcap = 4 * steps + 8  # in-kernel samples: workgroup 0 of each chunked launch (a W8 pair is two launches)
    kclk = torch.zeros(4 * kcap, dtype=torch.int64, device=dev)
    pa.debug_kernel_clock(kclk.data_ptr(), kcap)
    torch.cuda.synchronize(dev)
    R.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k, (e0, e1, e2) in enumerate(ev):
        e0.record(stream)
        seal()
        e1.record(stream)
        open_()
        e2.record(stream)
        if k == 0 or k == len(ev) - 1:  # (~20 us each, in a leg of ~0.1-1 s)
            pa.debug_clock_sample(clk.data_ptr() + (32 if k else 0), sp)
    torch.cuda.synchronize(dev)
    R.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    seal_ms = float(np.mean([a.elapsed_time(bb) for a, bb, _ in ev]))
    open_ms = float(np.mean([bb.elapsed_time(c) for _, bb, c in ev]))
    nk = min(pa.debug_kernel_clock_count(), kcap)
    pa.debug_kernel_clock(0, 0)

    res = {"records": b.n, "payload_bytes": b.payload_bytes, "wall_s": wall, "seal_ms": seal_ms, "open_ms": open_ms,
           "shard": [begin, end], "clock": shader_clock(clk.cpu().numpy(), kclk[:4 * nk].cpu().numpy())}
    res["sclk_mhz"] = res["clock"]["sclk_mhz"]
    lens = b.seal["len"]
    res["seal_alg_bytes"] = algorithmic_bytes(lens, b.seal["aad_len"], True)
    res["open_alg_bytes"] = algorithmic_bytes(lens, b.seal["aad_len"], False)
    # GHASH stream positions the seal kernel walks (8 lanes x steps per record, padding included): the LDS model's unit
    na = (b.seal["aad_len"].astype(np.int64) + 15) // 16
    nb = (lens.astype(np.int64) + 15) // 16
    res["stream_blocks"] = int((((na + nb + 1 + 7) // 8) * 8).sum())

    if verify:
        ok_all = bool(d_ok.min().item() == 1) if b.n else True
        same = bool(torch.equal(d_back, d_pt))
        res["verified_roundtrip"] = R.sum(float(ok_all and same)) == R.world  # every rank's shard round-trips
        # records for the bit-exact fusion check, which runs in the cpu_baseline leg (rank 0)
        res["sample"] = collect_sample(wl, b, keys, ivs, d_pt, d_aad, d_sealed, d_back, d_ok) if R.rank == 0 else None
    del d_pt, d_sealed, d_back, d_ok, d_seal, d_open, d_aad
    ks.free()
    torch.cuda.empty_cache()
    return res


def shader_clock(c, k=None) -> dict:
    """The shader clock over a timed leg. sclk_mhz: inside the kernels (ptls_mi355x_debug_kernel_clock: workgroup 0 of
    every chunked launch reads s_memtime and s_memrealtime at its start and end; cycles over real-time ticks, weighted by
    duration), the clock the chip holds under the load. after_*_mhz: a one-wave probe right after the leg's first and
    last steps (ptls_mi355x_debug_clock_sample: s_memtime over a ~20 us spin), the clock once the load has stopped, which
    runs higher under a power limit."""
    import picotls_amd as pa

    khz = pa.debug_wallclock_khz()
    mhz = [round(int(c[i]) / (int(c[i + 1]) / (khz * 1e3)) / 1e6, 1) if khz > 0 and int(c[i + 1]) > 0 else None for i in (0, 4)]
    ok = [m for m in mhz if m is not None]
    inside, launches = None, 0
    if k is not None and len(k) >= 4 and khz > 0:
        s = np.asarray(k, dtype=np.int64).reshape(-1, 4)
        cyc, ticks = (s[:, 1] - s[:, 0]).astype(np.float64), (s[:, 3] - s[:, 2]).astype(np.float64)
        keep = (ticks > 0) & (cyc > 0)
        launches = int(keep.sum())
        if launches:
            inside = round(float(cyc[keep].sum() / (ticks[keep].sum() / (khz * 1e3)) / 1e6), 1)
    return {"sclk_mhz": inside if inside is not None else (round(sum(ok) / len(ok), 1) if ok else None),
            "in_kernel_mhz": inside, "in_kernel_launches": launches,
            "after_probe_mhz": round(sum(ok) / len(ok), 1) if ok else None, "after_first_step_mhz": mhz[0],
            "after_last_step_mhz": mhz[1], "xcd": [int(c[2]), int(c[6])], "rtc_khz": khz}


def zero_slot_padding(arena, recs, dev):
    """Zeroes the bytes between the end of each record and the next 16-byte slot boundary."""
    import torch

    lens = recs["len"].astype(np.int64)
    pad = (-lens) % 16
    if not pad.any():
        return
    starts = torch.from_numpy(recs["in_off"].astype(np.int64) + lens).to(dev)
    padt = torch.from_numpy(pad).to(dev)
    for p in range(15):
        sel = starts[padt > p] + p
        arena[sel] = 0


def collect_sample(wl, b, keys, ivs, d_pt, d_aad, d_sealed, d_back, d_ok, nsample: int = 64):
    """Host copies of nsample records (inputs, the GPU's sealed output, and what the timed open of the full-size batch
    wrote for them: plaintext and ok byte), repacked as a small batch, for the bit-exact comparison with lib/fusion.c
    in the cpu_baseline leg."""
    rng = np.random.default_rng(99)
    idx = np.unique(np.concatenate([[0, b.n - 1], rng.integers(0, b.n, nsample)]))
    sub = b.seal[idx].copy()
    pt_parts, aad_parts, gpu_parts, back_parts, new_in, new_aad = [], [], [], [], [], []
    off = aoff = 0
    for r in sub:
        ln, al = int(r["len"]), int(r["aad_len"])
        pt_parts.append(d_pt[int(r["in_off"]):int(r["in_off"]) + ln].cpu().numpy())
        pt_parts.append(np.zeros(16, np.uint8))  # room for the tag (sealed in place)
        aad_parts.append(d_aad[int(r["aad_off"]):int(r["aad_off"]) + al].cpu().numpy())
        gpu_parts.append(d_sealed[int(r["out_off"]):int(r["out_off"]) + ln + 16].cpu().numpy())
        back_parts.append(d_back[int(r["in_off"]):int(r["in_off"]) + ln].cpu().numpy())  # (the open writes at the seal's in_off)
        new_in.append(off)
        new_aad.append(aoff)
        off += ln + 16
        aoff += al
    recs = sub.copy()
    recs["in_off"] = new_in
    recs["out_off"] = new_in
    recs["aad_off"] = new_aad
    return {"key_size": wl.key_size, "keys": keys, "ivs": ivs, "recs": recs,
            "pt": np.concatenate(pt_parts + [np.zeros(1, np.uint8)]),
            "aad": np.concatenate(aad_parts + [np.zeros(1, np.uint8)]), "gpu": np.concatenate(gpu_parts),
            "gpu_back": np.concatenate(back_parts + [np.zeros(1, np.uint8)]), "gpu_ok": d_ok[torch_index(idx)].cpu().numpy()}


def torch_index(idx):
    import torch

    return torch.from_numpy(np.asarray(idx, np.int64))


def check_sample(ref, sample) -> tuple[bool, bool]:
    """lib/fusion.c (ptls_aead_encrypt per record) on the sampled inputs, compared with the GPU's sealed records; and
    fusion opening the GPU's sealed records (ptls_aead_decrypt), compared with the plaintext and ok bytes the GPU's
    full-size open wrote for them."""
    out = np.zeros(len(sample["pt"]), np.uint8)
    ref.run_batch(True, sample["keys"], sample["ivs"], sample["key_size"], sample["recs"], sample["pt"], sample["aad"], out,
                  nthreads=1)
    fus = np.concatenate([out[int(r["out_off"]):int(r["out_off"]) + int(r["len"]) + 16] for r in sample["recs"]])
    seal_ok = bool(np.array_equal(fus, sample["gpu"]))
    # fusion opens the GPU's ciphertext || tag (repacked at the same offsets) into its own plaintext arena
    gpu_sealed = np.zeros(len(sample["pt"]), np.uint8)
    back = np.zeros(len(sample["pt"]), np.uint8)
    pos = 0
    for r in sample["recs"]:
        ln = int(r["len"])
        gpu_sealed[int(r["in_off"]):int(r["in_off"]) + ln + 16] = sample["gpu"][pos:pos + ln + 16]
        pos += ln + 16
    ok = np.zeros(len(sample["recs"]), np.uint8)
    ref.run_batch(False, sample["keys"], sample["ivs"], sample["key_size"], sample["recs"], gpu_sealed, sample["aad"], back,
                  ok=ok, nthreads=1)
    ref_back = np.concatenate([back[int(r["in_off"]):int(r["in_off"]) + int(r["len"])] for r in sample["recs"]] +
                              [np.zeros(1, np.uint8)])
    open_ok = bool(np.array_equal(ok, sample["gpu_ok"]) and np.array_equal(ref_back, sample["gpu_back"]) and ok.all())
    return seal_ok, open_ok


def run_ptlsbench(R, steps: int, warmup: int, rec_len: int = 16384):
    """configs[0] on the GPU: ptlsbench's 1000-record batch (picotls_amd.workloads.ptlsbench_batch: HKDF key from
    32 x 'z', AAD h[4] with h[0] = seq, zero plaintext) sealed and opened as one launch each, repeatedly. The
    launch-bound small-batch shape of picotls' own benchmark; fusion runs the same records in cpu_baseline."""
    import torch
    import picotls_amd as pa
    from picotls_amd.workloads import ptlsbench_batch

    b, key, iv, aad = ptlsbench_batch(rec_len=rec_len)
    ks = pa.Keyset(key, iv, 16)
    dev = R.device
    d_seal = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(aad).to(dev)
    d_pt = torch.zeros(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_sealed = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    d_back = torch.ones(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    reps = max(steps, 1) * 20  # a batch is 16 MiB: 20 batches per step

    def step():
        pa.seal_batch(ks, d_seal.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), sp)
        pa.open_batch(ks, d_open.data_ptr(), b.n, d_sealed.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(),
                      d_ok.data_ptr(), sp)

    for _ in range(max(warmup, 1) * 20):
        step()
    torch.cuda.synchronize(dev)
    R.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize(dev)
    R.barrier()
    wall = time.perf_counter() - t0
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    seal_ms = open_ms = 0.0
    for _ in range(10):
        e[0].record(stream)
        pa.seal_batch(ks, d_seal.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), sp)
        e[1].record(stream)
        pa.open_batch(ks, d_open.data_ptr(), b.n, d_sealed.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), sp)
        e[2].record(stream)
        torch.cuda.synchronize(dev)
        seal_ms += e[0].elapsed_time(e[1]) / 10
        open_ms += e[1].elapsed_time(e[2]) / 10
    res = {"records_per_batch": b.n, "record_len": rec_len, "batches": reps, "payload_bytes": b.payload_bytes,
           "wall_s": wall, "seal_ms_per_batch": round(seal_ms, 4), "open_ms_per_batch": round(open_ms, 4),
           "verified_roundtrip": bool(d_ok.min().item() == 1) and not bool(d_back.any().item())}
    # every sealed record of the batch goes to the bit-exact check against fusion's ptlsbench run (cpu_baseline)
    res["gpu_sealed"] = d_sealed.cpu().numpy() if R.rank == 0 else None
    ks.free()
    return res


def _cpu_share():
    """The cores this process may use (the box grants a CPU share smaller than the visible CPU set; OMP_NUM_THREADS /
    nproc report it)."""
    cpus = sorted(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(cpus)
    try:
        import subprocess

        share = min(share, int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip() or share))
    except Exception:
        pass
    return cpus[:max(1, min(share, len(cpus)))]


def cpu_topology(cpus) -> dict:
    """Physical cores behind the logical CPUs used (sysfs core_id / physical_package_id): how many distinct cores, and
    how many of the CPUs are SMT siblings of another CPU in the set."""
    cores = {}
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            key = (open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip())
        except OSError:
            return {"physical_cores": None, "smt_siblings_in_set": None, "logical_cpus": len(cpus)}
        cores.setdefault(key, []).append(c)
    return {"physical_cores": len(cores), "smt_siblings_in_set": len(cpus) - len(cores), "logical_cpus": len(cpus)}


def _fusion_leg(ref, wl, cpus, seconds: float, nontemporal: bool = False, sample_bytes: int = 256 << 20,
                max_reps: int = 200):
    """fusion sealing then opening a bounded sample of the workload with len(cpus) pinned threads (contiguous shards,
    CLOCK_MONOTONIC between a start barrier and the last thread's end), repeated for `seconds` (at most max_reps reps):
    the quartiles of the per-rep seal+open rate (value = median). The box's CPU share is not isolated, so a multi-thread
    leg's reps spread widely; the quartiles say how far (iqr_rel = (p75 - p25) / p50)."""
    from picotls_amd.workloads import payload_np

    n = min(wl.nrecs, max(1, sample_bytes // (wl.rec_len or 8192)))
    b = wl.descriptors(0, n)
    keys, ivs = wl.keys()
    pt = payload_np(wl.seed, 0, b.pt_bytes).copy()
    aad = wl.aad_arena(b, 0)
    sealed = np.ones(b.sealed_bytes, np.uint8)  # touched: no first-touch page faults inside a timed rep
    back = np.ones(b.pt_bytes, np.uint8)
    ok = np.zeros(b.n, np.uint8)
    rates, srates, orates = [], [], []
    for _ in range(2):  # warm-up reps (caches, clocks), not counted
        ref.run_batch(True, keys, ivs, wl.key_size, b.seal, pt, aad, sealed, nthreads=len(cpus), cpus=cpus, nontemporal=nontemporal)
    start = time.perf_counter()
    while len(rates) < 5 or (time.perf_counter() - start < seconds and len(rates) < max_reps):
        ts, _ = ref.run_batch(True, keys, ivs, wl.key_size, b.seal, pt, aad, sealed, nthreads=len(cpus), cpus=cpus,
                              nontemporal=nontemporal)
        to, fails = ref.run_batch(False, keys, ivs, wl.key_size, b.open, sealed, aad, back, ok=ok, nthreads=len(cpus),
                                  cpus=cpus, nontemporal=nontemporal)
        assert fails == 0
        gib = b.payload_bytes / 2**30
        rates.append(2 * gib / (ts + to))
        srates.append(gib / ts)
        orates.append(gib / to)
    algo = ("ptls_non_temporal_aes" if nontemporal else "ptls_fusion_aes") + f"{8 * wl.key_size}gcm"
    p25, p50, p75 = (float(np.percentile(rates, q)) for q in (25, 50, 75))
    return {"value": round(p50, 3), "min": round(min(rates), 3), "max": round(max(rates), 3),
            "p25": round(p25, 3), "p75": round(p75, 3), "iqr_rel": round((p75 - p25) / p50, 3) if p50 else None,
            "reps": len(rates), "seal_GiBps": round(float(np.median(srates)), 3),
            "open_GiBps": round(float(np.median(orates)), 3), "threads": len(cpus),
            "sample": f"{b.n} x {wl.rec_len or 'U[64,16384]'} B records of '{wl.name}' ({b.payload_bytes / 2**20:.0f} MiB), "
                      f"{algo} via ptls_aead_encrypt/decrypt"}


def cpu_baseline(wl, seconds: float, samples: dict, ptlsbench_gpu):
    """lib/fusion.c (the reference, compiled from /root/reference into oracle/_ref) on this host's cores, and the
    bit-exact checks of the GPU legs' sampled records against it."""
    try:
        from oracle import FusionRef, PtlsBenchRef

        ref = FusionRef()
    except Exception as e:
        return {"value": None, "unit": "GiB/s", "cores": 0, "kind": "reference", "sample": f"unavailable: {e}"}, {}
    from picotls_amd.workloads import WORKLOADS

    both = {name: check_sample(ref, smp) for name, smp in samples.items() if smp is not None}
    checks = {name: v[0] for name, v in both.items()}
    checks.update({name + ":open": v[1] for name, v in both.items()})
    cpus = _cpu_share()
    legs = {}
    primary = _fusion_leg(ref, wl, cpus, seconds)
    legs[wl.name] = {"fusion": primary}
    if wl.name == "tls16k":  # the TLS path (SURVEY §8(d) secondary baseline)
        legs[wl.name]["non_temporal"] = _fusion_leg(ref, wl, cpus, seconds, nontemporal=True)
    legs[wl.name]["fusion_1_thread"] = _fusion_leg(ref, wl, cpus[:1], seconds, sample_bytes=64 << 20)
    for name in ("quic1200", "mixed"):
        if name != wl.name:
            legs[name] = {"fusion": _fusion_leg(ref, WORKLOADS[name], cpus, seconds)}
    # configs[0]: t/ptlsbench.c's own loop (one thread, its CPU clock), 20 batches of 1000 x 16384 B
    try:
        pb = PtlsBenchRef()
        first = np.zeros(pb.BATCH * (16384 + 16), np.uint8)
        t = pb.run(20 * pb.BATCH, 16384, 16, first)
        gib = 20 * pb.BATCH * 16384 / 2**30
        legs["ptlsbench"] = {"fusion": {
            "value": round(2 * gib / (t["seal_cpu_s"] + t["open_cpu_s"]), 3), "seal_GiBps": round(gib / t["seal_cpu_s"], 3),
            "open_GiBps": round(gib / t["open_cpu_s"], 3),
            "seal_mbps": round(gib * 2**30 * 8 / (t["seal_cpu_s"] * 1e6), 1),
            "open_mbps": round(gib * 2**30 * 8 / (t["open_cpu_s"] * 1e6), 1), "threads": 1,
            "sample": "t/ptlsbench.c bench_run_one: 20 batches of 1000 x 16384 B, ptls_aead_new(ptls_fusion_aes128gcm, "
                      "sha256, 32 x 'z'), AAD h[4], zero plaintext; CPU time of the thread (ptlsbench's clock)"}}
        if ptlsbench_gpu is not None:
            checks["ptlsbench"] = bool(np.array_equal(ptlsbench_gpu, first))
    except Exception as e:
        legs["ptlsbench"] = {"fusion": {"value": None, "sample": f"unavailable: {e}"}}
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    one = legs[wl.name]["fusion_1_thread"]["value"]
    topo = cpu_topology(cpus)
    out = {"value": primary["value"], "unit": "GiB/s", "cores": len(cpus), "kind": "reference",
           "physical_cores": topo["physical_cores"], "smt_siblings_in_set": topo["smt_siblings_in_set"],
           "cpus": cpus,
           "sample": primary["sample"] + f", {len(cpus)} pinned threads, CLOCK_MONOTONIC, median of {primary['reps']} reps "
                                         f"(p25 {primary['p25']}, p75 {primary['p75']}, min {primary['min']}, max "
                                         f"{primary['max']}); CPU: {model}; {topo['physical_cores']} physical cores "
                                         f"({topo['smt_siblings_in_set']} of the threads on SMT siblings)",
           "p25": primary["p25"], "p75": primary["p75"], "iqr_rel": primary["iqr_rel"],
           "seal_GiBps": primary["seal_GiBps"], "open_GiBps": primary["open_GiBps"],
           "single_thread_GiBps": one,
           # the stable reference point: one core's rate (spread ~1-2 %) times the cores used, i.e. perfect scaling,
           # which the 16-thread median (a shared, noisy CPU share) never exceeds
           "single_thread_x_cores_GiBps": round(one * len(cpus), 3) if one else None,
           "legs": legs}
    return out, checks


def run_e2e(R, wl, nchunks: int = 16, reps: int = 3, schedule: str = "auto"):
    """Records that start and end in host memory (socket / NIC buffers): pinned host -> H2D -> seal -> D2H, then
    the sealed records back through H2D -> open -> D2H. Serial (one stream), pipelined (chunks over three streams, so
    copies in both directions overlap the kernels) and in place (the kernels read and write the pinned host arenas
    over PCIe, one launch per direction). Payload GiB/s per direction (seal+open averaged)."""
    import torch
    import picotls_amd as pa

    b = wl.descriptors(0, wl.nrecs)
    keys, ivs = wl.keys()
    ks = pa.Keyset(keys, ivs, wl.key_size)
    ks.set_schedule(schedule, allow_variable_time=True)
    dev = R.device
    from picotls_amd.workloads import payload_np

    h_pt = torch.from_numpy(payload_np(wl.seed, 0, b.pt_bytes).copy()).pin_memory()
    h_sealed = torch.empty(b.sealed_bytes, dtype=torch.uint8).pin_memory()
    h_back = torch.empty(b.pt_bytes, dtype=torch.uint8).pin_memory()
    d_aad = torch.from_numpy(wl.aad_arena(b, 0)).to(dev)
    d_pt = torch.empty(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_sealed = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    d_back = torch.empty(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.empty(b.n, dtype=torch.uint8, device=dev)
    # chunk c covers records [r0, r1): contiguous byte ranges in every arena; descriptors are rebased per chunk
    bounds = np.linspace(0, b.n, nchunks + 1).astype(np.int64)
    chunks = []
    for c in range(nchunks):
        r0, r1 = int(bounds[c]), int(bounds[c + 1])
        if r1 <= r0:
            continue
        seal = b.seal[r0:r1].copy()
        opn = b.open[r0:r1].copy()
        p0, s0 = int(b.seal["in_off"][r0]), int(b.seal["out_off"][r0])
        p1 = int(b.seal["in_off"][r1 - 1]) + (int(b.seal["len"][r1 - 1]) + 15) // 16 * 16
        s1 = int(b.seal["out_off"][r1 - 1]) + (int(b.seal["len"][r1 - 1]) + 31) // 16 * 16
        seal["in_off"] -= p0
        seal["out_off"] -= s0
        opn["in_off"] -= s0
        opn["out_off"] -= p0
        chunks.append((r0, r1, p0, p1, s0, s1, torch.from_numpy(seal.view(np.uint8).copy()).to(dev),
                       torch.from_numpy(opn.view(np.uint8).copy()).to(dev)))
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    m = np.zeros(b.pt_bytes, bool)  # the arena bytes that are record payload
    for o, ln in zip(b.seal["in_off"], b.seal["len"]):
        m[int(o):int(o) + int(ln)] = True

    def one_pass(pipelined: bool):
        for i, (r0, r1, p0, p1, s0, s1, ds, do) in enumerate(chunks):
            st = streams[i % 3] if pipelined else torch.cuda.current_stream(dev)
            with torch.cuda.stream(st):
                d_pt[p0:p1].copy_(h_pt[p0:p1], non_blocking=True)
                pa.seal_batch(ks, ds.data_ptr(), r1 - r0, d_pt.data_ptr() + p0, d_aad.data_ptr(), d_sealed.data_ptr() + s0,
                              st.cuda_stream)
                h_sealed[s0:s1].copy_(d_sealed[s0:s1], non_blocking=True)
        torch.cuda.synchronize(dev)
        t_seal = time.perf_counter()
        for i, (r0, r1, p0, p1, s0, s1, ds, do) in enumerate(chunks):
            st = streams[i % 3] if pipelined else torch.cuda.current_stream(dev)
            with torch.cuda.stream(st):
                d_sealed[s0:s1].copy_(h_sealed[s0:s1], non_blocking=True)
                pa.open_batch(ks, do.data_ptr(), r1 - r0, d_sealed.data_ptr() + s0, d_aad.data_ptr(), d_back.data_ptr() + p0,
                              d_ok.data_ptr() + r0, st.cuda_stream)
                h_back[p0:p1].copy_(d_back[p0:p1], non_blocking=True)
        torch.cuda.synchronize(dev)
        return t_seal

    def in_place_pass():
        # one launch per direction on the pinned host arenas themselves (device-mapped): the kernels read the records
        # and write the results over PCIe, no copy engine involved
        st = torch.cuda.current_stream(dev)
        pa.seal_batch(ks, d_seal_all.data_ptr(), b.n, h_pt.data_ptr(), d_aad.data_ptr(), h_sealed.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        t_seal = time.perf_counter()
        pa.open_batch(ks, d_open_all.data_ptr(), b.n, h_sealed.data_ptr(), d_aad.data_ptr(), h_back.data_ptr(),
                      d_ok.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        return t_seal

    d_seal_all = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_open_all = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    out = {}
    for mode in ("serial", "pipelined", "in_place"):
        run = in_place_pass if mode == "in_place" else (lambda: one_pass(mode == "pipelined"))
        h_back.zero_()
        d_ok.zero_()
        run()
        ts = to = 0.0
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            t_mid = run()
            t1 = time.perf_counter()
            ts += t_mid - t0
            to += t1 - t_mid
        gib = b.payload_bytes * reps / 2**30
        # every mode's round trip is checked: all tags verified, the opened records equal the plaintext
        verified = bool(d_ok.min().item() == 1) and bool(np.array_equal(h_back.numpy()[m], h_pt.numpy()[m]))
        out[mode] = {"seal_GiBps": round(gib / ts, 2), "open_GiBps": round(gib / to, 2),
                     "seal_open_GiBps": round(2 * gib / (ts + to), 2), "verified": verified}
    # the link itself: the same arenas copied H2D and D2H at once on two streams, no kernel (the ceiling of every mode
    # above, where a payload byte crosses once in each direction per seal and once per open)
    s_up, s_down = streams[0], streams[1]
    tl = 0.0
    for _ in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(s_up):
            d_pt.copy_(h_pt, non_blocking=True)
        with torch.cuda.stream(s_down):
            h_back.copy_(d_back, non_blocking=True)
        torch.cuda.synchronize(dev)
        if _ > 0:
            tl += time.perf_counter() - t0
    link = b.pt_bytes * reps / 2**30 / tl
    up_only = []
    for src, dst in ((h_pt, d_pt), (d_back, h_back)):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize(dev)
        up_only.append(b.pt_bytes * reps / 2**30 / (time.perf_counter() - t0))
    out["link"] = {"both_directions_GiBps_each": round(link, 2), "h2d_alone_GiBps": round(up_only[0], 2),
                   "d2h_alone_GiBps": round(up_only[1], 2)}
    out.update({"records": b.n, "payload_bytes": b.payload_bytes, "chunks": len(chunks),
                "verified": all(out[k]["verified"] for k in ("serial", "pipelined", "in_place")),
                "note": "pinned host buffers; PCIe Gen5 x16 ~63 GB/s/direction bounds this path; in_place: the kernels "
                        "read and write the device-mapped host arenas directly"})
    ks.free()
    return out


def per_rank(R, res) -> dict:
    """Every rank's seal / open launch time and wall time of the timed steps (rank order), so that a straggler of a
    multi-GPU run shows; value uses the max of wall_s."""
    rows = R.gather([res["seal_ms"], res["open_ms"], res["wall_s"], res.get("sclk_mhz") or 0.0])
    wall = [r[2] for r in rows]
    slow = int(np.argmax(wall))
    return {"seal_ms": [round(r[0], 4) for r in rows], "open_ms": [round(r[1], 4) for r in rows],
            "wall_s": [round(r[2], 5) for r in rows], "sclk_mhz": [round(r[3], 1) if r[3] else None for r in rows],
            "max_wall_s": round(max(wall), 5), "min_wall_s": round(min(wall), 5), "slowest_rank": slow,
            "max_over_min": round(max(wall) / min(wall), 4) if min(wall) > 0 else None}


W8_MIN_RECS = 256  # picotls_amd/csrc/engine/common.h: batches from this many records take the W8 kernels


def lds_model(res, key_size: int, nrecs: int):
    """The bound the seal kernel actually meets: LDS table lookups. Per GHASH stream block an AES-128
    block costs 133 ds_read_b32 (AES-256: 197) and its GHASH fold 16 ds_read_b128 (the W8 kernels' Horner step on the
    8-bit H^8 table, batches of at least W8_MIN_RECS records) or 32 (4-bit windows); at the MI355X aggregate LDS
    rates (MI355X_MICROARCH.md: ~75 TB/s ds_read_b32, ~150 TB/s ds_read_b128 with every CU at 2.4 GHz) that gives the
    chip's block rate ceiling; frac = achieved blocks/s over it (the clock under this load is lower)."""
    lookups = 133 if key_size == 16 else 197
    ghash = 16 if nrecs >= W8_MIN_RECS else 32
    sec_per_block = lookups * 4 / 75e12 + ghash * 16 / 150e12
    peak = 1.0 / sec_per_block
    achieved = res["stream_blocks"] / (res["seal_ms"] / 1e3)
    out = {"bound": "lds", "unit": "stream blocks/s", "achieved": round(achieved, -6), "peak_at_2.4GHz": round(peak, -6),
           "frac": round(achieved / peak, 4),
           "per_block": f"{lookups} ds_read_b32 (AES) + {ghash} ds_read_b128 (GHASH)"}
    mhz = (res.get("clock") or {}).get("in_kernel_mhz")
    if mhz:  # the same ceiling at the shader clock measured inside the kernels over this leg
        out["sclk_mhz"] = mhz
        out["frac_at_sclk"] = round(achieved / (peak * mhz / 2400.0), 4)
    return out


def traffic_from_profiles(workload: str, records: int, key: str = "seal_hbm_bytes_per_launch"):
    """Corrected HBM bytes per seal (or open: key "open_hbm_bytes_per_launch") launch from the committed rocprofv3 PMC
    summary (profiles/pmc_<workload>.json), scaled to this run's record count when the profile was taken on a different
    one."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        v = d.get(key)
        if v is None:
            return None
        n = d.get("records")
        return round(v * records / n) if n else round(v)
    except Exception:
        return None


def main():
    args = parse()
    rc = self_launch(args.gpus)
    if rc is not None:
        sys.exit(rc)
    from picotls_amd.workloads import WORKLOADS

    from picotls_amd.dist import aggregate_throughput

    R = make_rank(args.gpus)
    wl = WORKLOADS[args.workload]
    if args.records:
        wl = wl.scaled(args.records)
    shard_global = args.workload == "shard1200"
    res = run_workload(R, wl, args.steps, args.warmup, args.verify, shard_global, args.schedule)

    value, wall = aggregate_throughput(R, res["payload_bytes"], res["wall_s"], args.steps)
    seal_s, open_s = res["seal_ms"] / 1e3, res["open_ms"] / 1e3
    achieved = res["seal_alg_bytes"] / seal_s / 1e9
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": R.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if shard_global else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: splitmix64 payload (seed 0x5eed) generated on device; random-key AES-GCM",
        "config": {"workload": wl.name, "desc": wl.desc, "records_per_gpu": res["records"],
                   "shards": [[int(a), int(z)] for a, z in R.gather(res["shard"])] if shard_global else None,
                   "record_len": wl.rec_len or "U[64,16384]", "aad_len": wl.aad_len,
                   "aead": f"AES-{8 * wl.key_size}-GCM", "keys": wl.nkeys,
                   "parallelism": f"{R.world} independent per-GPU record shards, no data-path collective",
                   "dist_backend": R.backend},
        "seal_GiBps": round(res["payload_bytes"] / seal_s / 2**30, 3),
        "open_GiBps": round(res["payload_bytes"] / open_s / 2**30, 3),
        "roofline": {"bound": "hbm", "kernel": f"{'gcm_batch_kernel' if args.schedule == 'lockstep' else 'gcm_chunked_kernel'}"
                                               f"<{10 if wl.key_size == 16 else 14},seal>",
                     # (one seal launch of W8_MIN_RECS records or more is the W8 pair, EXT 4 + EXT 3:
                     # avg_launch_ms covers both, and profiles/pmc_<workload>.json sums their bytes)
                     "launch": "w8 pair" if args.schedule != "lockstep" and res["records"] >= W8_MIN_RECS else "single",
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic_from_profiles(wl.name, res["records"]),
                     "alg_bytes_per_launch": res["seal_alg_bytes"], "avg_launch_ms": round(res["seal_ms"], 4),
                     "open_achieved": round(res["open_alg_bytes"] / open_s / 1e9, 2),
                     "open_alg_bytes_per_launch": res["open_alg_bytes"],
                     "open_traffic": traffic_from_profiles(wl.name, res["records"], "open_hbm_bytes_per_launch")},
        "lds_model": lds_model(res, wl.key_size, res["records"]),
        "verified": {"roundtrip": res.get("verified_roundtrip"), "fusion_spot_check": None, "fusion_open_spot_check": None},
        # XCD 0's average shader clock over the timed steps (rank 0), so that box-to-box spread can be attributed
        "sclk_mhz": res.get("sclk_mhz"), "clock_probe": res.get("clock"),
    }
    if R.world > 1:
        out["per_rank"] = per_rank(R, res)
    samples = {wl.name: res.get("sample")}
    extra = {}
    ptlsbench_gpu = None
    for name in [x for x in args.extra.split(",") if x]:
        if name == args.workload:
            continue
        if name == "ptlsbench":
            r2 = run_ptlsbench(R, args.steps, args.warmup)
            v2, _ = aggregate_throughput(R, r2["payload_bytes"], r2["wall_s"], r2["batches"])
            ptlsbench_gpu = r2.pop("gpu_sealed")
            extra[name] = {"value": round(v2, 3), "unit": "GiB/s", "config": "configs[0]: t/ptlsbench.c conventions "
                           "(HKDF key from 32 x 'z', AAD h[4] with h[0] = seq, zero plaintext), 1000 x 16384 B per launch, "
                           "AES-128-GCM", **{k: r2[k] for k in ("records_per_batch", "batches", "seal_ms_per_batch",
                                                                 "open_ms_per_batch")},
                           "seal_GiBps": round(r2["records_per_batch"] * 16384 / (r2["seal_ms_per_batch"] / 1e3) / 2**30, 3),
                           "open_GiBps": round(r2["records_per_batch"] * 16384 / (r2["open_ms_per_batch"] / 1e3) / 2**30, 3),
                           "verified": {"roundtrip": r2["verified_roundtrip"], "fusion_spot_check": None}}
            continue
        w2 = WORKLOADS[name]
        if args.records:
            w2 = w2.scaled(max(1, args.records * (wl.rec_len or 8192) // (w2.rec_len or 8192)))
        r2 = run_workload(R, w2, args.steps, args.warmup, args.verify, name == "shard1200", args.schedule)
        samples[name] = r2.get("sample")
        v2, _ = aggregate_throughput(R, r2["payload_bytes"], r2["wall_s"], args.steps)
        extra[name] = {"value": round(v2, 3), "unit": "GiB/s", "desc": w2.desc,
                       "scaling": "strong" if name == "shard1200" else "weak", "n_gpus": R.world,
                       "records_total": int(R.sum(float(r2["records"]))),
                       "records_per_gpu": r2["records"], "record_len": w2.rec_len or "U[64,16384]",
                       # every rank's [begin, end) of the global batch (strong scaling: together exactly [0, total))
                       "shards": [[int(a), int(z)] for a, z in R.gather(r2["shard"])] if name == "shard1200" else None,
                       "aead": f"AES-{8 * w2.key_size}-GCM", "keys": w2.nkeys, "key_order": w2.key_order,
                       "seal_GiBps": round(r2["payload_bytes"] / (r2["seal_ms"] / 1e3) / 2**30, 3),
                       "open_GiBps": round(r2["payload_bytes"] / (r2["open_ms"] / 1e3) / 2**30, 3),
                       "seal_achieved_GBps": round(r2["seal_alg_bytes"] / (r2["seal_ms"] / 1e3) / 1e9, 2),
                       "seal_hbm_frac": round(r2["seal_alg_bytes"] / (r2["seal_ms"] / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                       "seal_avg_launch_ms": round(r2["seal_ms"], 4), "sclk_mhz": r2.get("sclk_mhz"),
                       "verified": {"roundtrip": r2.get("verified_roundtrip"), "fusion_spot_check": None,
                                    "fusion_open_spot_check": None}}
        if R.world > 1:
            extra[name]["per_rank"] = per_rank(R, r2)
    if extra:
        out["extra"] = extra
    if args.e2e or (args.e2e is None and R.world == 1 and not args.records):  # (N = 1 at full size: 12 GiB pinned)
        out["e2e_host_buffers"] = run_e2e(R, WORKLOADS[args.workload].scaled(min(wl.nrecs, max(1, (4 << 30) // (wl.rec_len or 8192)))), args.e2e_chunks,
                                          schedule=args.schedule)
    if R.rank == 0 and R.world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], checks = cpu_baseline(wl, args.cpu_seconds, samples if args.verify else {}, ptlsbench_gpu)
        cb = out["cpu_baseline"]
        if cb.get("value"):  # GPU / CPU, against the noisy 16-thread median and against the stable 1-thread x cores
            out["gpu_over_cpu"] = {"vs_threads_median": round(out["value"] / cb["value"], 2),
                                   "vs_single_thread_x_cores": round(out["value"] / cb["single_thread_x_cores_GiBps"], 2)
                                   if cb.get("single_thread_x_cores_GiBps") else None}
        out["verified"]["fusion_spot_check"] = checks.get(wl.name)
        out["verified"]["fusion_open_spot_check"] = checks.get(wl.name + ":open")
        for name, e in extra.items():
            e["verified"]["fusion_spot_check"] = checks.get(name)
            if name != "ptlsbench":
                e["verified"]["fusion_open_spot_check"] = checks.get(name + ":open")
    elif R.rank == 0:
        out["cpu_baseline"] = None
    if R.rank == 0:
        print(json.dumps(out), flush=True)
    R.close()


if __name__ == "__main__":
    main()
