"""Worker for engine behaviour that is fixed when a device is first used (environment read then), so it needs a fresh
process: run by tests/test_gpu_resources.py as `python gpu_engine_worker.py <mode>`; prints one JSON line.

  free_unordered  PTLS_MI355X_FAULT_ORDER=1: keyset_free cannot order its teardown on the device. A
                  batch launched on a side stream and freed at once must still seal correctly (the teardown then waits
                  for the keyset's launches on the host), and contexts created right after, which may reuse the entry,
                  must seal with their own keys.
  combine_slabs   PTLS_MI355X_COMBINE=4 with contexts in two entry slabs (1,024 entries each): calls of 16 threads are
                  combined only within a slab, and every result equals lib/fusion.c.
"""
import json
import os
import sys
import threading

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef  # noqa: E402
from picotls_amd.records import RecordBatch  # noqa: E402


def free_unordered(ref):
    rng = np.random.default_rng(91)
    n = 20000
    b = RecordBatch.build(np.full(n, 4096), 13, seqs=np.arange(n, dtype=np.uint64))
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    dev = torch.device("cuda:0")
    d_recs, d_pt, d_aad = (torch.from_numpy(x.view(np.uint8).copy()).to(dev) for x in (b.seal, pt, aad))
    side = torch.cuda.Stream(dev)
    outs, errors = [], []
    for r in range(3):
        key, iv = rng.bytes(16), rng.bytes(12)
        ks = pa.Keyset(key, iv, 16)
        d_out = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device=dev)
        side.wait_stream(torch.cuda.current_stream())
        pa.seal_batch(ks, d_recs.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), side.cuda_stream)
        ks.free()
        outs.append((key, iv, d_out))
        k2, v2 = rng.bytes(16), rng.bytes(12)
        ctx = pa.aead_new_direct(pa.aes128gcm, True, k2, v2)
        if ctx.encrypt(b"y" * 300, 5, b"a") != ref.seal(k2, v2, 5, b"a", b"y" * 300):
            errors.append(f"context after free {r}")
        ctx.free()
    side.synchronize()
    for i, (key, iv, d_out) in enumerate(outs):
        want = np.zeros(b.sealed_bytes, np.uint8)
        ref.run_batch(True, np.frombuffer(key, np.uint8), np.frombuffer(iv, np.uint8), 16, b.seal, pt, aad, want, nthreads=8)
        if not np.array_equal(d_out.cpu().numpy(), want):
            errors.append(f"batch {i} sealed under a cleared key")
    return {"errors": errors}


def combine_slabs(ref):
    rng = np.random.default_rng(92)
    # 1,100 live contexts: the first 1,024 fill one slab, the rest lie in a second one
    keys = [(rng.bytes(16), rng.bytes(12)) for _ in range(1100)]
    ctxs = [pa.aead_new_direct(pa.aes128gcm, True, k, v) for k, v in keys]
    nthreads, nops = 16, 40
    barrier = threading.Barrier(nthreads)
    errors = []

    def worker(t):
        r = np.random.default_rng(700 + t)
        try:
            for i in range(nops):
                if i % 4 == 0:
                    barrier.wait()
                c = int(r.integers(0, 1100)) if t % 2 else 1024 + int(r.integers(0, 76))  # odd threads: either slab
                pt, aad, seq = r.bytes(int(r.integers(0, 2000))), r.bytes(13), int(r.integers(0, 2**40))
                k, v = keys[c]
                if ctxs[c].encrypt(pt, seq, aad) != ref.seal(k, v, seq, aad, pt):
                    errors.append((t, i, c))
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))
            barrier.abort()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for c in ctxs:
        c.free()
    return {"errors": [str(e) for e in errors]}


if __name__ == "__main__":
    pa.load_library()
    out = {"free_unordered": free_unordered, "combine_slabs": combine_slabs}[sys.argv[1]](FusionRef())
    print(json.dumps(out), flush=True)
