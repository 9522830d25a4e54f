#!/usr/bin/env python3
"""Small-batch launches (the regime of configs[0]: ptlsbench's 1000-record batches): seal and open time per launch for
batches of a few hundred to a few thousand records, one library build or several (interleaved, one process), with
identical output checked across builds.

    python tools/small_batch.py [lib.so ...] [--rounds 5 --reps 20]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = [(10, 1 << 20), (2, 8 << 20), (40, 256 << 10), (64, 65536), (100, 16384), (256, 16384), (1000, 16384), (2000, 16384), (4096, 16384), (8192, 16384), (1000, 1200),
         (4096, 1200), (1000, 64)]


def bind(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.ptls_mi355x_keyset_new.argtypes = [vp, vp, sz, sz]
    lib.ptls_mi355x_keyset_new.restype = vp
    lib.ptls_mi355x_seal_batch.argtypes = [vp, vp, sz, vp, vp, vp, vp]
    lib.ptls_mi355x_open_batch.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*", default=["picotls_amd/_lib/libptls_mi355x.so"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--keys", type=int, default=1, help="connection keys (record i uses key i mod keys)")
    ap.add_argument("--cases", default="", help="n:len,... instead of the default list")
    a = ap.parse_args()

    import torch

    from picotls_amd.records import RecordBatch
    from picotls_amd.workloads import payload_torch

    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(3)
    key, iv = np.frombuffer(rng.bytes(16 * a.keys), np.uint8), np.frombuffer(rng.bytes(12 * a.keys), np.uint8)
    libs = [(p, bind(p)) for p in a.libs]
    kss = {p: ctypes.c_void_p(lib.ptls_mi355x_keyset_new(key.ctypes.data, iv.ctypes.data, a.keys, 16)) for p, lib in libs}
    cases = [tuple(int(x) for x in c.split(":")) for c in a.cases.split(",")] if a.cases else CASES
    for n, ln in cases:
        b = RecordBatch.build(np.full(n, ln, np.uint64), 13, seqs=np.arange(n, dtype=np.uint64),
                              key_idx=np.arange(n) % a.keys)
        d_seal = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
        d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
        d_aad = torch.from_numpy(np.frombuffer(rng.bytes(b.aad_bytes), np.uint8).copy()).to(dev)
        d_pt = payload_torch(7, b.pt_bytes, dev)
        d_out = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
        d_back = torch.empty(b.pt_bytes, dtype=torch.uint8, device=dev)
        d_ok = torch.empty(n, dtype=torch.uint8, device=dev)
        t = {p: ([], []) for p, _ in libs}
        sums = {}
        for rnd in range(a.rounds + 1):
            for p, lib in libs:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record()
                for _ in range(a.reps):
                    assert lib.ptls_mi355x_seal_batch(kss[p], d_seal.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(),
                                                      d_out.data_ptr(), s) == 0
                ev[1].record()
                for _ in range(a.reps):
                    assert lib.ptls_mi355x_open_batch(kss[p], d_open.data_ptr(), n, d_out.data_ptr(), d_aad.data_ptr(),
                                                      d_back.data_ptr(), d_ok.data_ptr(), s) == 0
                ev[2].record()
                torch.cuda.synchronize()
                if rnd:
                    t[p][0].append(ev[0].elapsed_time(ev[1]) * 1e3 / a.reps)
                    t[p][1].append(ev[1].elapsed_time(ev[2]) * 1e3 / a.reps)
                else:
                    sums[p] = (int(torch.sum(d_out.view(torch.int64) if d_out.numel() % 8 == 0 else d_out.long()).item()),
                               bool(d_ok.min().item() == 1))
        base = None
        for p, _ in libs:
            su, so = np.median(t[p][0]), np.median(t[p][1])
            gib = b.payload_bytes / 2**30
            same = "" if base is None or sums[p] == base else "  !! output differs"
            base = base or sums[p]
            print(f"{n:6d} x {ln:5d} B  {os.path.basename(p):24s} seal {su:8.1f} us ({gib / su * 1e6:7.1f} GiB/s)  open "
                  f"{so:8.1f} us ({gib / so * 1e6:7.1f} GiB/s)  ok={sums[p][1]}{same}", flush=True)


if __name__ == "__main__":
    main()
