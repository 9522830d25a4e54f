#!/usr/bin/env python3
"""A/B timing of engine variants in ONE process (interleaved rounds; guide §5.4 rule 24).

    python tools/ab.py tools/variants/libA.so tools/variants/libB.so [--workload tls16k --records 262144 --rounds 5]

Each variant is a separately built libptls_mi355x.so (same C ABI), loaded with RTLD_LOCAL. Checks that every variant
produces identical sealed output.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotls_amd.workloads import WORKLOADS, payload_torch  # noqa: E402


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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--workload", default="tls16k")
    ap.add_argument("--records", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--schedule", type=int, default=0, help="ptls_mi355x_keyset_set_schedule value (0 auto)")
    a = ap.parse_args()
    wl = WORKLOADS[a.workload].scaled(a.records)
    b = wl.descriptors(0, wl.nrecs)
    keys, ivs = wl.keys()
    dev = torch.device("cuda:0")
    d_seal = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, 0)).to(dev)
    d_pt = payload_torch(wl.seed, b.pt_bytes, dev)
    outs = {}
    # a variant is a library path, optionally suffixed ":ct" (the same build with ptls_mi355x_keyset_set_constant_time)
    libs = [(p, bind(p.split(":")[0])) for p in a.libs]
    kss = {}
    for p, lib in libs:
        kss[p] = ctypes.c_void_p(lib.ptls_mi355x_keyset_new(keys.ctypes.data, ivs.ctypes.data, wl.nkeys, wl.key_size))
        assert kss[p].value, p
        if a.schedule and hasattr(lib, "ptls_mi355x_keyset_set_schedule"):
            assert lib.ptls_mi355x_keyset_set_schedule(kss[p], a.schedule) == 0
        if p.endswith(":ct"):
            assert lib.ptls_mi355x_keyset_set_constant_time(kss[p], 1) == 0
    sealed = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    back = torch.empty(b.pt_bytes, dtype=torch.uint8, device=dev)
    ok = torch.empty(b.n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    times = {p: {"seal": [], "open": []} for p, _ in libs}
    for rnd in range(a.rounds + 1):
        for p, lib in libs:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            for _ in range(a.reps):
                assert lib.ptls_mi355x_seal_batch(kss[p], d_seal.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(),
                                                  sealed.data_ptr(), s) == 0
            ev[1].record()
            for _ in range(a.reps):
                assert lib.ptls_mi355x_open_batch(kss[p], d_open.data_ptr(), b.n, sealed.data_ptr(), d_aad.data_ptr(),
                                                  back.data_ptr(), ok.data_ptr(), s) == 0
            ev[2].record()
            torch.cuda.synchronize()
            if rnd > 0:
                times[p]["seal"].append(ev[0].elapsed_time(ev[1]) / a.reps)
                times[p]["open"].append(ev[1].elapsed_time(ev[2]) / a.reps)
            if rnd == 1:
                outs[p] = (torch.sum(sealed.view(torch.int64)).item(), bool(ok.min().item() == 1))
    ref = None
    for p, _ in libs:
        sm, so = np.median(times[p]["seal"]), np.median(times[p]["open"])
        gib = b.payload_bytes / 2**30
        print(f"{os.path.basename(p):40s} seal {sm:8.3f} ms {gib / sm * 1e3:8.1f} GiB/s  open {so:8.3f} ms "
              f"{gib / so * 1e3:8.1f} GiB/s  seal+open {2 * gib / (sm + so) * 1e3:8.1f} GiB/s  min seal {min(times[p]['seal']):.3f}"
              f"  checksum {outs[p][0]} ok={outs[p][1]}")
        if ref is None:
            ref = outs[p][0]
        elif outs[p][0] != ref:
            print("  !! output differs from the first variant")


if __name__ == "__main__":
    main()
