#!/usr/bin/env python3
"""A/B timing of engine variants on TLS 1.2 record batches (ptls_mi355x_seal_tls12_records / open_tls12_records), in ONE
process with interleaved rounds, as tools/ab.py does for unframed batches. Records: explicit nonce || plaintext in,
header || nonce || ciphertext || tag out (lib/picotls.c's TLS 1.2 AEAD record layout). Checks that every variant
produces identical wire records and opens them.

    python tools/ab_tls12.py tools/variants/libA.so tools/variants/libB.so [--records 131072 --len 16384]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotls_amd import RECORD_DTYPE  # noqa: E402
from picotls_amd.workloads import payload_torch  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.ptls_mi355x_keyset_new.argtypes = [vp, vp, sz, sz]
    lib.ptls_mi355x_keyset_new.restype = vp
    lib.ptls_mi355x_seal_tls12_records.argtypes = [vp, vp, sz, vp, vp, vp]
    lib.ptls_mi355x_open_tls12_records.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--records", type=int, default=131072)
    ap.add_argument("--len", type=int, default=16384)
    ap.add_argument("--key-size", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    n, ln = a.records, a.len
    rng = np.random.default_rng(1212)
    key = np.frombuffer(rng.bytes(a.key_size), np.uint8)
    iv = np.frombuffer(rng.bytes(4) + bytes(8), np.uint8)  # fixed IV || zero static IV (the TLS 1.2 AEAD IV)
    i = np.arange(n, dtype=np.uint64)
    seal = np.zeros(n, dtype=RECORD_DTYPE)
    seal["in_off"], seal["out_off"], seal["len"] = i * (8 + ln), i * (29 + ln), ln
    seal["seq"], seal["flags"] = i + 1, 23
    opn = seal.copy()
    opn["in_off"], opn["out_off"] = seal["out_off"], i * ln
    dev = torch.device("cuda:0")
    d_seal = torch.from_numpy(seal.view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(opn.view(np.uint8).copy()).to(dev)
    d_in = payload_torch(0x1212, n * (8 + ln), dev)
    wire = {p: torch.empty(n * (29 + ln), dtype=torch.uint8, device=dev) for p in a.libs}
    plain = torch.empty(n * ln, dtype=torch.uint8, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    libs = [(p, bind(p)) for p in a.libs]
    kss = {p: ctypes.c_void_p(lib.ptls_mi355x_keyset_new(key.ctypes.data, iv.ctypes.data, 1, a.key_size)) for p, lib in libs}
    s = torch.cuda.current_stream().cuda_stream
    t = {p: ([], []) for p in a.libs}
    for rnd in range(a.rounds + 1):
        for p, lib in libs:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            for _ in range(a.reps):
                assert lib.ptls_mi355x_seal_tls12_records(kss[p], d_seal.data_ptr(), n, d_in.data_ptr(), wire[p].data_ptr(), s) == 0
            ev[1].record()
            for _ in range(a.reps):
                assert lib.ptls_mi355x_open_tls12_records(kss[p], d_open.data_ptr(), n, wire[p].data_ptr(), plain.data_ptr(),
                                                          ok.data_ptr(), None, s) == 0
            ev[2].record()
            torch.cuda.synchronize()
            if rnd:  # round 0 warms up
                t[p][0].append(ev[0].elapsed_time(ev[1]) / a.reps)
                t[p][1].append(ev[1].elapsed_time(ev[2]) / a.reps)
            assert bool(ok.all()), f"{p}: open rejected a record"
    first = a.libs[0]
    same = all(torch.equal(wire[p], wire[first]) for p in a.libs)
    gib = n * ln / 2**30
    for p in a.libs:
        sm, om = float(np.median(t[p][0])), float(np.median(t[p][1]))
        print(f"{os.path.basename(p):32s} TLS 1.2 {n} x {ln} B  seal {sm:8.3f} ms {gib / sm * 1e3:8.1f} GiB/s  "
              f"open {om:8.3f} ms {gib / om * 1e3:8.1f} GiB/s  seal+open {2 * gib / (sm + om) * 1e3:8.1f} GiB/s")
    print(f"identical wire records across variants: {same}")
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
