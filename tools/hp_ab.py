#!/usr/bin/env python3
"""Header-protection cost of several engine builds, interleaved in ONE process (tools/hp_cost.py times one build per
process, whose box-to-box and run-to-run spread, +-2 %, is as large as the effects measured here): per round and build,
seal_batch then seal_batch_hp on the configs[2] batch (4M x 1200 B, a QUIC sample 4 bytes into each packet); medians
over the rounds, and every build's masks compared with the first build's.

    python tools/hp_ab.py tools/variants/libA.so tools/variants/libB.so [--records 4194304 --rounds 30]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotls_amd.records import HP_DTYPE  # noqa: E402
from picotls_amd.workloads import WORKLOADS, payload_torch  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.ptls_mi355x_keyset_new.argtypes = [vp, vp, sz, sz]
    lib.ptls_mi355x_keyset_new.restype = vp
    lib.ptls_mi355x_seal_batch.argtypes = [vp, vp, sz, vp, vp, vp, vp]
    lib.ptls_mi355x_seal_batch_hp.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp, vp, vp]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--records", type=int, default=4 << 20)
    ap.add_argument("--rounds", type=int, default=30)
    a = ap.parse_args()
    wl = WORKLOADS["quic1200"].scaled(a.records)
    b = wl.descriptors(0, wl.nrecs)
    keys, ivs = wl.keys()
    hp_key = np.frombuffer(bytes(range(16, 32)), np.uint8).copy()
    hp = np.zeros(b.n, HP_DTYPE)
    hp["sample_off"] = b.seal["out_off"] + 4
    dev = torch.device("cuda:0")
    d_recs = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_hp = torch.from_numpy(hp.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, 0)).to(dev)
    d_pt = payload_torch(wl.seed, b.pt_bytes, dev)
    d_out = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    libs = []
    for p in a.libs:
        lib = bind(p)
        ks = lib.ptls_mi355x_keyset_new(keys.ctypes.data, ivs.ctypes.data, 1, 16)
        hks = lib.ptls_mi355x_keyset_new(hp_key.ctypes.data, np.zeros(12, np.uint8).ctypes.data, 1, 16)
        assert ks and hks, p
        libs.append((p, lib, ctypes.c_void_p(ks), ctypes.c_void_p(hks),
                     torch.empty(b.n * 16, dtype=torch.uint8, device=dev)))
    t = {p: {"seal": [], "hp": []} for p, *_ in libs}
    for rnd in range(a.rounds + 1):
        for p, lib, ks, hks, d_mask in libs:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            assert lib.ptls_mi355x_seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(),
                                              d_out.data_ptr(), s) == 0
            ev[1].record()
            assert lib.ptls_mi355x_seal_batch_hp(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(),
                                                 d_out.data_ptr(), hks, d_hp.data_ptr(), d_mask.data_ptr(), s) == 0
            ev[2].record()
            torch.cuda.synchronize()
            if rnd:
                t[p]["seal"].append(ev[0].elapsed_time(ev[1]))
                t[p]["hp"].append(ev[1].elapsed_time(ev[2]))
    ref = libs[0][4]
    for p, *_, d_mask in libs:
        ms, mh = float(np.median(t[p]["seal"])), float(np.median(t[p]["hp"]))
        # per-round ratio, then its median: the pair shares the clock state of its round
        r = float(np.median(np.array(t[p]["hp"]) / np.array(t[p]["seal"])))
        print(f"hp_ab {os.path.basename(p):20s} seal {ms:.3f} ms  seal+HP {mh:.3f} ms  ({100 * (mh / ms - 1):+.2f} %; "
              f"median of per-round ratios {100 * (r - 1):+.2f} %)  masks equal to the first build's: "
              f"{bool(torch.equal(d_mask, ref))}")


if __name__ == "__main__":
    main()
