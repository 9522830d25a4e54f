#!/usr/bin/env python3
"""Cost of QUIC header protection in the batch path (fusion's supp `lib/fusion.c:425-430,636-651`):
seal_batch alone vs seal_batch_hp (one launch: the chunked seal computes each run's 16-byte AES-ECB masks from samples of
its sealed output under a second key) vs the two-launch form (seal_batch, then hp_mask_batch) on the configs[2] batch,
interleaved rounds in one process, HIP events.

    python tools/hp_cost.py [--records 4194304] [--rounds 5]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--records", type=int, default=4 << 20)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--lib", default=None, help="another build of libptls_mi355x.so (A/B)")
    a = p.parse_args()

    import torch

    import picotls_amd as pa

    if a.lib:
        pa.load_library(a.lib)
    from picotls_amd.records import HP_DTYPE
    from picotls_amd.workloads import WORKLOADS, payload_torch

    wl = WORKLOADS["quic1200"].scaled(a.records)
    b = wl.descriptors(0, wl.nrecs)
    keys, ivs = wl.keys()
    ks = pa.Keyset(keys, ivs, 16)
    hp_ks = pa.Keyset(np.frombuffer(os.urandom(16), np.uint8), np.zeros(12, np.uint8), 16)
    hp = np.zeros(b.n, HP_DTYPE)
    hp["sample_off"] = b.seal["out_off"] + 4  # a QUIC sample: 16 bytes from 4 past the packet-number offset
    dev = torch.device("cuda:0")
    d_recs = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_hp = torch.from_numpy(hp.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, 0)).to(dev)
    d_pt = payload_torch(wl.seed, b.pt_bytes, dev)
    d_out = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    d_mask = torch.empty(b.n * 16, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    t = {"seal": [], "seal_hp": [], "hp": [], "two": []}
    for rnd in range(a.rounds + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        ev[0].record()
        pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), s)
        ev[1].record()
        pa.seal_batch_hp(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), hp_ks,
                         d_hp.data_ptr(), d_mask.data_ptr(), s)
        ev[2].record()
        pa.hp_mask_batch(hp_ks, d_hp.data_ptr(), b.n, d_out.data_ptr(), d_mask.data_ptr(), s)
        ev[3].record()
        pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), s)
        pa.hp_mask_batch(hp_ks, d_hp.data_ptr(), b.n, d_out.data_ptr(), d_mask.data_ptr(), s)
        ev[4].record()
        torch.cuda.synchronize()
        if rnd:
            t["seal"].append(ev[0].elapsed_time(ev[1]))
            t["seal_hp"].append(ev[1].elapsed_time(ev[2]))
            t["hp"].append(ev[2].elapsed_time(ev[3]))
            t["two"].append(ev[3].elapsed_time(ev[4]))
    gib = b.payload_bytes / 2**30
    m = {k: float(np.median(v)) for k, v in t.items()}
    print(f"hp_cost: {b.n} x 1200 B records: seal {m['seal']:.3f} ms ({gib / m['seal'] * 1e3:.1f} GiB/s), seal + HP masks "
          f"{m['seal_hp']:.3f} ms ({gib / m['seal_hp'] * 1e3:.1f} GiB/s, {100 * (m['seal_hp'] / m['seal'] - 1):+.2f} %), "
          f"masks alone {m['hp']:.3f} ms ({b.n / m['hp'] / 1e3:.1f} M masks/s), two launches (seal, then masks) "
          f"{m['two']:.3f} ms ({100 * (m['two'] / m['seal'] - 1):+.2f} %)")
    ks.free()
    hp_ks.free()


if __name__ == "__main__":
    main()
