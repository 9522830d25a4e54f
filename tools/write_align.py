#!/usr/bin/env python3
"""Attribution of the seal kernel's extra HBM writes: seal 16 KiB TLS records with the sealed records
placed (a) back to back in 16400-byte slots (bench.py's layout) or (b) at out_off = 112 mod 128 in 16512-byte slots, so
that every 8-lane group's 128-byte store of a step covers exactly one 128-byte line (the stream's text block b sits at
position b + 7 for A = 5, L = 16384). Run each layout under rocprofv3 --pmc WRITE_SIZE (one process per layout).

    python tools/write_align.py --layout packed|aligned [--records 262144]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--layout", choices=["packed", "aligned"], default="packed")
    p.add_argument("--records", type=int, default=262144)
    p.add_argument("--reps", type=int, default=2)
    a = p.parse_args()

    import torch

    import picotls_amd as pa
    from picotls_amd.workloads import WORKLOADS, payload_torch

    wl = WORKLOADS["tls16k"].scaled(a.records)
    b = wl.descriptors(0, wl.nrecs)
    recs = b.seal.copy()
    out_bytes = b.sealed_bytes
    if a.layout == "aligned":
        recs["out_off"] = 112 + np.arange(b.n, dtype=np.uint64) * 16512
        out_bytes = 112 + b.n * 16512
    keys, ivs = wl.keys()
    ks = pa.Keyset(keys, ivs, 16)
    dev = torch.device("cuda:0")
    d_pt = payload_torch(wl.seed, b.pt_bytes, dev)
    d_recs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, 0)).to(dev)
    d_out = torch.zeros(out_bytes, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
    ev[0].record()
    for i in range(a.reps):
        pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), s)
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(1, a.reps))  # the first launch warms up
    ks.free()
    print(f"write_align: layout={a.layout} records={b.n} algorithmic writes per launch {b.n * 16400} B, "
          f"seal median {ms[len(ms) // 2]:.3f} ms over {len(ms)} launches")


if __name__ == "__main__":
    main()
