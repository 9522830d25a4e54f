#!/usr/bin/env python3
"""Attribution of the many-key mixed seal's extra HBM traffic: seal the configs[3] batch (64K keys,
U[64,16384], AES-256) in three layouts, one process per layout and per rocprofv3 --pmc pass:
  packed   bench.py's layout: records back to back in 16-byte slots
  slot128  every record's input and output slot starts on a 128-byte line (no line shared between records)
  lines    slot128, and each length cut to 16 * (8k + 7) bytes, so that the chunked kernel's step-aligned units put
           every 8-lane group store on exactly one 128-byte line (text block b at stream position b mod 8)
Prints the algorithmic bytes per launch and the median seal time.

    python tools/mixed_align.py --layout packed|slot128|lines [--records 4194304] [--ct]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _slots(lens, unit):
    s = (lens + np.uint64(unit - 1)) // np.uint64(unit) * np.uint64(unit)
    return np.concatenate([[0], np.cumsum(s)[:-1]]).astype(np.uint64), int(s.sum())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--layout", choices=["packed", "slot128", "lines"], default="packed")
    p.add_argument("--workload", default="mixed")
    p.add_argument("--records", type=int, default=4 << 20)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--ct", action="store_true", help="constant-time variant (another register allocation: fewer spills)")
    a = p.parse_args()

    import torch

    import picotls_amd as pa
    from picotls_amd.workloads import WORKLOADS, payload_torch

    wl = WORKLOADS[a.workload].scaled(a.records)
    b = wl.descriptors(0, wl.nrecs)
    recs = b.seal.copy()
    in_bytes, out_bytes = b.pt_bytes, b.sealed_bytes
    if a.layout != "packed":
        L = recs["len"].astype(np.uint64)
        if a.layout == "lines":
            nb = np.maximum(L // np.uint64(16), np.uint64(7))
            L = np.uint64(16) * ((nb - np.uint64(7)) // np.uint64(8) * np.uint64(8) + np.uint64(7))
            recs["len"] = L.astype(recs["len"].dtype)
        recs["in_off"], in_bytes = _slots(L, 128)
        recs["out_off"], out_bytes = _slots(L + np.uint64(16), 128)
    L = recs["len"].astype(np.int64)
    alg_r = int((L + recs["aad_len"].astype(np.int64) + 40).sum())
    alg_w = int((L + 16).sum())
    keys, ivs = wl.keys()
    ks = pa.Keyset(keys, ivs, wl.key_size)
    if a.ct:
        ks.set_constant_time(True)
    dev = torch.device("cuda:0")
    d_pt = payload_torch(wl.seed, in_bytes, dev)
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
    print(f"mixed_align: layout={a.layout} ct={a.ct} records={b.n} payload {int(L.sum())} B; algorithmic per launch: reads "
          f"{alg_r} B, writes {alg_w} B; seal median {ms[len(ms) // 2]:.3f} ms "
          f"({int(L.sum()) / ms[len(ms) // 2] / 1e6 / 1.073741824:.1f} GiB/s) over {len(ms)} launches")


if __name__ == "__main__":
    main()
