#!/usr/bin/env python3
"""Constant-time probe of the LDS table lookups: seal (and open) the same batch shape under a given
key and payload, so that rocprofv3 --pmc SQ_LDS_BANK_CONFLICT / SQ_WAIT_INST_LDS / SQ_LDS_IDX_ACTIVE / SQ_INSTS_LDS can
be compared across keys and payloads. Identical shapes: record count, lengths, AAD, sequence numbers.

    python tools/ct_probe.py --key-seed 1 --payload zero|random|ones [--ct] [--workload tls16k --records 65536 --reps 3]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--key-seed", type=int, default=1)
    p.add_argument("--payload", choices=["zero", "random", "ones"], default="random")
    p.add_argument("--workload", default="tls16k")
    p.add_argument("--records", type=int, default=65536)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--lib", default=None, help="engine build to probe (default: picotls_amd/_lib/libptls_mi355x.so)")
    p.add_argument("--ct", action="store_true", help="the constant-time GHASH variant (ptls_mi355x_keyset_set_constant_time)")
    p.add_argument("--permute", type=int, default=0, help="seed of a permutation of the record lengths (0: none)")
    p.add_argument("--keys", type=int, default=0, help="override the workload's key count (0: keep it)")
    p.add_argument("--no-check", action="store_true", help="skip the ok check (a CT_PROBE_CONST diagnosis build)")
    a = p.parse_args()

    import torch

    import picotls_amd as pa

    if a.lib:
        pa.load_library(a.lib)
    from picotls_amd.workloads import WORKLOADS, payload_torch

    wl = WORKLOADS[a.workload].scaled(a.records)
    if a.keys:
        from dataclasses import replace

        wl = replace(wl, nkeys=a.keys)
    if a.permute:  # the same lengths in another order (keys and sequence numbers as before)
        from picotls_amd.records import RecordBatch

        key, seq = wl.key_and_seq(0, wl.nrecs)
        lens = np.random.default_rng(a.permute).permutation(wl.lens(0, wl.nrecs))
        b = RecordBatch.build(lens, wl.aad_len, seqs=seq, key_idx=key)
    else:
        b = wl.descriptors(0, wl.nrecs)
    rng = np.random.default_rng(a.key_seed)
    keys = np.frombuffer(rng.bytes(wl.nkeys * wl.key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(wl.nkeys * 12), np.uint8)
    ks = pa.Keyset(keys, ivs, wl.key_size)
    if a.ct:
        ks.set_constant_time(True)
    dev = torch.device("cuda:0")
    if a.payload == "random":
        d_pt = payload_torch(wl.seed, b.pt_bytes, dev)
    else:
        d_pt = torch.full((b.pt_bytes,), 0 if a.payload == "zero" else 0xFF, dtype=torch.uint8, device=dev)
    d_seal = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, 0)).to(dev)
    d_out = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    d_back = torch.empty(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.empty(b.n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(a.reps):
        pa.seal_batch(ks, d_seal.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), s)
        pa.open_batch(ks, d_open.data_ptr(), b.n, d_out.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    torch.cuda.synchronize()
    assert a.no_check or bool(d_ok.min().item() == 1)
    ks.free()
    print(f"ct_probe: key_seed={a.key_seed} payload={a.payload} workload={a.workload} records={b.n} ct={a.ct} "
          f"permute={a.permute} keys={wl.nkeys} ok")


if __name__ == "__main__":
    main()
