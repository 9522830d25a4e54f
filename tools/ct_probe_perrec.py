#!/usr/bin/env python3
"""Constant-time probe of the per-record (picotls vtable) path: `calls` synchronous seals and opens of one record
length through a picotls-style context (pa.aead_new_direct: constant-time unless PTLS_MI355X_CONSTANT_TIME=0, as the
ptls_mi355x_aes*gcm objects), under a given key and payload, for rocprofv3 --pmc SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS
per dispatch. Identical shapes across runs: length, AAD, sequence numbers.

    python tools/ct_probe_perrec.py --key-seed 1 --payload zero|random --len 1200 [--calls 8]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--key-seed", type=int, default=1)
    p.add_argument("--payload", choices=["zero", "random"], default="random")
    p.add_argument("--len", type=int, default=1200)
    p.add_argument("--calls", type=int, default=8)
    a = p.parse_args()

    import torch

    import picotls_amd as pa

    torch.cuda.init()
    rng = np.random.default_rng(a.key_seed)
    key, iv = rng.bytes(16), rng.bytes(12)
    enc = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
    dec = pa.aead_new_direct(pa.aes128gcm, False, key, iv)
    pt = bytes(a.len) if a.payload == "zero" else np.random.default_rng(1000 + a.key_seed).bytes(a.len)
    aad = bytes(range(13))
    for i in range(a.calls):
        ct = enc.encrypt(pt, 100 + i, aad)
        assert dec.decrypt(ct, 100 + i, aad) == pt
    print(f"ct_probe_perrec: {a.calls} seal+open of {a.len} B, key {a.key_seed}, {a.payload}, constant-time "
          f"{enc.ks.constant_time}")


if __name__ == "__main__":
    main()
