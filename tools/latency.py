#!/usr/bin/env python3
"""Latency of the synchronous per-record path (the picotls vtable's batch of one: staging copy up, one launch, copy
down) -- ptls_mi355x_encrypt / _decrypt / _encrypt_block / _quiclb_transform on host buffers. Median of N calls."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picotls_amd as pa  # noqa: E402


def med(f, n=300):
    for _ in range(20):
        f()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        t.append(time.perf_counter() - t0)
    return float(np.median(t)) * 1e6


def main():
    import torch

    torch.cuda.init()
    if len(sys.argv) > 1:  # another build of libptls_mi355x.so (A/B)
        pa.load_library(sys.argv[1])
        print("library:", sys.argv[1])
    rng = np.random.default_rng(1)
    key, iv = rng.bytes(16), rng.bytes(12)
    enc = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
    dec = pa.aead_new_direct(pa.aes128gcm, False, key, iv)
    for ln in (16, 1200, 16384, 1 << 20, 4 << 20):
        pt, aad = rng.bytes(ln), rng.bytes(13)
        ct = enc.encrypt(pt, 7, aad)
        assert dec.decrypt(ct, 7, aad) == pt
        n = 300 if ln <= 16384 else 20
        print(f"encrypt {ln:8d} B: {med(lambda: enc.encrypt(pt, 7, aad), n):9.1f} us   decrypt: "
              f"{med(lambda: dec.decrypt(ct, 7, aad), n):9.1f} us")
    hp = pa.CtrCipher(rng.bytes(16))
    pt, aad = rng.bytes(1200), rng.bytes(13)
    print(f"encrypt_s 1200 B + header-protection mask (QUIC packet): {med(lambda: enc.encrypt_s(pt, 7, aad, hp, 4)[0]):8.1f} us")
    print(f"header-protection mask (encrypt_block): {med(lambda: hp.mask(bytes(16))):8.1f} us")
    lb = pa.QuicLbCipher(True, rng.bytes(16))
    print(f"QUIC-LB CID (quiclb_transform):         {med(lambda: lb.encrypt(bytes(12))):8.1f} us")


if __name__ == "__main__":
    main()
