#!/usr/bin/env python3
"""Per-record seal and open of long records (the multi-workgroup span path): wall time per call, for a kernel trace."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picotls_amd as pa  # noqa: E402


def main():
    import torch

    torch.cuda.init()
    rng = np.random.default_rng(3)
    key, iv = rng.bytes(16), rng.bytes(12)
    enc, dec = pa.aead_new_direct(pa.aes128gcm, True, key, iv), pa.aead_new_direct(pa.aes128gcm, False, key, iv)
    for ln in (1 << 20, 2 << 20, 4 << 20, 8 << 20):
        pt, aad = rng.bytes(ln), rng.bytes(13)
        ct = enc.encrypt(pt, 5, aad)
        assert dec.decrypt(ct, 5, aad) == pt
        te, td = [], []
        for _ in range(5):
            t0 = time.perf_counter()
            enc.encrypt(pt, 5, aad)
            t1 = time.perf_counter()
            dec.decrypt(ct, 5, aad)
            te.append(t1 - t0)
            td.append(time.perf_counter() - t1)
        print(f"{ln:9d} B: encrypt {np.median(te) * 1e6:8.1f} us  decrypt {np.median(td) * 1e6:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
