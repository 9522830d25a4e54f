#!/usr/bin/env python3
"""Per-record seals of 16 B and 1200 B (300 each) for a kernel trace of the per-record path (tools/gpu_recipes.sh latprof)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picotls_amd as pa  # noqa: E402


def main():
    import torch

    torch.cuda.init()
    rng = np.random.default_rng(1)
    key, iv = rng.bytes(16), rng.bytes(12)
    enc = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
    for ln in (16, 1200):
        pt, aad = rng.bytes(ln), rng.bytes(13)
        for _ in range(300):
            enc.encrypt(pt, 7, aad)
    enc.free()


if __name__ == "__main__":
    main()
