#!/usr/bin/env python3
"""300 synchronous per-record encrypts of one size (the picotls vtable path), for rocprofv3 kernel traces; with a
-DENGINE_PROFILE=1 build as the second argument it also prints the chunked kernel's phase split per launch.

    python tools/lat_one.py 16 [tools/variants/lib_prof.so]
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picotls_amd as pa  # noqa: E402


def main():
    import torch

    torch.cuda.init()
    lib = pa.load_library(sys.argv[2]) if len(sys.argv) > 2 else pa.load_library()
    rng = np.random.default_rng(1)
    enc = pa.aead_new_direct(pa.aes128gcm, True, rng.bytes(16), rng.bytes(12))
    pt, aad = rng.bytes(int(sys.argv[1])), rng.bytes(13)
    calls = 300
    for _ in range(20):
        enc.encrypt(pt, 7, aad)
    prof = (ctypes.c_ulonglong * 24)()  # PROF_SLOTS
    dbg = getattr(lib, "ptls_mi355x_debug_profile", None)  # exported by -DENGINE_PROFILE=1 builds only
    if dbg is not None:
        dbg.argtypes = [ctypes.c_void_p, ctypes.c_int]
        dbg(prof, 1)
    for _ in range(calls):
        enc.encrypt(pt, 7, aad)
    if dbg is None:
        return
    dbg(prof, 1)
    p = list(prof)
    if p[6]:  # cycles per launch (s_memtime), summed over the launch's workgroups
        wg = max(p[10], 1)
        print(f"{sys.argv[1]} B: {p[6] / calls:.1f} runs/launch, {wg / calls:.1f} workgroups/launch; cycles per "
              f"workgroup: AES tables {p[8] / wg:.0f}, first scan {p[9] / wg:.0f}, prologue {p[3] / wg:.0f}, "
              f"GHASH tables {p[1] / wg:.0f}, unit loop {p[2] / wg:.0f}, wave idle at the run barrier "
              f"{p[4] / wg / 16:.0f}")


if __name__ == "__main__":
    main()
