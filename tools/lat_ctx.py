#!/usr/bin/env python3
"""Per-context latency on an idle device: create a one-key keyset, seal one record through the per-record path, free;
run under rocprofv3 --kernel-trace --stats to split the setup kernel from the launch overheads."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picotls_amd as pa  # noqa: E402

lib = pa.load_library()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
rng = np.random.default_rng(1)
keys = np.frombuffer(rng.bytes(32 * n), np.uint8)
out = ctypes.create_string_buffer(1216)
pt = bytes(1200)
t = {"new": [], "seal1": [], "seal2": [], "free": []}
for i in range(n):
    t0 = time.perf_counter()
    h = ctypes.c_void_p(lib.ptls_mi355x_keyset_new(keys[32 * i:].ctypes.data, keys[32 * i:].ctypes.data, 1, 16))
    t1 = time.perf_counter()
    lib.ptls_mi355x_encrypt(h, 0, out, pt, 1200, i, None, 0)
    t2 = time.perf_counter()
    lib.ptls_mi355x_encrypt(h, 0, out, pt, 1200, i, None, 0)
    t3 = time.perf_counter()
    lib.ptls_mi355x_keyset_free(h)
    t4 = time.perf_counter()
    for k, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
        t[k].append(v * 1e6)
print({k: round(float(np.median(v[n // 10:])), 1) for k, v in t.items()})
