#!/usr/bin/env python3
"""Aggregate rate of the synchronous per-record path under concurrency: T host threads, each with its own one-key
keyset (a picotls context), call ptls_mi355x_encrypt on their own buffers in a loop for a fixed time. ctypes releases
the GIL around the call, so the threads overlap inside the engine. Prints calls/s over all threads and the median
call latency, per record length and thread count. Optional argv[1]: another build of libptls_mi355x.so (A/B)."""
import ctypes
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picotls_amd as pa  # noqa: E402


def run(lib, nthreads: int, ln: int, seconds: float):
    rng = np.random.default_rng(nthreads * 1000 + ln)
    kss = [pa.Keyset(rng.bytes(16), rng.bytes(12), 16) for _ in range(nthreads)]
    ins = [ctypes.create_string_buffer(rng.bytes(max(ln, 1)), max(ln, 1)) for _ in range(nthreads)]
    outs = [ctypes.create_string_buffer(ln + 16) for _ in range(nthreads)]
    aads = [ctypes.create_string_buffer(rng.bytes(13), 13) for _ in range(nthreads)]
    counts = [0] * nthreads
    lats = [[] for _ in range(nthreads)]
    errors = []
    start = threading.Barrier(nthreads + 1)
    stop = threading.Event()

    def worker(t):
        h = kss[t].handle
        enc = lib.ptls_mi355x_encrypt
        for _ in range(5):  # setup + warm-up
            enc(h, 0, outs[t], ins[t], ln, 1, aads[t], 13)
        start.wait()
        seq = 2
        while not stop.is_set():
            t0 = time.perf_counter()
            if enc(h, 0, outs[t], ins[t], ln, seq, aads[t], 13) != 0:
                errors.append(t)
                return
            lats[t].append(time.perf_counter() - t0)
            seq += 1
            counts[t] += 1

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    start.wait()
    t0 = time.perf_counter()
    time.sleep(seconds)
    stop.set()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    for ks in kss:
        ks.free()
    if errors:
        raise RuntimeError(f"encrypt failed in threads {errors}")
    allat = np.concatenate([np.asarray(v) for v in lats])
    return sum(counts) / dt, float(np.median(allat)) * 1e6, float(np.percentile(allat, 99)) * 1e6


def main():
    import torch

    torch.cuda.init()
    lib = pa.load_library(sys.argv[1]) if len(sys.argv) > 1 else pa.load_library()
    secs = float(os.environ.get("MT_SECONDS", "1.0"))
    for ln in (16, 1200, 16384):
        for nt in (1, 2, 4, 8, 16):
            rate, p50, p99 = run(lib, nt, ln, secs)
            print(f"len {ln:6d} threads {nt:2d}: {rate:10.0f} calls/s  {rate * ln / 2**20:8.1f} MiB/s  "
                  f"p50 {p50:7.1f} us  p99 {p99:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
