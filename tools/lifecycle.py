#!/usr/bin/env python3
"""Context lifecycle under load: does creating and freeing picotls-style contexts (one-key keysets,
ptls_mi355x_keyset_new / _free, what every ptls_aead_new_direct / ptls_aead_free on the MI355X objects does) disturb
bulk batches streaming on another stream?

Interleaved A/B in one process: `reps` rounds of [bulk alone, bulk while a second thread creates, uses once and frees
`contexts` contexts (bulk launches continue until the churn is done)]. Bulk = seal_batch over 256K x 16 KiB records
(4 GiB), back to back on one stream, timed with HIP events. Prints one JSON line: bulk GiB/s alone and under churn, their
ratio, and the churn thread's per-context costs (create, first seal, second seal, free) on an idle device and under the bulk load.

    python tools/lifecycle.py [--contexts 1000] [--reps 4] [--records 262144]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--contexts", type=int, default=1000)
    p.add_argument("--reps", type=int, default=4)
    p.add_argument("--records", type=int, default=262144)
    p.add_argument("--launches", type=int, default=40, help="bulk seal launches per alone measurement")
    a = p.parse_args()

    import torch

    import picotls_amd as pa
    from picotls_amd.workloads import WORKLOADS, payload_torch

    lib = pa.load_library()
    dev = torch.device("cuda:0")
    wl = WORKLOADS["tls16k"].scaled(a.records)
    b = wl.descriptors(0, wl.nrecs)
    keys, ivs = wl.keys()
    ks = pa.Keyset(keys, ivs, 16)
    d_recs = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, 0)).to(dev)
    d_pt = payload_torch(wl.seed, b.pt_bytes, dev)
    d_out = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    bulk = torch.cuda.Stream(dev)

    def run_bulk():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(bulk)
        for _ in range(a.launches):
            pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), bulk.cuda_stream)
        e1.record(bulk)
        return e0, e1

    rng = np.random.default_rng(5)
    ctx_keys = np.frombuffer(rng.bytes(a.contexts * 16), np.uint8)
    ctx_ivs = np.frombuffer(rng.bytes(a.contexts * 12), np.uint8)
    pt = bytes(1200)
    out = ctypes.create_string_buffer(1216)

    def churn(stats):
        # one context per iteration: create, seal one 1200-byte record (the first use waits for its setup), seal a
        # second one (a context in use), free
        t_new, t_first, t_second, t_free = [], [], [], []
        t00 = time.perf_counter()
        for n in range(a.contexts):
            t0 = time.perf_counter()
            h = lib.ptls_mi355x_keyset_new(ctx_keys[16 * n:].ctypes.data, ctx_ivs[12 * n:].ctypes.data, 1, 16)
            t1 = time.perf_counter()
            assert h, pa._err("keyset_new")
            assert lib.ptls_mi355x_encrypt(ctypes.c_void_p(h), 0, out, pt, len(pt), n, None, 0) == 0
            t2 = time.perf_counter()
            assert lib.ptls_mi355x_encrypt(ctypes.c_void_p(h), 0, out, pt, len(pt), n + 1, None, 0) == 0
            t3 = time.perf_counter()
            lib.ptls_mi355x_keyset_free(ctypes.c_void_p(h))
            t4 = time.perf_counter()
            t_new.append(t1 - t0)
            t_first.append(t2 - t1)
            t_second.append(t3 - t2)
            t_free.append(t4 - t3)
        us = lambda x, q: round(1e6 * float(np.percentile(x, q)), 1)  # noqa: E731
        stats.update({"contexts": a.contexts, "seconds": round(time.perf_counter() - t00, 4),
                      "new_us_p50": us(t_new, 50), "new_us_p99": us(t_new, 99),
                      "first_seal_us_p50": us(t_first, 50), "first_seal_us_p99": us(t_first, 99),
                      "second_seal_us_p50": us(t_second, 50), "second_seal_us_p99": us(t_second, 99),
                      "free_us_p50": us(t_free, 50), "free_us_p99": us(t_free, 99)})

    def bulk_while(th):
        """bulk launches back to back (at most 4 in flight) until the churn thread is done; GiB/s over the launches"""
        evs = []
        while th.is_alive() or len(evs) < 4:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(bulk)
            pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), bulk.cuda_stream)
            e1.record(bulk)
            evs.append((e0, e1))
            if len(evs) > 4:
                evs[-5][1].synchronize()
        torch.cuda.synchronize()
        return b.payload_bytes * len(evs) / (evs[0][0].elapsed_time(evs[-1][1]) / 1e3) / 2**30, len(evs)

    for _ in range(2):  # warm-up
        torch.cuda.synchronize()
        run_bulk()
        torch.cuda.synchronize()
    alone, loaded, rounds = [], [], []
    idle = {}
    churn(idle)  # the churn alone (no bulk): per-context costs on an idle device
    for _ in range(a.reps):
        torch.cuda.synchronize()
        e0, e1 = run_bulk()
        torch.cuda.synchronize()
        alone.append(b.payload_bytes * a.launches / (e0.elapsed_time(e1) / 1e3) / 2**30)
        stats = {}
        th = threading.Thread(target=churn, args=(stats,))
        th.start()
        v, nl = bulk_while(th)
        th.join()
        stats["bulk_launches"] = nl
        loaded.append(v)
        rounds.append(stats)
    ks.free()
    res = {"bulk_alone_GiBps": round(float(np.median(alone)), 2), "bulk_with_churn_GiBps": round(float(np.median(loaded)), 2),
           "ratio": round(float(np.median(loaded) / np.median(alone)), 4), "alone_all": [round(x, 1) for x in alone],
           "with_churn_all": [round(x, 1) for x in loaded], "bulk_launch_GiB": round(b.payload_bytes / 2**30, 2),
           "churn_idle_device": idle, "churn_under_bulk": rounds}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
