#!/usr/bin/env python3
"""Phase breakdown of the chunked kernel from a -DENGINE_PROFILE=1 build (tools/mkvariant.sh prof -DENGINE_PROFILE=1).

    python tools/prof_phases.py tools/variants/lib_prof.so --workload mixed --records 1048576
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotls_amd.workloads import WORKLOADS, payload_torch  # noqa: E402
from ab import bind  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--workload", default="mixed")
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--schedule", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    lib = bind(a.lib)
    lib.ptls_mi355x_debug_profile.argtypes = [ctypes.c_void_p, ctypes.c_int]
    wl = WORKLOADS[a.workload].scaled(a.records)
    b = wl.descriptors(0, wl.nrecs)
    keys, ivs = wl.keys()
    dev = torch.device("cuda:0")
    d_seal = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(wl.aad_arena(b, 0)).to(dev)
    d_pt = payload_torch(wl.seed, b.pt_bytes, dev)
    sealed = torch.empty(b.sealed_bytes, dtype=torch.uint8, device=dev)
    ks = ctypes.c_void_p(lib.ptls_mi355x_keyset_new(keys.ctypes.data, ivs.ctypes.data, wl.nkeys, wl.key_size))
    lib.ptls_mi355x_keyset_set_schedule(ks, a.schedule)
    s = torch.cuda.current_stream().cuda_stream
    prof = (ctypes.c_ulonglong * 24)()  # PROF_SLOTS
    lib.ptls_mi355x_seal_batch(ks, d_seal.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), sealed.data_ptr(), s)
    torch.cuda.synchronize()
    lib.ptls_mi355x_debug_profile(prof, 1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.reps):
        lib.ptls_mi355x_seal_batch(ks, d_seal.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), sealed.data_ptr(), s)
    ev[1].record()
    torch.cuda.synchronize()
    lib.ptls_mi355x_debug_profile(prof, 1)
    p = list(prof)
    ms = ev[0].elapsed_time(ev[1]) / a.reps
    runs = max(p[6], 1)
    tot = p[0] + p[1] + p[2] + p[3]
    print(f"{a.workload} n={a.records} schedule={a.schedule}: seal {ms:.3f} ms, runs/launch {p[6] / a.reps:.0f}, "
          f"units/run {p[5] / runs:.1f}, table builds/launch {p[7] / a.reps:.0f}")
    for i, name in enumerate(["run setup", "table build", "unit loop", "prologue"]):
        print(f"  {name:12s} {p[i] / runs:10.0f} cycles/run  {100 * p[i] / max(tot, 1):5.1f} %")
    if p[10]:
        print("  prologue split (cycles/workgroup): AES tables (waves 1-15) %.0f | first run scan (wave 0) %.0f" %
              (p[8] / p[10], p[9] / p[10]))
    if p[12]:
        print(f"  unit tails (partial store, record combine, tag): {p[11] / p[12]:.0f} cycles per wave-round, "
              f"{100 * p[11] / 16 / max(p[2], 1):.1f} % of the unit loop")
    if p[14] and not p[15]:  # (no MK run: the tail scans, ENGINE_PROFILE slots 13-14)
        print(f"  tail scans: {p[13] / runs:.0f} cycles per run; the scanning wave then waits {p[14] / runs:.0f} cycles "
              f"at the barrier")
    elif p[14]:
        print(f"  MK claims: {p[13] / p[14]:.0f} cycles per claim ({p[14] / runs:.1f} a run); early scans "
              f"{p[15] / runs:.0f} cycles per run")
    if p[19]:
        seg = p[16] + p[17] + p[18]
        print(f"  segments (serial W8 kernels, per wave): {p[19] / a.reps:.0f} a launch; setup {p[16] / p[19]:.0f}, steps "
              f"{p[17] / p[19]:.0f}, end {p[18] / p[19]:.0f} cycles each ({100 * p[16] / seg:.1f} / {100 * p[17] / seg:.1f} / "
              f"{100 * p[18] / seg:.1f} %)")
        print(f"  steps per segment {p[20] / p[19]:.2f}, of them steady {p[21] / p[19]:.2f} ({100 * p[21] / max(p[20], 1):.1f} %)")
        if p[22] and p[21] and p[20] > p[21]:
            print(f"  cycles per steady step {p[22] / p[21]:.0f}, per other step {(p[17] - p[22]) / (p[20] - p[21]):.0f}; "
                  f"the other steps take {100 * (p[17] - p[22]) / p[17]:.1f} % of the steps' time")
    waves = 16
    print(f"  wave idle at unit-loop barrier: {p[4] / runs / waves:.0f} cycles/run/wave "
          f"({100 * p[4] / waves / max(p[2], 1):.1f} % of the unit loop)")


if __name__ == "__main__":
    main()
