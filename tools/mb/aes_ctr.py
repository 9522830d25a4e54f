#!/usr/bin/env python3
"""T-table vs bitsliced AES-CTR (tools/mb/aes_ctr.hip) on the same 1 GiB buffer: identical output, GB/s, G blocks/s.

    python tools/mb/aes_ctr.py [--key-size 16] [--blocks 67108864]
"""
import argparse
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key-size", type=int, default=16)
    ap.add_argument("--blocks", type=int, default=1 << 26)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "libaesctr.so"))
    lib.aesctr_setup.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.aesctr_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    key = (ctypes.c_ubyte * 32)(*range(0x40, 0x60))
    assert lib.aesctr_setup(key, a.key_size) == 0
    n = a.blocks
    g = torch.Generator(device="cuda").manual_seed(1)
    src = torch.randint(0, 256, (16 * n,), dtype=torch.uint8, device="cuda", generator=g)
    outs = {}
    s = torch.cuda.current_stream().cuda_stream
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    for which, name, grid in ((0, "T-table (LDS)", ncu), (1, "bitsliced (VALU)", ncu * 8)):
        out = torch.empty_like(src)
        assert lib.aesctr_run(which, src.data_ptr(), out.data_ptr(), n, grid, s) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            lib.aesctr_run(which, src.data_ptr(), out.data_ptr(), n, grid, s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        outs[name] = out
        print(f"AES-{8 * a.key_size}-CTR {name:18s}: {ms:7.3f} ms  {16 * n / ms / 1e6:8.1f} GB/s  "
              f"{n / ms / 1e6:7.2f} G blocks/s  ({n / ms * 1e3 / ncu / 2.4e9:.3f} blocks/clk/CU at 2.4 GHz)")
    a_, b_ = outs.values()
    print("identical output:", bool(torch.equal(a_, b_)))


if __name__ == "__main__":
    main()
