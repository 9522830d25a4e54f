import ctypes, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmb.so"))
lib.ptls_mi355x_keyset_new.restype = ctypes.c_void_p
lib.ptls_mi355x_keyset_new.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t]
lib.mb_keyptr.restype = ctypes.c_void_p
lib.mb_keyptr.argtypes = [ctypes.c_void_p]
lib.mb_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
key = (ctypes.c_ubyte * 16)(*range(16)); iv = (ctypes.c_ubyte * 12)()
ks = lib.ptls_mi355x_keyset_new(key, iv, 1, 16)
kp = lib.mb_keyptr(ks)
grid = 256
out = torch.empty(grid * 1024, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for which, name, nbs, iters in ((0, "aes", (1, 2, 4), 2000), (1, "ghash", (1, 2), 4000)):
    for nb in nbs:
        lib.mb_run(which, nb, kp, 10, out.data_ptr(), grid, s); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); lib.mb_run(which, nb, kp, iters, out.data_ptr(), grid, s); e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        blocks = grid * 1024 * iters * nb
        per_cu = blocks / grid / (ms * 1e-3)
        print(f"{name} NB={nb}: {ms:.2f} ms, {blocks / ms / 1e6:.2f} G blocks/s, {per_cu / 2.0e9:.3f} blocks/clk/CU @2GHz, "
              f"= {blocks * 16 / ms / 1e6:.0f} GB/s of 16-B blocks")
