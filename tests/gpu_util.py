"""Helpers for the -m gpu tests: run a RecordBatch through the engine's C ABI with torch-owned device buffers."""
import numpy as np
import torch

import picotls_amd as pa


def dev(a: np.ndarray) -> torch.Tensor:
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy())
    return t.to("cuda:0")


def empty(nbytes: int, fill: int = 0) -> torch.Tensor:
    t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device="cuda:0")
    t.fill_(fill)
    return t


def gpu_seal(ks: pa.Keyset, recs: np.ndarray, pt: np.ndarray, aad: np.ndarray, out_bytes: int, out_fill: int = 0):
    d_recs, d_pt, d_aad = dev(recs), dev(pt if pt.size else np.zeros(1, np.uint8)), dev(aad if aad.size else np.zeros(1, np.uint8))
    d_out = empty(out_bytes, out_fill)
    pa.seal_batch(ks, d_recs.data_ptr(), len(recs), d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_out[:out_bytes].cpu().numpy()


def gpu_open(ks: pa.Keyset, recs: np.ndarray, sealed: np.ndarray, aad: np.ndarray, out_bytes: int, out_fill: int = 0):
    d_recs, d_in, d_aad = dev(recs), dev(sealed if sealed.size else np.zeros(1, np.uint8)), dev(aad if aad.size else np.zeros(1, np.uint8))
    d_out = empty(out_bytes, out_fill)
    d_ok = empty(len(recs), 0xAA)
    pa.open_batch(ks, d_recs.data_ptr(), len(recs), d_in.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), d_ok.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_out[:out_bytes].cpu().numpy(), d_ok[:len(recs)].cpu().numpy()
