"""picotls_amd -- MI355X-native AES-GCM record engine for picotls (Python host mirror of the C ABI).

The product is the C ABI in ``include/picotls/mi355x.h`` (``libptls_mi355x.so``: hand-written gfx950 HIP kernels) and
the picotls plugin objects in ``include/picotls/mi355x_picotls.h``. This module binds the same entry points with
ctypes so that Python tests and ``bench.py`` drive exactly the code a C caller would, and mirrors picotls' AEAD
operator interface (``include/picotls.h:519-580, 2082-2164``; ``lib/picotls.c:6547-6601``):

* :data:`aes128gcm` / :data:`aes256gcm` -- algorithm descriptors (``ptls_mi355x_aes{128,256}gcm``)
* :func:`aead_new_direct` / :func:`aead_new` (traffic secret -> key, IV) -> :class:`AeadContext` with ``encrypt`` / ``encrypt_s`` / ``decrypt`` / ``get_iv`` /
  ``set_iv`` / ``xor_iv`` (``decrypt`` returns ``None`` where picotls returns ``SIZE_MAX``)
* :class:`Keyset`, :func:`seal_batch`, :func:`open_batch`, :func:`ecb_batch`, :func:`hp_mask_batch`,
  :func:`seal_batch_hp`, :func:`quiclb_batch` -- the batch extension.
* :class:`QuicLbCipher` -- mirror of ``ptls_mi355x_quiclb`` (fusion's ``ptls_fusion_quiclb``).

There is no CPU fallback: when the shared object or a gfx950 device is missing every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from .records import (CID_DTYPE, HP_DTYPE, QUICLB_MAX_LEN, QUICLB_MIN_LEN, RECORD_DTYPE, TLS_BAD_HEADER, TLS_BAD_MAC, TLS_OK, TLS_RESULT_DTYPE,  # noqa: F401
                      TLS_UNEXPECTED_MESSAGE, RecordBatch, shard_ranges)

_PKG = os.path.dirname(os.path.abspath(__file__))
# PTLS_MI355X_LIB: another build of the same engine (an A/B variant under tools/variants/) for the GPU suite
_DEFAULT_LIB = os.path.join(_PKG, "_lib", "libptls_mi355x.so")
LIB_PATH = os.environ.get("PTLS_MI355X_LIB") or _DEFAULT_LIB
PICOTLS_LIB_PATH = os.path.join(_PKG, "_lib", "libptls_mi355x_picotls.so")

# every function of include/picotls/mi355x.h (tests check the .so exports exactly these)
ABI_FUNCTIONS = (
    "ptls_mi355x_is_supported",
    "ptls_mi355x_keyset_new",
    "ptls_mi355x_keyset_free",
    "ptls_mi355x_keyset_size",
    "ptls_mi355x_keyset_key_size",
    "ptls_mi355x_keyset_device",
    "ptls_mi355x_keyset_get_iv",
    "ptls_mi355x_keyset_set_iv",
    "ptls_mi355x_keyset_update",
    "ptls_mi355x_keyset_set_schedule",
    "ptls_mi355x_keyset_set_constant_time",
    "ptls_mi355x_keyset_get_constant_time",
    "ptls_mi355x_seal_batch",
    "ptls_mi355x_open_batch",
    "ptls_mi355x_seal_tls_records",
    "ptls_mi355x_open_tls_records",
    "ptls_mi355x_seal_tls12_records",
    "ptls_mi355x_open_tls12_records",
    "ptls_mi355x_ecb_batch",
    "ptls_mi355x_hp_mask_batch",
    "ptls_mi355x_seal_batch_hp",
    "ptls_mi355x_quiclb_batch",
    "ptls_mi355x_quiclb_transform",
    "ptls_mi355x_encrypt",
    "ptls_mi355x_encrypt_v",
    "ptls_mi355x_encrypt_s",
    "ptls_mi355x_decrypt",
    "ptls_mi355x_encrypt_block",
    "ptls_mi355x_encrypt_blocks",
    "ptls_mi355x_staging_bytes",
    "ptls_mi355x_release_staging",
    "ptls_mi355x_last_error",
)
# include/picotls/mi355x_debug.h: test and measurement hooks (not the picotls boundary)
DEBUG_FUNCTIONS = (
    "ptls_mi355x_debug_counters",
    "ptls_mi355x_debug_inject_error",
    "ptls_mi355x_debug_clock_sample",
    "ptls_mi355x_debug_wallclock_khz",
    "ptls_mi355x_debug_kernel_clock",
    "ptls_mi355x_debug_kernel_clock_count",
)

SIZE_MAX = ctypes.c_size_t(-1).value
_lib = None


class EngineError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Loads libptls_mi355x.so (no device calls). Raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise EngineError(f"{path} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    if path == _DEFAULT_LIB:  # the in-tree build must be of the sources beside it (build.py's digest stamp)
        from . import build as _b

        if os.path.exists(_b.ENGINE_SRCS[0]) and _b._stamp(path) != _b.engine_digest():
            raise EngineError(f"{path} was not built from the current sources (its {path}.sha256 differs): rebuild with "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    vp, sz, u64, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int
    lib.ptls_mi355x_is_supported.restype = ci
    lib.ptls_mi355x_keyset_new.argtypes = [vp, vp, sz, sz]
    lib.ptls_mi355x_keyset_new.restype = vp
    lib.ptls_mi355x_keyset_free.argtypes = [vp]
    lib.ptls_mi355x_keyset_size.argtypes = [vp]
    lib.ptls_mi355x_keyset_size.restype = sz
    lib.ptls_mi355x_keyset_key_size.argtypes = [vp]
    lib.ptls_mi355x_keyset_key_size.restype = sz
    lib.ptls_mi355x_keyset_device.argtypes = [vp]
    lib.ptls_mi355x_keyset_device.restype = ci
    lib.ptls_mi355x_staging_bytes.restype = sz
    lib.ptls_mi355x_release_staging.restype = None
    lib.ptls_mi355x_keyset_get_iv.argtypes = [vp, sz, vp]
    lib.ptls_mi355x_keyset_set_iv.argtypes = [vp, sz, vp]
    lib.ptls_mi355x_keyset_update.argtypes = [vp, vp, vp, vp, sz]
    lib.ptls_mi355x_keyset_set_schedule.argtypes = [vp, ci]
    lib.ptls_mi355x_keyset_set_constant_time.argtypes = [vp, ci]
    lib.ptls_mi355x_keyset_get_constant_time.argtypes = [vp]
    lib.ptls_mi355x_keyset_get_constant_time.restype = ci
    lib.ptls_mi355x_seal_batch.argtypes = [vp, vp, sz, vp, vp, vp, vp]
    lib.ptls_mi355x_open_batch.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp]
    lib.ptls_mi355x_ecb_batch.argtypes = [vp, vp, vp, vp, sz, vp]
    lib.ptls_mi355x_hp_mask_batch.argtypes = [vp, vp, sz, vp, vp, vp]
    lib.ptls_mi355x_seal_tls_records.argtypes = [vp, vp, sz, vp, vp, vp]
    lib.ptls_mi355x_open_tls_records.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp]
    lib.ptls_mi355x_seal_tls12_records.argtypes = [vp, vp, sz, vp, vp, vp]
    lib.ptls_mi355x_open_tls12_records.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp]
    lib.ptls_mi355x_seal_batch_hp.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp, vp, vp]
    lib.ptls_mi355x_encrypt.argtypes = [vp, sz, vp, vp, sz, u64, vp, sz]
    lib.ptls_mi355x_encrypt_v.argtypes = [vp, sz, vp, vp, sz, u64, vp, sz]
    lib.ptls_mi355x_encrypt_s.argtypes = [vp, sz, vp, vp, sz, u64, vp, sz, vp, sz, sz, vp]
    lib.ptls_mi355x_decrypt.argtypes = [vp, sz, vp, vp, sz, u64, vp, sz]
    lib.ptls_mi355x_decrypt.restype = sz
    lib.ptls_mi355x_encrypt_block.argtypes = [vp, sz, vp, vp]
    lib.ptls_mi355x_encrypt_blocks.argtypes = [vp, sz, vp, vp, sz]
    lib.ptls_mi355x_quiclb_batch.argtypes = [vp, vp, sz, vp, vp, vp]
    lib.ptls_mi355x_quiclb_transform.argtypes = [vp, sz, vp, vp, sz, ci]
    lib.ptls_mi355x_last_error.restype = ctypes.c_char_p
    lib.ptls_mi355x_debug_counters.argtypes = [vp, ci]
    lib.ptls_mi355x_debug_inject_error.restype = ci
    lib.ptls_mi355x_debug_clock_sample.argtypes = [vp, vp]
    lib.ptls_mi355x_debug_wallclock_khz.restype = ci
    lib.ptls_mi355x_debug_kernel_clock.argtypes = [vp, ctypes.c_uint]
    lib.ptls_mi355x_debug_kernel_clock_count.restype = ci
    _lib = lib
    return lib


def _err(what: str) -> EngineError:
    msg = load_library().ptls_mi355x_last_error()
    return EngineError(f"{what}: {msg.decode() if msg else 'unknown error'}")


def is_supported() -> bool:
    return bool(load_library().ptls_mi355x_is_supported())


def _buf(b) -> ctypes.c_void_p | None:
    if b is None or len(b) == 0:
        return None
    if isinstance(b, bytes):
        return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)
    if isinstance(b, bytearray):
        return ctypes.c_void_p(ctypes.addressof((ctypes.c_char * len(b)).from_buffer(b)))
    if isinstance(b, np.ndarray):
        return ctypes.c_void_p(b.ctypes.data)
    raise TypeError(type(b))


# ------------------------------------------------------------------------------------------------ keysets / batches


class Keyset:
    """N AES-GCM traffic keys resident on the current device (ptls_mi355x_keyset_new)."""

    def __init__(self, keys: bytes | np.ndarray, ivs: bytes | np.ndarray, key_size: int):
        lib = load_library()
        keys = np.frombuffer(bytes(keys), dtype=np.uint8) if not isinstance(keys, np.ndarray) else np.ascontiguousarray(keys, np.uint8)
        ivs = np.frombuffer(bytes(ivs), dtype=np.uint8) if not isinstance(ivs, np.ndarray) else np.ascontiguousarray(ivs, np.uint8)
        if key_size not in (16, 32) or keys.size % key_size or ivs.size != keys.size // key_size * 12:
            raise ValueError("keys must be n*key_size bytes and ivs n*12 bytes")
        self.n = keys.size // key_size
        self.key_size = key_size
        h = lib.ptls_mi355x_keyset_new(_buf(keys), _buf(ivs), self.n, key_size)
        if not h:
            raise _err("ptls_mi355x_keyset_new")
        self.handle = ctypes.c_void_p(h)

    def free(self):
        if getattr(self, "handle", None):
            load_library().ptls_mi355x_keyset_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def get_iv(self, idx: int = 0) -> bytes:
        out = bytearray(12)
        if load_library().ptls_mi355x_keyset_get_iv(self.handle, idx, _buf(out)) != 0:
            raise _err("get_iv")
        return bytes(out)

    def set_iv(self, iv: bytes, idx: int = 0) -> None:
        if load_library().ptls_mi355x_keyset_set_iv(self.handle, idx, _buf(bytes(iv))) != 0:
            raise _err("set_iv")

    def update(self, key_idx, keys: bytes, ivs: bytes) -> None:
        """Rekeys entries key_idx (ptls_mi355x_keyset_update), e.g. after a TLS 1.3 KeyUpdate."""
        idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
        k = np.frombuffer(bytes(keys), np.uint8)
        v = np.frombuffer(bytes(ivs), np.uint8)
        if k.size != idx.size * self.key_size or v.size != idx.size * 12:
            raise ValueError("keys must be n*key_size bytes and ivs n*12 bytes")
        if load_library().ptls_mi355x_keyset_update(self.handle, _buf(idx), _buf(k), _buf(v), idx.size) != 0:
            raise _err("keyset_update")

    def set_constant_time(self, on: bool = True) -> None:
        """Constant-time GHASH variant (ptls_mi355x_keyset_set_constant_time)."""
        if load_library().ptls_mi355x_keyset_set_constant_time(self.handle, 1 if on else 0) != 0:
            raise _err("set_constant_time")

    @property
    def constant_time(self) -> bool:
        return bool(load_library().ptls_mi355x_keyset_get_constant_time(self.handle))

    SCHEDULES = {"auto": 0, "lockstep": 1, "chunked": 2}

    def set_schedule(self, schedule: str, allow_variable_time: bool = False) -> None:
        """Batch schedule (ptls_mi355x_keyset_set_schedule): "auto", "lockstep" or "chunked".

        The lockstep schedule (the round-1 kernel, kept for comparison) has data-dependent LDS bank conflicts, so the
        engine never runs it for a constant-time keyset (every keyset is one by default since round 4): the C call
        records the schedule and such a keyset keeps the chunked kernels. Here asking for "lockstep" on a constant-time
        keyset raises, unless allow_variable_time=True, which (after the schedule is set) turns the keyset's
        constant-time setting off so that the lockstep kernel is the one that runs."""
        if schedule not in self.SCHEDULES:
            raise ValueError(f"unknown schedule {schedule!r}")
        lockstep_ct = schedule == "lockstep" and self.constant_time
        if lockstep_ct and not allow_variable_time:
            raise EngineError("set_schedule('lockstep') on a constant-time keyset: the lockstep kernel is not constant-time; "
                              "pass allow_variable_time=True to turn the keyset's constant-time setting off")
        if load_library().ptls_mi355x_keyset_set_schedule(self.handle, self.SCHEDULES[schedule]) != 0:
            raise _err("set_schedule")
        if lockstep_ct:
            self.set_constant_time(False)


def seal_batch(ks: Keyset, recs_ptr: int, nrecs: int, in_ptr: int, aad_ptr: int, out_ptr: int, stream: int = 0) -> None:
    """Device pointers (ints, e.g. torch ``tensor.data_ptr()``); asynchronous on ``stream`` (a hipStream_t)."""
    if load_library().ptls_mi355x_seal_batch(ks.handle, recs_ptr, nrecs, in_ptr, aad_ptr or None, out_ptr, stream or None) != 0:
        raise _err("ptls_mi355x_seal_batch")


def open_batch(ks: Keyset, recs_ptr: int, nrecs: int, in_ptr: int, aad_ptr: int, out_ptr: int, ok_ptr: int,
               stream: int = 0) -> None:
    if load_library().ptls_mi355x_open_batch(ks.handle, recs_ptr, nrecs, in_ptr, aad_ptr or None, out_ptr, ok_ptr,
                                             stream or None) != 0:
        raise _err("ptls_mi355x_open_batch")


def ecb_batch(ks: Keyset, key_idx_ptr: int, in_ptr: int, out_ptr: int, nblocks: int, stream: int = 0) -> None:
    if load_library().ptls_mi355x_ecb_batch(ks.handle, key_idx_ptr or None, in_ptr, out_ptr, nblocks, stream or None) != 0:
        raise _err("ptls_mi355x_ecb_batch")


def seal_tls_records(ks: Keyset, recs_ptr: int, nrecs: int, in_ptr: int, out_ptr: int, stream: int = 0) -> None:
    """TLS 1.3 wire records (header || ciphertext || tag) from payloads + inner content types (flags); device pointers."""
    if load_library().ptls_mi355x_seal_tls_records(ks.handle, recs_ptr, nrecs, in_ptr, out_ptr, stream or None) != 0:
        raise _err("ptls_mi355x_seal_tls_records")


def open_tls_records(ks: Keyset, recs_ptr: int, nrecs: int, in_ptr: int, out_ptr: int, ok_ptr: int, results_ptr: int = 0,
                     stream: int = 0) -> None:
    """Opens TLS 1.3 wire records and strips the inner type and padding (TLS_RESULT_DTYPE results); device pointers."""
    if load_library().ptls_mi355x_open_tls_records(ks.handle, recs_ptr, nrecs, in_ptr, out_ptr, ok_ptr, results_ptr or None,
                                                   stream or None) != 0:
        raise _err("ptls_mi355x_open_tls_records")


def seal_tls12_records(ks: Keyset, recs_ptr: int, nrecs: int, in_ptr: int, out_ptr: int, stream: int = 0) -> None:
    """TLS 1.2 wire records (header || explicit nonce || ciphertext || tag) from explicit nonce || payload; device pointers."""
    if load_library().ptls_mi355x_seal_tls12_records(ks.handle, recs_ptr, nrecs, in_ptr, out_ptr, stream or None) != 0:
        raise _err("ptls_mi355x_seal_tls12_records")


def open_tls12_records(ks: Keyset, recs_ptr: int, nrecs: int, in_ptr: int, out_ptr: int, ok_ptr: int, results_ptr: int = 0,
                       stream: int = 0) -> None:
    """Opens TLS 1.2 wire records (TLS_RESULT_DTYPE results: content type, length, status); device pointers."""
    if load_library().ptls_mi355x_open_tls12_records(ks.handle, recs_ptr, nrecs, in_ptr, out_ptr, ok_ptr, results_ptr or None,
                                                     stream or None) != 0:
        raise _err("ptls_mi355x_open_tls12_records")


def hp_mask_batch(hp_ks: Keyset, hp_ptr: int, n: int, base_ptr: int, masks_ptr: int, stream: int = 0) -> None:
    """QUIC header-protection masks (HP_DTYPE entries); device pointers."""
    if load_library().ptls_mi355x_hp_mask_batch(hp_ks.handle, hp_ptr, n, base_ptr, masks_ptr, stream or None) != 0:
        raise _err("ptls_mi355x_hp_mask_batch")


def seal_batch_hp(ks: Keyset, recs_ptr: int, nrecs: int, in_ptr: int, aad_ptr: int, out_ptr: int, hp_ks: Keyset,
                  hp_ptr: int, masks_ptr: int, stream: int = 0) -> None:
    """seal_batch followed by the header-protection masks of samples in the sealed output (fusion's supp)."""
    if load_library().ptls_mi355x_seal_batch_hp(ks.handle, recs_ptr, nrecs, in_ptr, aad_ptr or None, out_ptr, hp_ks.handle,
                                                hp_ptr, masks_ptr, stream or None) != 0:
        raise _err("ptls_mi355x_seal_batch_hp")


def quiclb_batch(ks: Keyset, cids_ptr: int, n: int, in_ptr: int, out_ptr: int, stream: int = 0) -> None:
    """QUIC-LB CID encryption / decryption (CID_DTYPE entries, AES-128 keyset); device pointers."""
    if load_library().ptls_mi355x_quiclb_batch(ks.handle, cids_ptr, n, in_ptr, out_ptr, stream or None) != 0:
        raise _err("ptls_mi355x_quiclb_batch")


# ------------------------------------------------------------------------------------------------ picotls mirror


@dataclass(frozen=True)
class AeadAlgorithm:
    """Mirror of ptls_aead_algorithm_t (include/picotls.h:519-580) for ptls_mi355x_aes{128,256}gcm."""

    name: str
    key_size: int
    iv_size: int = 12
    tag_size: int = 16
    confidentiality_limit: int = 0x2000000  # PTLS_AESGCM_CONFIDENTIALITY_LIMIT, include/picotls.h:89
    integrity_limit: int = 0x40000000000000  # PTLS_AESGCM_INTEGRITY_LIMIT, include/picotls.h:90
    tls12_fixed_iv_size: int = 0
    tls12_record_iv_size: int = 0
    non_temporal: int = 0
    align_bits: int = 0


aes128gcm = AeadAlgorithm("AES128-GCM", 16)
aes256gcm = AeadAlgorithm("AES256-GCM", 32)


class AeadContext:
    """Mirror of ptls_aead_context_t created by ptls_aead_new_direct (lib/picotls.c:6553-6568)."""

    def __init__(self, algo: AeadAlgorithm, is_enc: bool, key: bytes, iv: bytes):
        if len(key) != algo.key_size or len(iv) != algo.iv_size:
            raise ValueError("key / iv size mismatch")
        self.algo = algo
        self.is_enc = is_enc
        self._iv = bytes(iv)
        self.ks = Keyset(key, iv, algo.key_size)
        # as the picotls objects (ptls_mi355x.c aesgcm_setup): constant-time unless PTLS_MI355X_CONSTANT_TIME=0
        self.ks.set_constant_time(os.environ.get("PTLS_MI355X_CONSTANT_TIME") != "0")

    def free(self):
        self.ks.free()

    # do_get_iv / do_set_iv / ptls_aead_xor_iv (lib/picotls.c:6576-6585)
    def get_iv(self) -> bytes:
        return self._iv

    def set_iv(self, iv: bytes) -> None:
        self._iv = bytes(iv)
        self.ks.set_iv(self._iv)

    def xor_iv(self, data: bytes) -> None:
        iv = bytearray(self._iv)
        for i, b in enumerate(data):
            iv[i] ^= b
        self.set_iv(bytes(iv))

    # ptls_aead_encrypt (include/picotls.h:2102-2107): returns ciphertext || tag
    def encrypt(self, pt: bytes, seq: int, aad: bytes = b"") -> bytes:
        out = bytearray(len(pt) + self.algo.tag_size)
        if load_library().ptls_mi355x_encrypt(self.ks.handle, 0, _buf(out), _buf(bytes(pt)), len(pt), seq,
                                             _buf(bytes(aad)), len(aad)) != 0:
            raise _err("ptls_mi355x_encrypt")
        return bytes(out)

    # ptls_aead_encrypt_v (include/picotls.h:2115-2119): the vectors sealed as one record
    def encrypt_v(self, vecs: list, seq: int, aad: bytes = b"") -> bytes:
        bufs = [bytes(v) for v in vecs]
        arr = (ctypes.c_void_p * (2 * max(len(bufs), 1)))()
        for i, b in enumerate(bufs):
            arr[2 * i] = ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value if b else None
            arr[2 * i + 1] = len(b)
        total = sum(len(b) for b in bufs)
        out = bytearray(total + self.algo.tag_size)
        if load_library().ptls_mi355x_encrypt_v(self.ks.handle, 0, _buf(out), ctypes.cast(arr, ctypes.c_void_p), len(bufs), seq,
                                               _buf(bytes(aad)), len(aad)) != 0:
            raise _err("ptls_mi355x_encrypt_v")
        return bytes(out)

    # ptls_aead_encrypt_s with a header-protection cipher (include/picotls.h:2109-2113, lib/fusion.c:425-430,636-651):
    # the mask of the sealed sample at sample_off, computed in the seal's round trip (ptls_mi355x_encrypt_s)
    def encrypt_s(self, pt: bytes, seq: int, aad: bytes, hp: "CtrCipher", sample_off: int) -> tuple[bytes, bytes]:
        out = bytearray(len(pt) + self.algo.tag_size)
        mask = bytearray(16)
        if load_library().ptls_mi355x_encrypt_s(self.ks.handle, 0, _buf(out), _buf(bytes(pt)), len(pt), seq, _buf(bytes(aad)),
                                               len(aad), hp.ks.handle, 0, sample_off, _buf(mask)) != 0:
            raise _err("ptls_mi355x_encrypt_s")
        return bytes(out), bytes(mask)

    # ptls_aead_decrypt (include/picotls.h:2160-2164): plaintext, or None for SIZE_MAX
    def decrypt(self, ct_tag: bytes, seq: int, aad: bytes = b"") -> bytes | None:
        if len(ct_tag) < 16:
            return None
        out = bytearray(len(ct_tag) - 16 + 1)
        r = load_library().ptls_mi355x_decrypt(self.ks.handle, 0, _buf(out), _buf(bytes(ct_tag)), len(ct_tag), seq,
                                               _buf(bytes(aad)), len(aad))
        if r == SIZE_MAX:
            return None
        return bytes(out[:r])


class CtrCipher:
    """Mirror of ptls_mi355x_aes{128,256}ctr (fusion's 16-byte AES-CTR, lib/fusion.c:1051-1101)."""

    def __init__(self, key: bytes):
        self.ks = Keyset(key, bytes(12), len(key))

    def mask(self, iv16: bytes) -> bytes:
        out = bytearray(16)
        if load_library().ptls_mi355x_encrypt_block(self.ks.handle, 0, _buf(out), _buf(bytes(iv16))) != 0:
            raise _err("ptls_mi355x_encrypt_block")
        return bytes(out)


class QuicLbCipher:
    """Mirror of ptls_cipher_new(&ptls_mi355x_quiclb, is_enc, key) + ptls_cipher_encrypt (t/quiclb.c:36-45): the QUIC-LB
    CID cipher of lib/quiclb-impl.h, one CID of 7..19 bytes per call."""

    key_size = 16
    block_size = 8  # PTLS_QUICLB_DEFAULT_BLOCK_SIZE, include/picotls.h:119-122

    def __init__(self, is_enc: bool, key: bytes):
        if len(key) != 16:
            raise ValueError("QUIC-LB keys are 16 bytes (PTLS_QUICLB_KEY_SIZE)")
        self.is_enc = is_enc
        self.ks = Keyset(key, bytes(12), 16)

    def encrypt(self, data: bytes) -> bytes:
        if not QUICLB_MIN_LEN <= len(data) <= QUICLB_MAX_LEN:
            raise ValueError("QUIC-LB transforms 7..19 bytes")
        out = bytearray(len(data))
        if load_library().ptls_mi355x_quiclb_transform(self.ks.handle, 0, _buf(out), _buf(bytes(data)), len(data),
                                                       1 if self.is_enc else 0) != 0:
            raise _err("ptls_mi355x_quiclb_transform")
        return bytes(out)


def staging_bytes() -> int:
    """Pinned host bytes held by the per-record path's staging pools (ptls_mi355x_staging_bytes)."""
    return int(load_library().ptls_mi355x_staging_bytes())


def release_staging() -> None:
    """Frees the idle staging buffers (ptls_mi355x_release_staging)."""
    load_library().ptls_mi355x_release_staging()


# ------------------------------------------------------------------------------------------------ debug hooks


COUNTER_NAMES = ("chunked", "spread", "seal_hp", "w8_tree", "w8_serial", "lockstep", "span", "w8_g4")


def debug_counters(reset: bool = False) -> dict:
    """ptls_mi355x_debug_counters: {"launches": {kind: n}, "runs": {kind: n}} (chunked kinds: EXT 0..4). Waits for the
    device."""
    out = (ctypes.c_uint64 * 16)()
    if load_library().ptls_mi355x_debug_counters(ctypes.cast(out, ctypes.c_void_p), 1 if reset else 0) != 0:
        raise _err("ptls_mi355x_debug_counters")
    runs = dict(zip(COUNTER_NAMES[:5], out[8:13]))
    runs["w8_g4"] = out[15]  # (of the w8_serial runs: whole runs in 4-lane groups)
    runs["w8_mk"] = out[14]  # (of the w8_serial runs: multi-key runs, round 6)
    return {"launches": dict(zip(COUNTER_NAMES[:7], out[:7])), "runs": runs}


def debug_inject_error() -> int:
    """Leaves a HIP error as this thread's last error (ptls_mi355x_debug_inject_error); returns its code."""
    return int(load_library().ptls_mi355x_debug_inject_error())


def debug_clock_sample(dev_ptr: int, stream: int = 0) -> None:
    """Writes (s_memtime, s_memrealtime, XCC id) of the XCD the probe wave ran on (the id is out[2]) to 3 x u64 at dev_ptr,
    in stream order."""
    if load_library().ptls_mi355x_debug_clock_sample(dev_ptr, stream or None) != 0:
        raise _err("ptls_mi355x_debug_clock_sample")


def debug_wallclock_khz() -> int:
    return int(load_library().ptls_mi355x_debug_wallclock_khz())


def debug_kernel_clock(dev_ptr: int, cap: int) -> None:
    """From the next launch on, workgroup 0 of each chunked launch appends (memtime start, end, realtime start, end) as
    4 x u64 to the device buffer at dev_ptr (room for cap launches); dev_ptr 0 stops (ptls_mi355x_debug_kernel_clock)."""
    if load_library().ptls_mi355x_debug_kernel_clock(dev_ptr or None, cap if dev_ptr else 0) != 0:
        raise _err("ptls_mi355x_debug_kernel_clock")


def debug_kernel_clock_count() -> int:
    """Launches sampled since the last debug_kernel_clock (may exceed the buffer's cap)."""
    n = int(load_library().ptls_mi355x_debug_kernel_clock_count())
    if n < 0:
        raise _err("ptls_mi355x_debug_kernel_clock_count")
    return n


def aead_new_direct(algo: AeadAlgorithm, is_enc: bool, key: bytes, iv: bytes) -> AeadContext:
    return AeadContext(algo, is_enc, key, iv)


def aead_new(algo: AeadAlgorithm, hash_name: str, is_enc: bool, secret: bytes, label_prefix: str | None = None) -> AeadContext:
    """ptls_aead_new (lib/picotls.c:6529-6551): traffic key and IV from a secret (get_traffic_keys), then
    ptls_aead_new_direct. hash_name is the suite hash ("sha256", "sha384")."""
    from .keyschedule import traffic_keys

    key, iv = traffic_keys(algo.key_size, hash_name, secret, algo.iv_size, label_prefix)
    return AeadContext(algo, is_enc, key, iv)
