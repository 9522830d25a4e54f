"""TEST INFRASTRUCTURE ONLY -- the checkers for the MI355X AES-GCM record engine.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this package, and
only to *check* or *time the reference*; the product (``picotls_amd``) never routes through it.

Two checkers:

* :class:`GcmOracle` -- ``oracle/gcm_ref.c``, a plain-C restatement of SP 800-38D AES-GCM with picotls' TLS 1.3
  nonce rule (see the file header for the reference file:line each function follows).
* :class:`FusionRef` -- picotls' own ``lib/fusion.c`` compiled unmodified from ``/root/reference`` by
  ``oracle/Makefile`` into ``oracle/_ref/libfusion_ref.so`` (driven through ``ptls_aead_new_direct`` /
  ``ptls_aead_encrypt`` / ``ptls_aead_decrypt``, ``t/ptlsbench.c:88-185``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")

# numpy view of the 40-byte record descriptor (include/picotls/mi355x.h, ptls_mi355x_record_t)
RECORD_DTYPE = np.dtype(
    [
        ("in_off", "<u8"),
        ("out_off", "<u8"),
        ("seq", "<u8"),
        ("aad_off", "<u4"),
        ("len", "<u4"),
        ("key_idx", "<u4"),
        ("aad_len", "<u2"),
        ("flags", "<u2"),
    ]
)
assert RECORD_DTYPE.itemsize == 40


def build(force: bool = False) -> None:
    """Builds oracle/_ref (the restatement always; lib/fusion.c only where /root/reference exists)."""
    target = os.path.join(REF_DIR, "libgcm_oracle.so")
    if force or not os.path.exists(target) or (
        os.path.exists("/root/reference/lib/fusion.c") and not os.path.exists(os.path.join(REF_DIR, "libfusion_ref.so"))
    ):
        subprocess.run(["make", "-s", "-C", HERE], check=True)


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, (bytes, bytearray)):
        a = np.frombuffer(a, dtype=np.uint8)
    return a.ctypes.data_as(ctypes.c_void_p)


class GcmOracle:
    """ctypes front-end of oracle/gcm_ref.c."""

    def __init__(self):
        path = os.path.join(REF_DIR, "libgcm_oracle.so")
        if not os.path.exists(path):
            build()
        lib = ctypes.CDLL(path)
        vp, sz, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
        lib.oracle_aes_encrypt.argtypes = [vp, sz, vp, vp]
        lib.oracle_gf128_mul.argtypes = [vp, vp, vp]
        lib.oracle_ghash.argtypes = [vp, vp, vp, sz]
        lib.oracle_gcm_seal.argtypes = [vp, sz, vp, u64, vp, sz, vp, sz, vp]
        lib.oracle_gcm_open.argtypes = [vp, sz, vp, u64, vp, sz, vp, sz, vp]
        lib.oracle_gcm_open.restype = sz
        lib.oracle_seal_batch.argtypes = [vp, vp, sz, vp, sz, vp, vp, vp]
        lib.oracle_open_batch.argtypes = [vp, vp, sz, vp, sz, vp, vp, vp, vp]
        lib.oracle_quiclb_transform.argtypes = [vp, vp, vp, sz, ctypes.c_int]
        self.lib = lib

    def aes_encrypt(self, key: bytes, block: bytes) -> bytes:
        out = bytearray(16)
        self.lib.oracle_aes_encrypt(_ptr(key), len(key), _ptr(out), _ptr(block))
        return bytes(out)

    def gf128_mul(self, x: bytes, y: bytes) -> bytes:
        out = bytearray(16)
        self.lib.oracle_gf128_mul(_ptr(out), _ptr(x), _ptr(y))
        return bytes(out)

    def ghash(self, h: bytes, data: bytes) -> bytes:
        assert len(data) % 16 == 0
        out = bytearray(16)
        self.lib.oracle_ghash(_ptr(out), _ptr(h), _ptr(data) if data else None, len(data) // 16)
        return bytes(out)

    def seal(self, key: bytes, iv: bytes, seq: int, aad: bytes, pt: bytes) -> bytes:
        out = bytearray(len(pt) + 16)
        self.lib.oracle_gcm_seal(_ptr(key), len(key), _ptr(iv), seq, _ptr(aad) if aad else None, len(aad),
                                 _ptr(pt) if pt else None, len(pt), _ptr(out))
        return bytes(out)

    def open(self, key: bytes, iv: bytes, seq: int, aad: bytes, ct_tag: bytes):
        """Returns the plaintext, or None when the tag does not verify (ptls_aead_decrypt -> SIZE_MAX)."""
        out = bytearray(max(len(ct_tag) - 16, 0) + 1)
        r = self.lib.oracle_gcm_open(_ptr(key), len(key), _ptr(iv), seq, _ptr(aad) if aad else None, len(aad),
                                     _ptr(ct_tag) if ct_tag else None, len(ct_tag), _ptr(out))
        if r == ctypes.c_size_t(-1).value:
            return None
        return bytes(out[:r])

    def quiclb(self, key: bytes, data: bytes, encrypt: bool) -> bytes:
        """picotls_quiclb_transform (lib/quiclb-impl.h:107-162) restated in oracle/gcm_ref.c."""
        out = bytearray(len(data))
        if self.lib.oracle_quiclb_transform(_ptr(key), _ptr(out), _ptr(bytes(data)), len(data), 1 if encrypt else 0) != 0:
            raise ValueError("QUIC-LB length must be 7..19")
        return bytes(out)

    def seal_batch(self, keys, ivs, key_size, recs, in_arena, aad_arena, out_arena):
        self.lib.oracle_seal_batch(_ptr(keys), _ptr(ivs), key_size, _ptr(recs), len(recs), _ptr(in_arena),
                                   _ptr(aad_arena), _ptr(out_arena))

    def open_batch(self, keys, ivs, key_size, recs, in_arena, aad_arena, out_arena, ok):
        self.lib.oracle_open_batch(_ptr(keys), _ptr(ivs), key_size, _ptr(recs), len(recs), _ptr(in_arena),
                                   _ptr(aad_arena), _ptr(out_arena), _ptr(ok))


class FusionRef:
    """ctypes front-end of picotls' lib/fusion.c (oracle/_ref/libfusion_ref.so, built from /root/reference)."""

    def __init__(self):
        path = os.path.join(REF_DIR, "libfusion_ref.so")
        if not os.path.exists(path):
            build()
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: build it with `make -C oracle` where /root/reference exists")
        lib = ctypes.CDLL(path)
        vp, sz, u64, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int
        lib.ref_cpu_supported.restype = ci
        lib.ref_run_batch.argtypes = [ci, ci, vp, vp, sz, vp, sz, vp, vp, vp, vp, ci, vp, ctypes.POINTER(sz)]
        lib.ref_run_batch.restype = ctypes.c_double
        lib.ref_seal.argtypes = [vp, sz, vp, u64, vp, sz, vp, sz, vp]
        lib.ref_open.argtypes = [vp, sz, vp, u64, vp, sz, vp, sz, vp]
        lib.ref_open.restype = sz
        lib.ref_fusion_raw_seal.argtypes = [vp, sz, vp, sz, vp, sz, vp]
        lib.ref_seal_with_hp.argtypes = [vp, sz, vp, u64, vp, sz, vp, sz, vp, vp, sz, vp]
        lib.ref_aesecb.argtypes = [vp, sz, vp, vp]
        lib.ref_quiclb.argtypes = [vp, vp, vp, sz, ci]
        self.lib = lib
        if not lib.ref_cpu_supported():
            raise RuntimeError("host CPU lacks AES-NI/PCLMUL/AVX2: lib/fusion.c cannot run here")

    def seal(self, key, iv, seq, aad, pt):
        out = bytearray(len(pt) + 16)
        self.lib.ref_seal(_ptr(key), len(key), _ptr(iv), seq, _ptr(aad) if aad else None, len(aad),
                          _ptr(pt) if pt else None, len(pt), _ptr(out))
        return bytes(out)

    def open(self, key, iv, seq, aad, ct_tag):
        out = bytearray(max(len(ct_tag) - 16, 0) + 1)
        r = self.lib.ref_open(_ptr(key), len(key), _ptr(iv), seq, _ptr(aad) if aad else None, len(aad),
                              _ptr(ct_tag) if ct_tag else None, len(ct_tag), _ptr(out))
        if r == ctypes.c_size_t(-1).value:
            return None
        return bytes(out[:r])

    def raw_seal_zero_ctr(self, key, pt, aad):
        out = bytearray(len(pt) + 16)
        self.lib.ref_fusion_raw_seal(_ptr(key), len(key), _ptr(pt) if pt else None, len(pt), _ptr(aad) if aad else None,
                                     len(aad), _ptr(out))
        return bytes(out)

    def seal_with_hp(self, key, iv, seq, aad, pt, hp_key, sample_off):
        out = bytearray(len(pt) + 16)
        mask = bytearray(16)
        self.lib.ref_seal_with_hp(_ptr(key), len(key), _ptr(iv), seq, _ptr(aad) if aad else None, len(aad),
                                  _ptr(pt) if pt else None, len(pt), _ptr(out), _ptr(hp_key), sample_off, _ptr(mask))
        return bytes(out), bytes(mask)

    def aesecb(self, key, block):
        out = bytearray(16)
        self.lib.ref_aesecb(_ptr(key), len(key), _ptr(out), _ptr(block))
        return bytes(out)

    def quiclb(self, key: bytes, data: bytes, encrypt: bool) -> bytes:
        """ptls_fusion_quiclb through ptls_cipher_new / ptls_cipher_encrypt (t/quiclb.c:36-45)."""
        out = bytearray(len(data))
        self.lib.ref_quiclb(_ptr(key), _ptr(out), _ptr(bytes(data)), len(data), 1 if encrypt else 0)
        return bytes(out)

    def run_batch(self, is_seal, keys, ivs, key_size, recs, in_arena, aad_arena, out_arena, ok=None, nthreads=1,
                  cpus=None, nontemporal=False):
        """Seal/open a whole batch with `nthreads` pinned threads; returns (seconds, failures)."""
        fails = ctypes.c_size_t(0)
        cpu_arr = None
        if cpus is not None:
            cpu_arr = np.asarray(cpus, dtype=np.int32)
        t = self.lib.ref_run_batch(1 if is_seal else 0, 1 if nontemporal else 0, _ptr(keys), _ptr(ivs), key_size,
                                   _ptr(recs), len(recs), _ptr(in_arena), _ptr(aad_arena), _ptr(out_arena), _ptr(ok),
                                   nthreads, _ptr(cpu_arr), ctypes.byref(fails))
        return t, fails.value


class PtlsBenchRef:
    """ctypes front-end of oracle/ptlsbench_harness.c (in oracle/_ref/libtls12_ref.so): t/ptlsbench.c's benchmark loop
    over fusion with its own conventions (BASELINE.json configs[0])."""

    BATCH = 1000  # BENCH_BATCH, t/ptlsbench.c:86
    SECRET = b"z" * 64  # memset(secret, 'z', sizeof(secret)), t/ptlsbench.c:223

    def __init__(self):
        path = os.path.join(REF_DIR, "libtls12_ref.so")
        if not os.path.exists(path):
            build()
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: build it with `make -C oracle` where /root/reference exists")
        lib = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.ref_ptlsbench_keys.argtypes = [sz, vp, vp, vp]
        lib.ref_ptlsbench.argtypes = [sz, sz, sz, vp, vp]
        self.lib = lib

    def keys(self, key_size: int = 16) -> tuple[bytes, bytes]:
        """(key, IV) of ptls_aead_new(aead, hash, is_enc, 32 x 'z', NULL) (get_traffic_keys, lib/picotls.c:1634)."""
        key, iv = bytearray(key_size), bytearray(12)
        if self.lib.ref_ptlsbench_keys(key_size, _ptr(self.SECRET), _ptr(key), _ptr(iv)) != 0:
            raise RuntimeError("ptls_hkdf_expand_label failed")
        return bytes(key), bytes(iv)

    def run(self, n: int, l: int, key_size: int = 16, first_batch: np.ndarray | None = None) -> dict:
        """bench_run_one over n records of l bytes; first_batch (uint8, >= min(n, 1000) * (l + 16) bytes) receives the
        first batch's sealed records. Returns CPU (ptlsbench's clock) and wall seconds per direction."""
        times = np.zeros(4, np.float64)
        if self.lib.ref_ptlsbench(key_size, l, n, _ptr(first_batch), _ptr(times)) != 0:
            raise RuntimeError("ptlsbench: a record failed to open")
        return {"seal_cpu_s": times[0] * 1e-6, "open_cpu_s": times[1] * 1e-6, "seal_wall_s": times[2], "open_wall_s": times[3]}


class Tls12Ref:
    """ctypes front-end of picotls' own record layer (oracle/_ref/libtls12_ref.so, oracle/tls12_harness.c): TLS 1.2 over
    fusion's non-temporal AEADs (ptls_import of ptls_build_tls12_export_params) and TLS 1.3 over the same objects
    (ptls_import of traffic secrets), then ptls_send (server) / ptls_receive (client)."""

    def __init__(self):
        path = os.path.join(REF_DIR, "libtls12_ref.so")
        if not os.path.exists(path):
            build()
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: build it with `make -C oracle` where /root/reference exists")
        lib = ctypes.CDLL(path)
        vp, sz, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
        lib.ref_tls12_server_keys.argtypes = [sz, vp, vp, vp, vp]
        lib.ref_tls12_send.argtypes = [sz, vp, vp, u64, vp, sz, vp, sz]
        lib.ref_tls12_send.restype = sz
        lib.ref_tls12_receive.argtypes = [sz, vp, vp, vp, sz, vp, sz]
        lib.ref_tls12_receive.restype = ctypes.c_long
        lib.ref_tls13_traffic_keys.argtypes = [sz, vp, vp, vp]
        lib.ref_tls13_send.argtypes = [sz, vp, u64, vp, sz, vp, sz]
        lib.ref_tls13_send.restype = sz
        lib.ref_tls13_receive.argtypes = [sz, vp, u64, vp, sz, vp, sz]
        lib.ref_tls13_receive.restype = ctypes.c_long
        lib.ref_tls13_send_rekeyed.argtypes = [sz, vp, u64, vp, sz, vp, sz, vp, vp, vp]
        lib.ref_tls13_send_rekeyed.restype = sz
        self.lib = lib

    def server_keys(self, key_size: int, master_secret: bytes, randoms: bytes) -> tuple[bytes, bytes]:
        """(server write key, 4-byte fixed IV) of the key block (lib/picotls.c:5308-5335)."""
        key, iv = bytearray(key_size), bytearray(4)
        if self.lib.ref_tls12_server_keys(key_size, _ptr(master_secret), _ptr(randoms), _ptr(key), _ptr(iv)) != 0:
            raise RuntimeError("ptls_tls12_phash failed")
        return bytes(key), bytes(iv)

    def send(self, key_size: int, master_secret: bytes, randoms: bytes, record_iv: int, data: bytes) -> bytes:
        """The server's wire records for `data` (sequence numbers from 1, explicit nonces from record_iv)."""
        cap = len(data) + (len(data) // 16384 + 1) * 64
        out = bytearray(cap)
        n = self.lib.ref_tls12_send(key_size, _ptr(master_secret), _ptr(randoms), record_iv, _ptr(bytes(data)) if data else None,
                                    len(data), _ptr(out), cap)
        if n == 0:
            raise RuntimeError("ptls_send failed")
        return bytes(out[:n])

    def receive(self, key_size: int, master_secret: bytes, randoms: bytes, wire: bytes):
        """Plaintext of the server's records as the client decrypts them, or a negative picotls error code."""
        out = bytearray(len(wire) + 1)
        r = self.lib.ref_tls12_receive(key_size, _ptr(master_secret), _ptr(randoms), _ptr(bytes(wire)), len(wire), _ptr(out),
                                       len(out))
        return bytes(out[:r]) if r >= 0 else r

    # TLS 1.3 (ptls_import of traffic secrets, ptls_send / ptls_receive over ptls_non_temporal_aes{128,256}gcm)
    def tls13_keys(self, key_size: int, secret: bytes) -> tuple[bytes, bytes]:
        """(key, static IV) that setup_traffic_protection derives from a TLS 1.3 traffic secret (ptls_get_traffic_keys)."""
        key, iv = bytearray(key_size), bytearray(12)
        if self.lib.ref_tls13_traffic_keys(key_size, _ptr(secret), _ptr(key), _ptr(iv)) != 0:
            raise RuntimeError("ptls_import / ptls_get_traffic_keys failed")
        return bytes(key), bytes(iv)

    def tls13_send(self, key_size: int, secret: bytes, seq: int, data: bytes) -> bytes:
        cap = len(data) + (len(data) // 16384 + 1) * 64
        out = bytearray(cap)
        n = self.lib.ref_tls13_send(key_size, _ptr(secret), seq, _ptr(bytes(data)) if data else None, len(data), _ptr(out), cap)
        if n == 0:
            raise RuntimeError("ptls_send failed")
        return bytes(out[:n])

    def tls13_send_rekeyed(self, key_size: int, secret: bytes, seq: int, data: bytes):
        """(wire, key, IV, next seq) of the send direction after ptls_send: from seq >= 2^24 the wire starts with a
        KeyUpdate record under the old key and the data records use the next traffic secret from seq 0."""
        cap = len(data) + (len(data) // 16384 + 2) * 64
        out, key, iv, nseq = bytearray(cap), bytearray(key_size), bytearray(12), ctypes.c_uint64()
        n = self.lib.ref_tls13_send_rekeyed(key_size, _ptr(secret), seq, _ptr(bytes(data)) if data else None, len(data),
                                            _ptr(out), cap, _ptr(key), _ptr(iv), ctypes.byref(nseq))
        if n == 0:
            raise RuntimeError("ptls_send failed")
        return bytes(out[:n]), bytes(key), bytes(iv), nseq.value

    def tls13_receive(self, key_size: int, secret: bytes, seq: int, wire: bytes):
        out = bytearray(len(wire) + 1)
        r = self.lib.ref_tls13_receive(key_size, _ptr(secret), seq, _ptr(bytes(wire)), len(wire), _ptr(out), len(out))
        return bytes(out[:r]) if r >= 0 else r
