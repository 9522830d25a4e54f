"""Host-side layout of record batches (descriptor arrays + arenas) and shard planning.

A batch is described by a ``RECORD_DTYPE`` array (the 40-byte ``ptls_mi355x_record_t`` of include/picotls/mi355x.h)
plus three byte arenas: the input arena (plaintext when sealing; ciphertext||tag when opening), the output arena and
the AAD arena. Record slots are 16-byte aligned so the kernels' 16-byte accesses stay inside one record.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

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

# ptls_mi355x_hp_t: one QUIC header-protection sample per packet
HP_DTYPE = np.dtype([("sample_off", "<u8"), ("key_idx", "<u4"), ("reserved", "<u4")])
assert HP_DTYPE.itemsize == 16

# ptls_mi355x_cid_t (include/picotls/mi355x.h): one QUIC-LB connection ID to encrypt / decrypt
CID_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("key_idx", "<u4"), ("len", "u1"), ("encrypt", "u1"),
                      ("reserved", "<u2")])
assert CID_DTYPE.itemsize == 24
QUICLB_MIN_LEN, QUICLB_MAX_LEN = 7, 19  # PTLS_QUICLB_{MIN,MAX}_BLOCK_SIZE, include/picotls.h:117-118

# ptls_mi355x_tls_result_t: per-record outcome of ptls_mi355x_open_tls_records
TLS_RESULT_DTYPE = np.dtype([("plain_len", "<u4"), ("content_type", "u1"), ("status", "u1"), ("reserved", "<u2")])
assert TLS_RESULT_DTYPE.itemsize == 8
TLS_OK, TLS_BAD_MAC, TLS_BAD_HEADER, TLS_UNEXPECTED_MESSAGE = 0, 1, 2, 3


def _round16(x):
    if isinstance(x, np.ndarray):
        return (x + np.uint64(15)) // np.uint64(16) * np.uint64(16)
    return (int(x) + 15) // 16 * 16


@dataclass
class RecordBatch:
    """Descriptors for sealing (``seal``) and for opening the sealed output again (``open``)."""

    seal: np.ndarray  # RECORD_DTYPE, in = plaintext arena, out = sealed arena
    open: np.ndarray  # RECORD_DTYPE, in = sealed arena, out = plaintext-out arena
    pt_bytes: int  # size of the plaintext arena (also of the plaintext-out arena)
    sealed_bytes: int  # size of the sealed (ciphertext || tag) arena
    aad_bytes: int  # size of the AAD arena

    @property
    def n(self) -> int:
        return len(self.seal)

    @property
    def payload_bytes(self) -> int:
        return int(self.seal["len"].astype(np.uint64).sum())

    @classmethod
    def build(cls, lens, aad_lens, seqs=None, key_idx=None, pt_gap=0, sealed_gap=0, aad_gap=0) -> "RecordBatch":
        """Packs records back to back in 16-byte aligned slots (``*_gap`` extra bytes between slots, for
        unaligned-offset tests use :meth:`build_offsets`)."""
        lens = np.asarray(lens, dtype=np.uint64)
        n = len(lens)
        aad_lens = np.broadcast_to(np.asarray(aad_lens, dtype=np.uint64), (n,))
        seqs = np.arange(n, dtype=np.uint64) if seqs is None else np.asarray(seqs, dtype=np.uint64)
        key_idx = np.zeros(n, dtype=np.uint32) if key_idx is None else np.asarray(key_idx, dtype=np.uint32)
        pt_slot = _round16(lens) + np.uint64(pt_gap)
        sealed_slot = _round16(lens + np.uint64(16)) + np.uint64(sealed_gap)
        aad_slot = _round16(aad_lens) + np.uint64(aad_gap)
        pt_off = np.concatenate([[0], np.cumsum(pt_slot)[:-1]]).astype(np.uint64) if n else np.zeros(0, np.uint64)
        sealed_off = np.concatenate([[0], np.cumsum(sealed_slot)[:-1]]).astype(np.uint64) if n else np.zeros(0, np.uint64)
        aad_off = np.concatenate([[0], np.cumsum(aad_slot)[:-1]]).astype(np.uint64) if n else np.zeros(0, np.uint64)
        if n and int(aad_off[-1] + aad_slot[-1]) >= 1 << 32:
            raise ValueError("AAD arena exceeds 4 GiB (aad_off is 32-bit)")
        seal = np.zeros(n, dtype=RECORD_DTYPE)
        seal["in_off"], seal["out_off"], seal["seq"] = pt_off, sealed_off, seqs
        seal["aad_off"], seal["len"], seal["key_idx"], seal["aad_len"] = aad_off, lens, key_idx, aad_lens
        opn = seal.copy()
        opn["in_off"], opn["out_off"] = sealed_off, pt_off
        return cls(seal, opn, int(pt_slot.sum()) if n else 0, int(sealed_slot.sum()) if n else 0,
                   int(aad_slot.sum()) if n else 0)


def algorithmic_bytes(lens, aad_lens, is_seal: bool) -> int:
    """HBM bytes a perfect implementation must move for one pass:
    seal reads L + A + 40 (descriptor) and writes L + 16; open reads L + 16 + A + 40 and writes L + 1 (ok byte)."""
    lens = np.asarray(lens, dtype=np.uint64)
    aad_lens = np.broadcast_to(np.asarray(aad_lens, dtype=np.uint64), lens.shape)
    n = lens.size
    base = int(lens.sum()) * 2 + int(aad_lens.sum()) + 40 * n
    return base + (16 * n if is_seal else 17 * n)


def shard_ranges(weights, nshards: int) -> list[tuple[int, int]]:
    """Contiguous [begin, end) record ranges, balanced by weight (bytes), one per shard (rank / thread)."""
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if nshards < 1:
        raise ValueError("nshards must be >= 1")
    if n == 0:
        return [(0, 0)] * nshards
    cum = np.cumsum(w)
    total = cum[-1]
    bounds = [0]
    for s in range(1, nshards):
        bounds.append(int(np.searchsorted(cum, total * s / nshards, side="left")) + 1 if total > 0 else n * s // nshards)
    bounds.append(n)
    bounds = [min(max(b, 0), n) for b in bounds]
    for i in range(1, len(bounds)):
        bounds[i] = max(bounds[i], bounds[i - 1])
    return [(bounds[i], bounds[i + 1]) for i in range(nshards)]
