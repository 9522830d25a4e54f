"""The benchmark / parity workloads of BASELINE.json (synthetic record batches) and their deterministic generators.

configs (BASELINE.json):
  ptlsbench  1000-record batches of 16384 B under t/ptlsbench.c's conventions (ptlsbench_batch)          (configs[0])
  tls16k     1M x 16384 B TLS records, AES-128-GCM, one traffic key, AAD = TLS header {23,3,3,len}   (configs[1])
  quic1200   4M x 1200 B QUIC-sized records, AES-128-GCM, one key, 13-byte AAD                      (configs[2])
  mixed      4M records, L ~ U[64, 16384], AES-256-GCM, 64K keys (many-connection case)             (configs[3])
  shard1200  32M x 1200 B sharded evenly across GPUs, AES-128-GCM                                   (configs[4])

Payload and key bytes come from a seekable splitmix64 stream (seed 0x5eed), identical on host (numpy) and device
(torch), so every shard of a batch is a slice of one global batch.
"""
from __future__ import annotations

from dataclasses import dataclass, replace

import numpy as np

from .records import RecordBatch

GOLDEN = 0x9E3779B97F4A7C15
C1 = 0xBF58476D1CE4E5B9
C2 = 0x94D049BB133111EB
M64 = (1 << 64) - 1


def _to_i64(x: int) -> int:
    x &= M64
    return x - (1 << 64) if x >= 1 << 63 else x


def splitmix_words_np(seed: int, word_off: int, nwords: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        i = np.arange(word_off + 1, word_off + nwords + 1, dtype=np.uint64)
        z = np.uint64(seed & M64) + i * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(C1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(C2)
        return z ^ (z >> np.uint64(31))


def payload_np(seed: int, byte_off: int, nbytes: int) -> np.ndarray:
    w0 = byte_off // 8
    w1 = (byte_off + nbytes + 7) // 8
    words = splitmix_words_np(seed, w0, w1 - w0)
    b = words.astype("<u8").view(np.uint8)
    s = byte_off - 8 * w0
    return b[s:s + nbytes]


def payload_torch(seed: int, nbytes: int, device, out=None, chunk_words: int = 1 << 25):
    """Device-side splitmix64 byte stream (bytes [0, nbytes) of the stream), written into `out` (uint8) if given."""
    import torch

    if out is None:
        out = torch.empty(nbytes, dtype=torch.uint8, device=device)
    nwords = (nbytes + 7) // 8
    m30, m27, m31 = (1 << 34) - 1, (1 << 37) - 1, (1 << 33) - 1  # logical right shifts on int64
    g, c1, c2, sd = _to_i64(GOLDEN), _to_i64(C1), _to_i64(C2), _to_i64(seed)
    for w0 in range(0, nwords, chunk_words):
        n = min(chunk_words, nwords - w0)
        z = torch.arange(w0 + 1, w0 + n + 1, dtype=torch.int64, device=device)
        z.mul_(g).add_(sd)
        z = (z ^ ((z >> 30) & m30)) * c1
        z = (z ^ ((z >> 27) & m27)) * c2
        z = z ^ ((z >> 31) & m31)
        bytes_ = z.view(torch.uint8)
        lo, hi = 8 * w0, min(8 * (w0 + n), nbytes)
        out[lo:hi] = bytes_[: hi - lo]
        del z, bytes_
    return out


def tls_aad(length: int) -> bytes:
    """TLS 1.3 record header used as AAD (lib/picotls.c:719-726): type 23, legacy version 0x0303, length incl. tag."""
    n = length + 16
    return bytes([23, 3, 3, (n >> 8) & 0xFF, n & 0xFF])


@dataclass(frozen=True)
class Workload:
    name: str
    nrecs: int
    rec_len: int | None  # None: mixed lengths
    aad_len: int
    key_size: int
    nkeys: int = 1
    min_len: int = 64
    max_len: int = 16384
    tls_header_aad: bool = False
    seed: int = 0x5EED
    desc: str = ""
    key_order: str = "grouped"  # many keys: "grouped" by connection, or "random" (key_idx = splitmix(i) mod nkeys)
    sorted_lens: bool = False  # mixed lengths in ascending order over the batch (a batch built by record size)
    conn_classes: bool = False  # each connection (key) bulk (U[8 KiB, 16 KiB], one in four) or interactive (U[64, 1500])
    scatter_mem: bool = False  # records keep their batch order but sit at random places in the arenas
    bulk_every: int = 0  # every bulk_every-th connection sends uniform 8200-byte records (whole runs of a W8 pair's EXT 3)

    def scaled(self, nrecs: int) -> "Workload":
        return replace(self, nrecs=nrecs)

    # -- per-record attributes of the GLOBAL batch, sliced [begin, end)
    def lens(self, begin: int, end: int) -> np.ndarray:
        if self.rec_len is not None:
            return np.full(end - begin, self.rec_len, dtype=np.uint64)
        if self.conn_classes:
            w = splitmix_words_np(self.seed ^ 0x4C454E, begin, end - begin)
            key, _ = self.key_and_seq(begin, end)
            bulk = (splitmix_words_np(self.seed ^ 0x434C53, 0, self.nkeys)[key] % np.uint64(4)) == 0
            lo = np.where(bulk, np.uint64(8192), np.uint64(64))
            span = np.where(bulk, np.uint64(16384 - 8192 + 1), np.uint64(1500 - 64 + 1))
            return (lo + w % span).astype(np.uint64)
        if self.sorted_lens:
            w = np.sort(splitmix_words_np(self.seed ^ 0x4C454E, 0, self.nrecs) % np.uint64(self.max_len - self.min_len + 1))
            return (np.uint64(self.min_len) + w[begin:end]).astype(np.uint64)
        w = splitmix_words_np(self.seed ^ 0x4C454E, begin, end - begin)
        lens = (np.uint64(self.min_len) + w % np.uint64(self.max_len - self.min_len + 1)).astype(np.uint64)
        if self.bulk_every:
            key, _ = self.key_and_seq(begin, end)
            lens = np.where(key % self.bulk_every == 0, np.uint64(8200), lens).astype(np.uint64)
        return lens

    def key_and_seq(self, begin: int, end: int) -> tuple[np.ndarray, np.ndarray]:
        """Single key: seq = record index. Many keys: records are grouped by connection (a server batches per
        connection), i.e. key_idx = floor(i * nkeys / nrecs) and seq counts per key."""
        i = np.arange(begin, end, dtype=np.uint64)
        if self.nkeys == 1:
            return np.zeros(end - begin, np.uint32), i
        if self.key_order.startswith("bursts"):
            # analysis order: connections' records in bursts of B (key order "burstsB"): mixed's 64 records a key cut
            # into bursts, the bursts in a random order over the batch
            B = int(self.key_order[6:])
            even = (np.arange(self.nrecs, dtype=np.uint64) * np.uint64(self.nkeys) // np.uint64(self.nrecs)).astype(np.uint32)
            nb = (self.nrecs + B - 1) // B
            border = np.argsort(splitmix_words_np(self.seed ^ 0x425253, 0, nb), kind="stable")
            idx = (border[:, None] * B + np.arange(B)[None, :]).reshape(-1)
            idx = idx[idx < self.nrecs]
            allk = even[idx]
            order = np.argsort(allk, kind="stable")
            ks = allk[order]
            starts = np.searchsorted(ks, ks, side="left")
            seq = np.empty(self.nrecs, np.uint64)
            seq[order] = (np.arange(self.nrecs) - starts).astype(np.uint64)
            return allk[begin:end], seq[begin:end]
        if self.key_order in ("sorted_random", "shuffled"):
            # analysis orders: mixedrand's keys sorted (its uneven record counts per key, grouped in batch order), or
            # mixed's exactly even counts in a random order
            if self.key_order == "sorted_random":
                allk = np.sort((splitmix_words_np(self.seed ^ 0x4B4958, 0, self.nrecs) % np.uint64(self.nkeys)).astype(np.uint32))
            else:
                even = (np.arange(self.nrecs, dtype=np.uint64) * np.uint64(self.nkeys) // np.uint64(self.nrecs)).astype(np.uint32)
                allk = even[np.argsort(splitmix_words_np(self.seed ^ 0x534855, 0, self.nrecs), kind="stable")]
            order = np.argsort(allk, kind="stable")
            ks = allk[order]
            starts = np.searchsorted(ks, ks, side="left")
            seq = np.empty(self.nrecs, np.uint64)
            seq[order] = (np.arange(self.nrecs) - starts).astype(np.uint64)
            return allk[begin:end], seq[begin:end]
        if self.key_order == "random":
            # SURVEY §8(d) config 4 as written: key_idx = splitmix(i) mod nkeys over the whole batch, seq counting each
            # connection's records in batch order
            allk = (splitmix_words_np(self.seed ^ 0x4B4958, 0, self.nrecs) % np.uint64(self.nkeys)).astype(np.uint32)
            order = np.argsort(allk, kind="stable")
            ks = allk[order]
            starts = np.searchsorted(ks, ks, side="left")
            seq = np.empty(self.nrecs, np.uint64)
            seq[order] = (np.arange(self.nrecs) - starts).astype(np.uint64)
            return allk[begin:end], seq[begin:end]
        key = (i * np.uint64(self.nkeys) // np.uint64(self.nrecs)).astype(np.uint32)
        first = (key.astype(np.uint64) * np.uint64(self.nrecs) + np.uint64(self.nkeys) - np.uint64(1)) // np.uint64(self.nkeys)
        return key, i - first

    def descriptors(self, begin: int, end: int) -> RecordBatch:
        key, seq = self.key_and_seq(begin, end)
        if not self.scatter_mem:
            return RecordBatch.build(self.lens(begin, end), self.aad_len, seqs=seq, key_idx=key)
        # the arenas laid out in a random order of the records, the descriptors in batch order: a run's records are as
        # scattered over memory as the random key order scatters them, without the key grouping
        perm = np.argsort(splitmix_words_np(self.seed ^ 0x534354, begin, end - begin), kind="stable")
        b = RecordBatch.build(self.lens(begin, end)[perm], self.aad_len, seqs=seq[perm], key_idx=key[perm])
        inv = np.empty(end - begin, np.int64)
        inv[perm] = np.arange(end - begin)
        b.seal, b.open = b.seal[inv], b.open[inv]
        return b

    def keys(self) -> tuple[np.ndarray, np.ndarray]:
        kb = payload_np(self.seed ^ 0x4B4559, 0, self.nkeys * self.key_size).copy()
        ivb = payload_np(self.seed ^ 0x4956, 0, self.nkeys * 12).copy()
        return kb, ivb

    def aad_arena(self, batch: RecordBatch, begin: int) -> np.ndarray:
        if batch.aad_bytes == 0:
            return np.zeros(1, np.uint8)
        if self.tls_header_aad:
            arena = np.zeros(batch.aad_bytes, np.uint8)
            lens = batch.seal["len"].astype(np.int64) + 16
            offs = batch.seal["aad_off"].astype(np.int64)
            arena[offs + 0] = 23
            arena[offs + 1] = 3
            arena[offs + 2] = 3
            arena[offs + 3] = (lens >> 8) & 0xFF
            arena[offs + 4] = lens & 0xFF
            return arena
        slot = batch.aad_bytes // max(batch.n, 1)
        return payload_np(self.seed ^ 0x414144, begin * slot, batch.aad_bytes).copy()


# BASELINE.json configs[0]: t/ptlsbench.c's conventions (bench_run_aead :187-247, bench_run_one :88-185)
PTLSBENCH_BATCH = 1000  # BENCH_BATCH, t/ptlsbench.c:86
PTLSBENCH_SECRET = b"z" * 64  # memset(secret, 'z', sizeof(secret)), t/ptlsbench.c:223


def ptlsbench_batch(n: int = PTLSBENCH_BATCH, rec_len: int = 16384, key_size: int = 16):
    """One ptlsbench batch as a record batch: key and IV from ptls_aead_new(aead, hash, is_enc, 32 x 'z', NULL)
    (:223-225; SHA-256 for AES-128, SHA-384 for AES-256, :271-274), seq = 1..n, AAD = uint64_t h[4] with h[0] = seq
    (32 bytes, little endian, :130, :141), all-zero plaintext (:117). Returns (batch, key, iv, aad arena); the
    plaintext arena is b.pt_bytes zero bytes."""
    from .keyschedule import traffic_keys

    key, iv = traffic_keys(key_size, "sha256" if key_size == 16 else "sha384", PTLSBENCH_SECRET)
    seqs = np.arange(1, n + 1, dtype=np.uint64)
    b = RecordBatch.build(np.full(n, rec_len, dtype=np.uint64), 32, seqs=seqs)
    aad = np.zeros(b.aad_bytes, np.uint8)
    aad.view("<u8").reshape(n, 4)[:, 0] = seqs
    return b, key, iv, aad


WORKLOADS = {
    "tls16k": Workload("tls16k", 1 << 20, 16384, 5, 16, tls_header_aad=True,
                       desc="1M x 16384 B TLS records, AES-128-GCM, single traffic key"),
    "quic1200": Workload("quic1200", 4 << 20, 1200, 13, 16, desc="4M x 1200 B QUIC-sized records, AES-128-GCM, single key"),
    "mixed": Workload("mixed", 4 << 20, None, 13, 32, nkeys=65536,
                      desc="4M mixed-length records 64 B-16 KiB, AES-256-GCM, 64K traffic keys"),
    "mixedrand": Workload("mixedrand", 4 << 20, None, 13, 32, nkeys=65536, key_order="random",
                          desc="4M mixed-length records 64 B-16 KiB, AES-256-GCM, 64K traffic keys in random order"),
    "shard1200": Workload("shard1200", 32 << 20, 1200, 13, 16,
                          desc="32M x 1200 B records sharded evenly across GPUs, AES-128-GCM"),
    # analysis variants (not BASELINE configs): isolate key switching and length mix from the AES-256 cost; batches
    # ordered by record size (mixedsorted) and connections of two size classes (mixedconn) for the workgroup split
    "mixed1key": Workload("mixed1key", 4 << 20, None, 13, 32,
                          desc="4M mixed-length records 64 B-16 KiB, AES-256-GCM, one key"),
    "mixedsorted": Workload("mixedsorted", 4 << 20, None, 13, 32, sorted_lens=True,
                            desc="4M mixed-length records 64 B-16 KiB sorted by length, AES-256-GCM, one key"),
    "mixedconn": Workload("mixedconn", 4 << 20, None, 13, 32, nkeys=65536, conn_classes=True,
                          desc="4M records of 64K connections grouped, a quarter bulk (8-16 KiB records), the rest "
                               "interactive (64-1500 B), AES-256-GCM"),
    "mixedscatter": Workload("mixedscatter", 4 << 20, None, 13, 32, nkeys=65536, scatter_mem=True,
                             desc="mixed (keys grouped) with the records at random places in the arenas"),
    "mixedpois": Workload("mixedpois", 4 << 20, None, 13, 32, nkeys=65536, key_order="sorted_random",
                          desc="mixedrand's keys in sorted order (uneven record counts per key, grouped)"),
    "mixedshuf": Workload("mixedshuf", 4 << 20, None, 13, 32, nkeys=65536, key_order="shuffled",
                          desc="mixed's keys (64 records each) in a random order"),
    "mixedbulk": Workload("mixedbulk", 4 << 20, None, 13, 32, nkeys=16384, bulk_every=16,
                          desc="4M records of 16K connections grouped (256 records each), every 16th a bulk transfer of "
                               "uniform 8200-byte records, the rest U[64, 16384], AES-256-GCM"),
    "quic64k": Workload("quic64k", 4 << 20, 1200, 13, 16, nkeys=65536,
                        desc="4M x 1200 B QUIC packets of 64K connections (64 each, grouped), AES-128-GCM"),
    "tls64k": Workload("tls64k", 1 << 20, 16384, 5, 16, tls_header_aad=True, nkeys=65536,
                       desc="1M x 16384 B TLS records of 64K connections (16 each, grouped), AES-128-GCM"),
    "mixedburst": Workload("mixedburst", 4 << 20, None, 13, 32, nkeys=65536, key_order="bursts10",
                           desc="mixed's 64 records a connection in bursts of 10, the bursts in random order"),
    "tls16k256": Workload("tls16k256", 1 << 20, 16384, 5, 32, tls_header_aad=True,
                          desc="1M x 16384 B TLS records, AES-256-GCM, one key"),
    "u8k256": Workload("u8k256", 4 << 20, 8192, 13, 32, desc="4M x 8192 B records, AES-256-GCM, one key"),
}
