"""BASELINE.json's configs run through the engine (C ABI) at their own conventions, bit-exact against lib/fusion.c.

  configs[0]  t/ptlsbench.c's 1000-record batch: HKDF key from 32 x 'z', AAD h[4] with h[0] = seq, zero plaintext,
              16384-byte records -- compared with fusion running ptlsbench's own loop (oracle/ptlsbench_harness.c)
  configs[3]  4M x U[64,16384] B, AES-256-GCM, 65,536 keys, key_idx = splitmix(i) mod 65536 (random order),
              per-key sequence numbers -- the workload generator of bench.py at 1M records, where every key appears
              (~16 records each): every record sealed and compared, then opened with 1 % of the records tampered
The other configs ([1] tls16k, [2] quic1200, [4] per-GPU shards of 1200 B) are covered at the same shapes by
test_gpu_parity.py::test_chunked_uniform_runs_vs_fusion and tests/test_gpu_dist.py.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef, PtlsBenchRef  # noqa: E402
from picotls_amd.workloads import WORKLOADS, payload_torch, ptlsbench_batch  # noqa: E402

pytestmark = pytest.mark.gpu

REF_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref")


@pytest.fixture(scope="module", autouse=True)
def engine():
    assert torch.cuda.is_available(), "no GPU visible"
    pa.load_library()
    assert pa.is_supported(), "engine reports no gfx950 device"


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def test_config0_ptlsbench_batch_vs_fusion_ptlsbench():
    if not os.path.exists(os.path.join(REF_DIR, "libtls12_ref.so")):
        pytest.skip("oracle/_ref/libtls12_ref.so not shipped")
    pb = PtlsBenchRef()
    b, key, iv, aad = ptlsbench_batch()
    # the key schedule of the host side equals picotls' own (ptls_hkdf_expand_label over SHA-256)
    assert (key, iv) == pb.keys(16)
    want = np.zeros(pb.BATCH * (16384 + 16), np.uint8)
    pb.run(pb.BATCH, 16384, 16, want)  # ptlsbench's first batch, sealed by fusion
    ks = pa.Keyset(key, iv, 16)
    dev = torch.device("cuda:0")
    d_recs = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    d_pt = torch.zeros(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_aad = torch.from_numpy(aad).to(dev)
    d_sealed = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device=dev)
    d_back = torch.ones(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), s)
    pa.open_batch(ks, d_open.data_ptr(), b.n, d_sealed.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    torch.cuda.synchronize()
    assert np.array_equal(d_sealed.cpu().numpy(), want)  # records are back to back: 16384 + 16 bytes each
    assert d_ok.cpu().numpy().all()
    assert not d_back.any().item()
    ks.free()


def test_config3_mixedrand_64k_keys_vs_fusion():
    if not os.path.exists(os.path.join(REF_DIR, "libfusion_ref.so")):
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    ref = FusionRef()
    wl = WORKLOADS["mixedrand"].scaled(1 << 20)
    b = wl.descriptors(0, wl.nrecs)
    assert len(np.unique(b.seal["key_idx"])) == wl.nkeys == 65536  # every connection has records in the batch
    assert (np.diff(b.seal["key_idx"].astype(np.int64)) != 0).mean() > 0.99  # random key order: nearly every neighbour differs
    keys, ivs = wl.keys()
    dev = torch.device("cuda:0")
    d_pt = payload_torch(wl.seed, b.pt_bytes, dev)
    pt = d_pt.cpu().numpy()
    aad = wl.aad_arena(b, 0)
    ks = pa.Keyset(keys, ivs, wl.key_size)
    s = torch.cuda.current_stream().cuda_stream
    d_recs = torch.from_numpy(b.seal.view(np.uint8).copy()).to(dev)
    d_aad = torch.from_numpy(aad).to(dev)
    d_sealed = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device=dev)
    pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), s)
    torch.cuda.synchronize()
    sealed = d_sealed.cpu().numpy()
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, wl.key_size, b.seal, pt, aad, want, nthreads=_threads())
    # the slots' padding is zero in both arenas, so whole-arena equality is per-record equality
    assert np.array_equal(sealed, want)

    # open with 1 % of the records tampered (a ciphertext or tag bit): ok bytes and plaintexts equal fusion's
    rng = np.random.default_rng(3)
    bad = rng.random(b.n) < 0.01
    bad_idx = np.flatnonzero(bad)
    pos = b.seal["out_off"][bad_idx].astype(np.int64) + rng.integers(0, b.seal["len"][bad_idx].astype(np.int64) + 16)
    tampered = want.copy()
    tampered[pos] ^= np.uint8(1) << rng.integers(0, 8, len(pos)).astype(np.uint8)
    d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    d_in = torch.from_numpy(tampered).to(dev)
    d_back = torch.zeros(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.full((b.n,), 0xAA, dtype=torch.uint8, device=dev)
    pa.open_batch(ks, d_open.data_ptr(), b.n, d_in.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    torch.cuda.synchronize()
    ok = d_ok.cpu().numpy()
    back_want = np.zeros(b.pt_bytes, np.uint8)
    ok_want = np.zeros(b.n, np.uint8)
    _, fails = ref.run_batch(False, keys, ivs, wl.key_size, b.open, tampered, aad, back_want, ok=ok_want,
                             nthreads=_threads())
    assert fails == len(bad_idx)
    assert np.array_equal(ok, ok_want)
    assert np.array_equal(ok.astype(bool), ~bad)
    assert np.array_equal(d_back.cpu().numpy(), back_want)  # plaintext written for every record, as fusion does
    ks.free()


def test_sorted_lengths_dealt_chunks_vs_fusion():
    # a batch large enough for the chunked kernel's dealt-out chunks (BatchArgs::chunk: each workgroup walks chunks
    # spread over the batch instead of one contiguous range): 300,000 records sorted by length (0..2000 B), 300 keys
    # grouped by connection, so chunk edges cut key runs and whole-record runs; every record equals fusion's, and an
    # open with 1 % of the records tampered reports exactly those
    if not os.path.exists(os.path.join(REF_DIR, "libfusion_ref.so")):
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    from picotls_amd.records import RecordBatch

    ref = FusionRef()
    rng = np.random.default_rng(17)
    n, nkeys = 300000, 300
    lens = np.sort(rng.integers(0, 2001, n)).astype(np.uint64)
    key_idx = (np.arange(n) * nkeys // n).astype(np.uint32)
    b = RecordBatch.build(lens, 13, seqs=np.arange(n, dtype=np.uint64), key_idx=key_idx)
    keys, ivs = rng.bytes(16 * nkeys), rng.bytes(12 * nkeys)
    keys_np, ivs_np = np.frombuffer(keys, np.uint8), np.frombuffer(ivs, np.uint8)
    dev = torch.device("cuda:0")
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    ks = pa.Keyset(keys, ivs, 16)
    s = torch.cuda.current_stream().cuda_stream
    d_recs, d_pt, d_aad = (torch.from_numpy(x.view(np.uint8).copy()).to(dev) for x in (b.seal, pt, aad))
    d_sealed = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device=dev)
    pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), s)
    torch.cuda.synchronize()
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys_np, ivs_np, 16, b.seal, pt, aad, want, nthreads=_threads())
    sealed = d_sealed.cpu().numpy()
    for i in (0, n // 2, n - 1):  # padding between slots is zero in both arenas: compare per record, then whole
        o, ln = int(b.seal["out_off"][i]), int(b.seal["len"][i]) + 16
        assert np.array_equal(sealed[o:o + ln], want[o:o + ln]), i
    assert np.array_equal(sealed, want)

    bad = rng.random(n) < 0.01
    bad_idx = np.flatnonzero(bad)
    pos = b.seal["out_off"][bad_idx].astype(np.int64) + rng.integers(0, b.seal["len"][bad_idx].astype(np.int64) + 16)
    tampered = want.copy()
    tampered[pos] ^= np.uint8(0x10)
    d_open = torch.from_numpy(b.open.view(np.uint8).copy()).to(dev)
    d_in = torch.from_numpy(tampered).to(dev)
    d_back = torch.zeros(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.full((n,), 0xAA, dtype=torch.uint8, device=dev)
    pa.open_batch(ks, d_open.data_ptr(), n, d_in.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    torch.cuda.synchronize()
    assert np.array_equal(d_ok.cpu().numpy().astype(bool), ~bad)
    m = np.zeros(b.pt_bytes, bool)
    for o, ln in zip(b.seal["in_off"][~bad][:2000], b.seal["len"][~bad][:2000]):
        m[int(o):int(o) + int(ln)] = True
    assert np.array_equal(d_back.cpu().numpy()[m], pt[m])
    ks.free()


def test_balanced_many_key_batch_with_skew_and_rejects_vs_fusion():
    # a many-key batch large enough for the work-balanced workgroup ranges (balance_*_kernel): 150,000 records over 97
    # connections, mostly 0-300 B but eight 256 KiB records at the front (one workgroup's share by count would hold
    # them all), and rejected descriptors (length above the cap, key outside the keyset) among them: every valid record
    # equals fusion's, the rejected ones write nothing and open with ok = 0
    if not os.path.exists(os.path.join(REF_DIR, "libfusion_ref.so")):
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    from picotls_amd.records import RecordBatch

    ref = FusionRef()
    rng = np.random.default_rng(23)
    n, nkeys = 150000, 97
    lens = rng.integers(0, 301, n).astype(np.uint64)
    lens[rng.choice(2000, 8, replace=False)] = 256 * 1024
    key_idx = (np.arange(n) * nkeys // n).astype(np.uint32)
    b = RecordBatch.build(lens, rng.integers(0, 40, n), seqs=rng.integers(0, 2**40, n, dtype=np.uint64), key_idx=key_idx)
    keys, ivs = rng.bytes(32 * nkeys), rng.bytes(12 * nkeys)
    keys_np, ivs_np = np.frombuffer(keys, np.uint8), np.frombuffer(ivs, np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys_np, ivs_np, 32, b.seal, pt, aad, want, nthreads=_threads())
    bad = np.sort(rng.choice(n, 40, replace=False))
    seal, opn = b.seal.copy(), b.open.copy()
    seal["len"][bad[:20]] = opn["len"][bad[:20]] = (1 << 30) + 7  # above PTLS_MI355X_MAX_RECORD_LEN
    seal["key_idx"][bad[20:]] = opn["key_idx"][bad[20:]] = nkeys + 3  # not in the keyset
    dev = torch.device("cuda:0")
    ks = pa.Keyset(keys, ivs, 32)
    s = torch.cuda.current_stream().cuda_stream
    d_recs, d_pt, d_aad = (torch.from_numpy(x.view(np.uint8).copy()).to(dev) for x in (seal, pt, aad))
    d_sealed = torch.full((b.sealed_bytes,), 0xEE, dtype=torch.uint8, device=dev)
    pa.seal_batch(ks, d_recs.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), s)
    torch.cuda.synchronize()
    sealed = d_sealed.cpu().numpy()
    isbad = np.zeros(n, bool)
    isbad[bad] = True
    mask = np.zeros(b.sealed_bytes, bool)  # the bytes of the valid records' outputs
    for o, ln in zip(b.seal["out_off"][~isbad], b.seal["len"][~isbad]):
        mask[int(o):int(o) + int(ln) + 16] = True
    assert np.array_equal(sealed[mask], want[mask])
    for i in bad:  # nothing written for a rejected record
        o, ln = int(b.seal["out_off"][i]), int(b.seal["len"][i]) + 16
        assert (sealed[o:o + ln] == 0xEE).all(), i
    d_open = torch.from_numpy(opn.view(np.uint8).copy()).to(dev)
    d_in = torch.from_numpy(want).to(dev)
    d_back = torch.zeros(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.full((n,), 0xAA, dtype=torch.uint8, device=dev)
    pa.open_batch(ks, d_open.data_ptr(), n, d_in.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    torch.cuda.synchronize()
    assert np.array_equal(d_ok.cpu().numpy().astype(bool), ~isbad)
    big = np.flatnonzero(lens == 256 * 1024)
    back = d_back.cpu().numpy()
    for i in big:
        o = int(b.seal["in_off"][i])
        assert np.array_equal(back[o:o + 256 * 1024], pt[o:o + 256 * 1024]), i
    ks.free()
