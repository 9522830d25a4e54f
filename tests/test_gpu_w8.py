"""The W8 kernels (the Horner step on an 8-bit window-major H^8 table, ghash.h gmul8; round 4) bit-exact against
lib/fusion.c. Every run of a chunked batch of at least W8_MIN_RECS records takes them (unframed or TLS framed): EXT 4 (segment ends by a serial lane
Horner with one window-major H table, w8_lane_end) for cut runs and whole runs of short records, EXT 3 (the butterfly
end, w8_tree_end) for whole runs of records of at least W8_MIN_STEPS steps, launched after EXT 4 and skipping its runs
(the EXT 4 workgroups tell it which have none). Cases: one key and several, AES-128 and AES-256, the 64-step threshold
inside one run, seal / open / tamper, in place, and batches mixing long whole runs with short whole runs and cut runs, so
that both kernels work and skip the other's runs. The reference's per-block GHASH amortisation is lib/fusion.c:515-620
(six blocks per reduction); the tests hold for any build (with W8_HORNER 0 the same records take the 4-bit path)."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef  # noqa: E402
from picotls_amd.records import RecordBatch  # noqa: E402
from gpu_util import dev, empty, gpu_open, gpu_seal  # noqa: E402

pytestmark = pytest.mark.gpu

HAVE_REF = os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                                       "libfusion_ref.so"))


@pytest.fixture(scope="module")
def ref():
    assert torch.cuda.is_available(), "no GPU visible"
    pa.load_library()
    if not HAVE_REF:
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    return FusionRef()


def _check(ref, rng, lens, aads, key_size, nkeys, tamper=8, after_seal=None):
    n = len(lens)
    key_idx = np.sort(rng.integers(0, nkeys, n)) if nkeys > 1 else None
    b = RecordBatch.build(np.asarray(lens), np.asarray(aads), seqs=rng.integers(0, 2**62, n, dtype=np.uint64),
                          key_idx=key_idx)
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, key_size)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, key_size, b.seal, pt, aad, want, nthreads=8)
    bad_recs = [i for i in range(n) if not np.array_equal(
        sealed[int(b.seal[i]["out_off"]):int(b.seal[i]["out_off"]) + int(lens[i]) + 16],
        want[int(b.seal[i]["out_off"]):int(b.seal[i]["out_off"]) + int(lens[i]) + 16])]
    assert bad_recs == [], f"{len(bad_recs)} records differ from fusion, first {bad_recs[:8]}"
    assert np.array_equal(sealed, want)
    if after_seal is not None:
        after_seal()
    # open fusion's records with tampering (ciphertext, tag, AAD bits); the plaintext is written either way, as fusion
    bad, badaad = want.copy(), aad.copy()
    victims = rng.choice(n, min(tamper, n), replace=False)
    for t, v in enumerate(victims):
        o, ln = int(b.open[v]["in_off"]), int(lens[v])
        if t % 3 == 0:
            bad[o + int(rng.integers(0, ln + 16))] ^= 1 << int(rng.integers(0, 8))
        elif t % 3 == 1 or int(b.seal[v]["aad_len"]) == 0:
            bad[o + ln + int(rng.integers(0, 16))] ^= 0x20
        else:
            badaad[int(b.seal[v]["aad_off"]) + int(rng.integers(0, int(b.seal[v]["aad_len"])))] ^= 2
    back, ok = gpu_open(ks, b.open, bad, badaad, b.pt_bytes)
    expect_ok = np.ones(n, np.uint8)
    expect_ok[victims] = 0
    assert np.array_equal(ok, expect_ok)
    ref_back = np.zeros(b.pt_bytes, np.uint8)
    ref.run_batch(False, keys, ivs, key_size, b.open, bad, badaad, ref_back, ok=np.zeros(n, np.uint8), nthreads=8)
    assert np.array_equal(back, ref_back)
    ks.free()


@pytest.mark.parametrize("key_size,nkeys,n", [(16, 1, 2048), (32, 1, 2100), (16, 5, 3000), (32, 3, 2500)])
def test_w8_uniform_long_records_vs_fusion(ref, key_size, nkeys, n):
    # 16 KiB TLS records (129 steps), one key (runs of up to 4096 records) and a few keys (runs cut at key changes)
    rng = np.random.default_rng(8000 + key_size * 10 + nkeys)
    _check(ref, rng, np.full(n, 16384), np.full(n, 13), key_size, nkeys)


def test_w8_threshold_inside_a_run_vs_fusion(ref):
    # lengths of 62..66 steps inside one uniform run (within its 2-step slack): the run's first record decides W8
    rng = np.random.default_rng(8101)
    n = 3000
    lens = rng.integers(7800, 8400, n)
    _check(ref, rng, lens, rng.integers(0, 30, n), 16, 1)


def test_w8_mixed_with_short_and_cut_runs_vs_fusion(ref):
    # blocks of 16 KiB records (W8 runs), of 1200-byte records (whole runs below 64 steps: the plain kernel) and of
    # U[64, 16384] lengths (cut runs: the plain kernel), interleaved over the batch, so that every workgroup of both
    # kernels of the pair meets both kinds of runs
    rng = np.random.default_rng(8102)
    blocks = []
    for i in range(60):
        kind = i % 3
        blocks.append(np.full(300, 16384) if kind == 0 else np.full(300, 1200) if kind == 1 else rng.integers(64, 16385, 300))
    lens = np.concatenate(blocks)
    _check(ref, rng, lens, rng.integers(0, 20, len(lens)), 16, 1, tamper=30)


def test_w8_aes256_many_keys_mixed_vs_fusion(ref):
    rng = np.random.default_rng(8103)
    lens = np.concatenate([np.full(1000, 16384), rng.integers(64, 16385, 1000), np.full(1000, 12000)])
    _check(ref, rng, lens, np.full(len(lens), 13), 32, 7, tamper=20)


def test_w8_in_place_vs_fusion(ref):
    # seal in place (ciphertext over plaintext, tag after it) and open in place, 16 KiB records at odd offsets
    rng = np.random.default_rng(8104)
    n = 2048
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    off, aoff = 5, 3
    for i in range(n):
        recs[i]["in_off"] = recs[i]["out_off"] = off
        recs[i]["len"] = 16384
        recs[i]["aad_off"], recs[i]["aad_len"] = aoff, 13
        recs[i]["seq"] = 1000 + i
        off += 16384 + 16 + int(rng.integers(0, 40))
        aoff += 13 + int(rng.integers(0, 3))
    keys, ivs = np.frombuffer(rng.bytes(16), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    arena = np.frombuffer(rng.bytes(off + 16), np.uint8).copy()
    aad = np.frombuffer(rng.bytes(aoff + 1), np.uint8)
    want = arena.copy()
    ref.run_batch(True, keys, ivs, 16, recs, arena, aad, want, nthreads=8)
    ks = pa.Keyset(keys, ivs, 16)
    d_arena, d_recs, d_aad = dev(arena), dev(recs), dev(aad)
    pa.seal_batch(ks, d_recs.data_ptr(), n, d_arena.data_ptr(), d_aad.data_ptr(), d_arena.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(d_arena.cpu().numpy(), want)
    d_ok = empty(n, 0x55)
    pa.open_batch(ks, d_recs.data_ptr(), n, d_arena.data_ptr(), d_aad.data_ptr(), d_arena.data_ptr(), d_ok.data_ptr())
    torch.cuda.synchronize()
    assert d_ok.cpu().numpy().all()
    assert np.array_equal(d_arena.cpu().numpy()[:off], np.where(_record_mask(recs, off), arena[:off], want[:off]))
    ks.free()


def _record_mask(recs, size):
    m = np.zeros(size, bool)
    for r in recs:
        m[int(r["in_off"]):int(r["in_off"]) + int(r["len"])] = True
    return m


def _pair_batch_lens(rng, n):
    """Lengths of a batch whose every workgroup (256 CUs, contiguous ranges of 130 records) holds whole runs: mostly
    8200-byte records (65 steps: EXT 3's long whole runs), 1200-byte ones in the first ten ranges (EXT 4's short whole
    runs) and random lengths in the next ten (EXT 4's cut runs), so both kernels of a pair work and skip each other's
    runs and EXT 4 writes the flag words that EXT 3 reads (at 2,048 records no flag word was ever
    written on the device)."""
    lens = np.full(n, 8200)
    lens[:1300] = 1200
    lens[1300:2600] = rng.integers(64, 16385, 1300)
    return lens


def test_w8_pairs_on_many_streams_vs_fusion(ref):
    """W8 pairs of one keyset on 9 streams at once (more than W8_FLAG_STREAMS = 8, so a stream takes over the least
    recently used flag buffer): each stream has its own flag words, so the pairs run concurrently; every batch (long
    whole runs, short whole runs and cut runs, so that both kernels of each pair skip runs) equals fusion, twice over,
    and the counters show both kernels processing runs."""
    rng = np.random.default_rng(8105)
    nstreams, n = 9, 256 * 130
    key = np.frombuffer(rng.bytes(16), np.uint8)
    iv = np.frombuffer(rng.bytes(12), np.uint8)
    ks = pa.Keyset(key, iv, 16)
    jobs = []
    for i in range(nstreams):
        lens = _pair_batch_lens(rng, n)
        b = RecordBatch.build(lens, np.full(n, 13), seqs=rng.integers(0, 2**62, n, dtype=np.uint64))
        pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
        aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
        want = np.zeros(b.sealed_bytes, np.uint8)
        ref.run_batch(True, key, iv, 16, b.seal, pt, aad, want, nthreads=8)
        jobs.append((b, dev(b.seal), dev(pt), dev(aad), empty(b.sealed_bytes), want))
        del pt
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    torch.cuda.synchronize()
    pa.debug_counters(reset=True)
    for rnd in range(2):
        for (b, d_recs, d_pt, d_aad, d_out, _), st in zip(jobs, streams if rnd == 0 else streams[::-1]):
            with torch.cuda.stream(st):
                d_out.fill_(0)
            pa.seal_batch(ks, d_recs.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        for i, (b, _, _, _, d_out, want) in enumerate(jobs):
            assert np.array_equal(d_out[:b.sealed_bytes].cpu().numpy(), want), f"round {rnd}, stream {i}"
    c = pa.debug_counters(reset=True)
    assert c["launches"]["w8_serial"] == 2 * nstreams and c["launches"]["w8_tree"] == 2 * nstreams, c
    # (at 256 CUs: ~236 EXT 3 runs and ~30 EXT 4 runs per batch)
    assert c["runs"]["w8_tree"] >= 2 * nstreams * 100 and c["runs"]["w8_serial"] >= 2 * nstreams * 10, c
    ks.free()


@pytest.mark.parametrize("n,length,key_size,nkeys", [(256, 16384, 16, 1), (300, 1200, 32, 1), (1000, 0, 16, 1),
                                                   (2047, 700, 16, 3), (255, 1200, 16, 1)])
def test_w8_small_batches_vs_fusion(ref, n, length, key_size, nkeys):
    """(round 5) Batches from W8_MIN_RECS = 256 records take the W8 serial kernel (EXT 4 alone: a workgroup's share is
    too small for whole runs of long records, so no EXT 3), against fusion, sealed and opened with tampering; 255
    records keep the 4-bit kernels."""
    rng = np.random.default_rng(8700 + n + length)
    pa.debug_counters(reset=True)
    _check(ref, rng, np.full(n, length), np.full(n, 13), key_size, nkeys, tamper=3)
    c = pa.debug_counters(reset=True)
    if n >= 256:
        assert c["launches"]["w8_serial"] >= 2 and c["launches"]["w8_tree"] == 0, c
    else:
        assert c["launches"]["w8_serial"] == 0 and c["launches"]["w8_tree"] == 0, c


@pytest.mark.parametrize("length,aad,key_size,nkeys", [
    (1200, 13, 16, 1), (0, 13, 16, 1), (1, 0, 32, 1), (16, 16, 16, 2), (100, 17, 32, 3), (4095, 40, 16, 1),
    (7800, 5, 32, 1), (1223, 70, 16, 4)])
def test_w8_g4_whole_runs_vs_fusion(ref, length, aad, key_size, nkeys):
    """Whole runs of short uniform records (under W8_MIN_STEPS steps: the EXT 4 kernel) in 4-lane groups (ghash.h,
    round 5): 33,280 records (130 per workgroup at 256 CUs) of empty to 7800-byte records, AADs of 0 to 70 bytes
    (several blocks), one to four keys; every record and tag against fusion, then opened with tampering. The counters
    show the runs taken in 4-lane groups."""
    rng = np.random.default_rng(8300 + length + aad)
    n = 256 * 130
    pa.debug_counters(reset=True)
    _check(ref, rng, np.full(n, length), np.full(n, aad), key_size, nkeys, tamper=12)
    c = pa.debug_counters(reset=True)
    # (a run cut at a key change with fewer than 128 records left in its workgroup's range is cut into units instead)
    assert c["runs"]["w8_g4"] >= 2 * 200 and c["runs"]["w8_g4"] >= 0.9 * c["runs"]["w8_serial"], c


@pytest.mark.parametrize("key_size,nkeys", [(16, 1), (32, 3)])
def test_w8_tree_kernel_long_whole_runs_vs_fusion(ref, key_size, nkeys):
    """The EXT 3 kernel (butterfly segment ends) takes whole runs of records of at least W8_MIN_STEPS steps, which need
    at least 128 records per workgroup: 33,280 records of 16 KiB (130 per workgroup at 256 CUs; one key in dealt
    contiguous ranges, or three keys in work-balanced ranges), with 1200-byte records (EXT 4's whole runs) and cut runs
    mixed in at the front so that both kernels of the pair work and skip each other's runs; every record and tag
    against fusion, then opened with tampering."""
    rng = np.random.default_rng(8200 + key_size + nkeys)
    n = 256 * 130
    lens = np.full(n, 16384)
    lens[:600] = 1200
    lens[600:900] = rng.integers(64, 16385, 300)
    _check(ref, rng, lens, np.full(n, 13), key_size, nkeys, tamper=12)


def test_w8_pairs_from_many_threads_vs_fusion(ref):
    """Nine threads, each on its own stream, seal their own batches (whole-run sized, _pair_batch_lens) through one
    shared keyset three times over: the per-stream flag buffers are taken under the keyset's lock, and past
    W8_FLAG_STREAMS = 8 streams the least recently used one is taken over after its stream's last use, while the
    launches overlap on the device. Every output equals fusion's; the counters show both kernels processing runs."""
    import threading

    rng = np.random.default_rng(8106)
    nthreads, n = 9, 256 * 130
    key = np.frombuffer(rng.bytes(32), np.uint8)
    iv = np.frombuffer(rng.bytes(12), np.uint8)
    ks = pa.Keyset(key, iv, 32)
    jobs = []
    for t in range(nthreads):
        lens = _pair_batch_lens(rng, n)
        b = RecordBatch.build(lens, np.full(n, 13), seqs=rng.integers(0, 2**62, n, dtype=np.uint64))
        pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
        aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
        want = np.zeros(b.sealed_bytes, np.uint8)
        ref.run_batch(True, key, iv, 32, b.seal, pt, aad, want, nthreads=8)
        jobs.append((b, dev(b.seal), dev(pt), dev(aad), [empty(b.sealed_bytes) for _ in range(3)], want))
        del pt
    torch.cuda.synchronize()
    pa.debug_counters(reset=True)
    errors = []

    def worker(t):
        try:
            b, d_recs, d_pt, d_aad, outs, _ = jobs[t]
            st = torch.cuda.Stream()
            for k in range(3):
                with torch.cuda.stream(st):
                    outs[k].fill_(0)
                pa.seal_batch(ks, d_recs.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(), outs[k].data_ptr(), st.cuda_stream)
            st.synchronize()
        except Exception as e:  # reported below
            errors.append(f"thread {t}: {e!r}")

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    torch.cuda.synchronize()
    assert errors == []
    for t, (b, _, _, _, outs, want) in enumerate(jobs):
        for k, o in enumerate(outs):
            assert np.array_equal(o[:b.sealed_bytes].cpu().numpy(), want), f"thread {t}, launch {k}"
    c = pa.debug_counters(reset=True)
    assert c["launches"]["w8_tree"] == 3 * nthreads and c["runs"]["w8_tree"] >= 3 * nthreads * 100, c
    assert c["runs"]["w8_serial"] >= 3 * nthreads * 10, c
    ks.free()


def test_w8_records_beyond_the_run_unit_cap_vs_fusion(ref):
    """A W8 pair cuts its runs at W8_RUN_UNITS = 512 units (run_unit_cap), so in its kernels records from 1 MiB take
    units of a multiple length (unit_mul > 1: partials combined with the unit power applied that many times) where the
    4-bit kernel starts at 2 MiB. Records of 1 MiB - 40 B to 5 MiB + 7 B among 2,100 short ones, sealed and opened
    (two tampered) against fusion."""
    rng = np.random.default_rng(8107)
    lens = rng.integers(0, 2000, 2100)
    big = [(1 << 20) - 40, (1 << 20) + 1, 3 << 19, 3 << 20, (5 << 20) + 7]
    for k, ln in enumerate(big):
        lens[300 * k + 7] = ln
    _check(ref, rng, lens, rng.integers(0, 40, len(lens)), 32, 1, tamper=2)


def test_w8_many_key_range_edges_stay_cut_vs_fusion(ref):
    """A many-key batch with uneven record counts per key (sorted random keys, ~64 records each) is split among the
    workgroups at tile edges that fall inside connections, so a workgroup's range can start or end with one or two
    records of a key. Such a run is cut into units like any many-key run of fewer records than the workgroup has
    groups (round 5: it was a whole run, and when long an EXT 3 run, for which that workgroup's EXT 3 kernel re-scanned
    all its runs). 262,144 U[64, 16384] records over 4,096 AES-256 keys against fusion; the counters show no EXT 3
    run in the seal or the open."""
    rng = np.random.default_rng(8420)
    n = 262144
    seen = {}

    def seal_done():
        seen["seal"] = pa.debug_counters(reset=True)["runs"]

    pa.debug_counters(reset=True)
    _check(ref, rng, rng.integers(64, 16385, n), np.full(n, 13), 32, 4096, tamper=16, after_seal=seal_done)
    opened = pa.debug_counters(reset=True)["runs"]
    assert seen["seal"]["w8_tree"] == 0 and opened["w8_tree"] == 0, (seen, opened)
    assert seen["seal"]["w8_serial"] >= 4096 and opened["w8_serial"] >= 4096, (seen, opened)


def test_w8_pair_run_list_vs_fusion(ref):
    """A W8 pair's first kernel (EXT 4) lists where the runs it leaves to the second (EXT 3) start, and EXT 3 visits just
    those (round 5; before, it re-scanned every run of its workgroup). 131,071 records (dealt chunks of 256, two per
    workgroup, no weight balance) of 1,024 keys, 128 records each, alternating 8200-byte records (EXT 3's long whole
    runs) and 1200-byte ones (EXT 4's whole runs in 4-lane groups): every workgroup leaves two runs to EXT 3. Against
    fusion, sealed and opened with tampering; the counters show both kernels' runs."""
    rng = np.random.default_rng(8430)
    n = 131071
    key = np.arange(n) // 128
    lens = np.where(key % 2 == 0, 8200, 1200)
    seen = {}

    def seal_done():
        seen["seal"] = pa.debug_counters(reset=True)

    pa.debug_counters(reset=True)
    b = RecordBatch.build(lens, np.full(n, 13), seqs=rng.integers(0, 2**62, n, dtype=np.uint64), key_idx=key)
    nkeys = int(key.max()) + 1
    keys = np.frombuffer(rng.bytes(nkeys * 16), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    ks = pa.Keyset(keys, ivs, 16)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    seal_done()
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 16, b.seal, pt, aad, want, nthreads=8)
    assert np.array_equal(sealed, want)
    victims = rng.choice(n, 12, replace=False)
    bad = want.copy()
    for v in victims:
        bad[int(b.open[v]["in_off"]) + int(rng.integers(0, int(lens[v]) + 16))] ^= 0x10
    back, ok = gpu_open(ks, b.open, bad, aad, b.pt_bytes)
    expect_ok = np.ones(n, np.uint8)
    expect_ok[victims] = 0
    assert np.array_equal(ok, expect_ok)
    ref_back = np.zeros(b.pt_bytes, np.uint8)
    ref.run_batch(False, keys, ivs, 16, b.open, bad, aad, ref_back, ok=np.zeros(n, np.uint8), nthreads=8)
    assert np.array_equal(back, ref_back)
    opened = pa.debug_counters(reset=True)
    for c in (seen["seal"], opened):
        assert c["launches"]["w8_tree"] == 1 and c["runs"]["w8_tree"] >= 500 and c["runs"]["w8_g4"] >= 500, c
    ks.free()


@pytest.mark.parametrize("length,aad,key_size,per_key,n", [
    (1200, 13, 16, 64, 256 * 256), (1200, 13, 32, 64, 40000), (37, 0, 16, 48, 30000), (600, 21, 16, 17, 30000),
    (3000, 13, 32, 100, 40000), (1, 5, 16, 5, 20000)])
def test_w8_multi_key_runs_vs_fusion(ref, length, aad, key_size, per_key, n):
    """(round 6) Multi-key runs (MK runs, gcm_kernels.h scan_mk): a many-key batch's connections of short uniform
    records with fewer records than the workgroup has groups (QUIC packets of many connections) are joined, up to four
    connections and 256 records, into one whole run in 4-lane groups, each connection's tables in its own LDS slot
    (ghash.h gmul4w). Connections of 5 to 100 records (claims of 16 records, partial claims), 1 to 3000-byte records,
    AES-128 and AES-256, against fusion, sealed and opened with tampering; the counters show MK runs in both."""
    rng = np.random.default_rng(8800 + length + per_key)
    nkeys = (n + per_key - 1) // per_key
    key = np.arange(n) // per_key
    b = RecordBatch.build(np.full(n, length), np.full(n, aad), seqs=rng.integers(0, 2**62, n, dtype=np.uint64),
                          key_idx=key)
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aadb = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, key_size)
    pa.debug_counters(reset=True)
    sealed = gpu_seal(ks, b.seal, pt, aadb, b.sealed_bytes)
    c_seal = pa.debug_counters(reset=True)
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, key_size, b.seal, pt, aadb, want, nthreads=8)
    bad_recs = [i for i in range(n) if not np.array_equal(
        sealed[int(b.seal[i]["out_off"]):int(b.seal[i]["out_off"]) + length + 16],
        want[int(b.seal[i]["out_off"]):int(b.seal[i]["out_off"]) + length + 16])]
    assert bad_recs == [], f"{len(bad_recs)} records differ from fusion, first {bad_recs[:8]}"
    assert np.array_equal(sealed, want)
    victims = rng.choice(n, 16, replace=False)
    bad = want.copy()
    for t, v in enumerate(victims):
        bad[int(b.open[v]["in_off"]) + int(rng.integers(0, length + 16))] ^= 1 << (t % 8)
    back, ok = gpu_open(ks, b.open, bad, aadb, b.pt_bytes)
    c_open = pa.debug_counters(reset=True)
    expect_ok = np.ones(n, np.uint8)
    expect_ok[victims] = 0
    assert np.array_equal(ok, expect_ok)
    ref_back = np.zeros(b.pt_bytes, np.uint8)
    ref.run_batch(False, keys, ivs, key_size, b.open, bad, aadb, ref_back, ok=np.zeros(n, np.uint8), nthreads=8)
    assert np.array_equal(back, ref_back)
    # most connections run in MK runs (a workgroup's range edges leave a few cut ones)
    for c in (c_seal, c_open):
        assert c["runs"]["w8_mk"] >= 0.5 * nkeys / 4, (c, nkeys)
    ks.free()


@pytest.mark.parametrize("length,aad,key_size,per_key,shift", [
    (1200, 13, 16, 0, "16"), (1200, 13, 16, 0, "byte"), (1000, 0, 32, 0, "16"), (200, 40, 16, 0, "16"),
    (100, 17, 16, 0, "byte"), (4095, 13, 16, 0, "16"), (63, 5, 32, 0, "16"), (1200, 13, 16, 64, "16"),
    (700, 21, 32, 40, "byte")])
def test_w8_g4_open_into_shifted_outputs_vs_fusion(ref, length, aad, key_size, per_key, shift):
    """(round 6) A 4-lane group's open aligns its steps to the record's text (G4_OPEN_TEXT_STEPS), so its output is no
    longer aligned to the steps, and its steady steps hold blocks until a 128-byte line is whole (G4_LINE_HOLD: early
    and late lanes, the range's first and last steps). The plaintexts go to outputs shifted by 16 x (i mod 8) bytes or
    by any byte count, for one key (short whole runs) and for connections of 40-64 records (MK runs), with AADs of
    0-3 blocks (text block 0 at every position of a step); every byte of the output buffer, tags and ok bytes against
    fusion, with tampering."""
    rng = np.random.default_rng(8900 + length + aad + per_key + (1 if shift == "byte" else 0))
    n = 256 * 130
    nkeys = 1 if per_key == 0 else (n + per_key - 1) // per_key
    key = None if per_key == 0 else np.arange(n) // per_key
    b = RecordBatch.build(np.full(n, length), np.full(n, aad), seqs=rng.integers(0, 2**62, n, dtype=np.uint64),
                          key_idx=key)
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aadb = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    sealed = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, key_size, b.seal, pt, aadb, sealed, nthreads=8)
    victims = rng.choice(n, 16, replace=False)
    for t, v in enumerate(victims):
        sealed[int(b.open[v]["in_off"]) + int(rng.integers(0, length + 16))] ^= 1 << (t % 8)
    recs = b.open.copy()
    stride = (length + 127) // 128 * 128 + 128
    sh = 16 * (np.arange(n) % 8) if shift == "16" else (np.arange(n) * 37) % 128
    recs["out_off"] = (np.arange(n) * stride + sh).astype(np.uint64)
    out_bytes = n * stride + 128
    ks = pa.Keyset(keys, ivs, key_size)
    pa.debug_counters(reset=True)
    back, ok = gpu_open(ks, recs, sealed, aadb, out_bytes, out_fill=0x5A)
    c = pa.debug_counters(reset=True)
    expect_ok = np.ones(n, np.uint8)
    expect_ok[victims] = 0
    assert np.array_equal(ok, expect_ok)
    ref_back = np.full(out_bytes, 0x5A, np.uint8)
    ref.run_batch(False, keys, ivs, key_size, recs, sealed, aadb, ref_back, ok=np.zeros(n, np.uint8), nthreads=8)
    bad_recs = [i for i in range(n) if not np.array_equal(back[i * stride:(i + 1) * stride],
                                                          ref_back[i * stride:(i + 1) * stride])]
    assert bad_recs == [], f"{len(bad_recs)} record slots differ from fusion, first {bad_recs[:8]}"
    assert np.array_equal(back, ref_back)
    if per_key == 0:
        assert c["runs"]["w8_g4"] >= 200, c
    else:
        assert c["runs"]["w8_mk"] >= 0.5 * nkeys / 4, (c, nkeys)
    ks.free()


@pytest.mark.parametrize("length,aad,shift", [(1200, 13, 16), (1000, 0, 1), (333, 40, 7)])
def test_w8_g4_open_in_place_shifted_vs_fusion(ref, length, aad, shift):
    """(round 6) The 4-lane open with line holding stores each block up to two steps after it was read: opened in place
    (plaintext over its ciphertext) at offsets shifted by 16 x (i mod 8) or by odd byte counts, every record's plaintext
    and ok byte equal fusion's, and the bytes between records untouched."""
    rng = np.random.default_rng(8950 + length + shift)
    n = 256 * 130
    stride = (length + 16 + 127) // 128 * 128 + 128
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    recs["in_off"] = recs["out_off"] = (np.arange(n) * stride + (np.arange(n) * shift) % 128).astype(np.uint64)
    recs["len"] = length
    recs["aad_off"] = (np.arange(n) * max(aad, 1)).astype(np.uint32)
    recs["aad_len"] = aad
    recs["seq"] = rng.integers(0, 2**62, n, dtype=np.uint64)
    key, iv = np.frombuffer(rng.bytes(16), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    arena = np.frombuffer(rng.bytes(n * stride + 128), np.uint8).copy()
    aadb = np.frombuffer(rng.bytes(n * max(aad, 1) + 1), np.uint8)
    sealed = arena.copy()
    ref.run_batch(True, key, iv, 16, recs, arena, aadb, sealed, nthreads=8)  # in place: ciphertext and tag at in_off
    victims = rng.choice(n, 12, replace=False)
    for t, v in enumerate(victims):
        sealed[int(recs[v]["in_off"]) + int(rng.integers(0, length + 16))] ^= 1 << (t % 8)
    want = sealed.copy()
    ref.run_batch(False, key, iv, 16, recs, sealed, aadb, want, ok=np.zeros(n, np.uint8), nthreads=8)
    ks = pa.Keyset(key, iv, 16)
    d_arena, d_recs, d_aad = dev(sealed), dev(recs), dev(aadb)
    d_ok = empty(n, 0x55)
    pa.debug_counters(reset=True)
    pa.open_batch(ks, d_recs.data_ptr(), n, d_arena.data_ptr(), d_aad.data_ptr(), d_arena.data_ptr(), d_ok.data_ptr())
    torch.cuda.synchronize()
    c = pa.debug_counters(reset=True)
    expect_ok = np.ones(n, np.uint8)
    expect_ok[victims] = 0
    assert np.array_equal(d_ok.cpu().numpy(), expect_ok)
    got = d_arena.cpu().numpy()
    bad = [i for i in range(n) if not np.array_equal(got[i * stride:(i + 1) * stride], want[i * stride:(i + 1) * stride])]
    assert bad == [], f"{len(bad)} record slots differ from fusion, first {bad[:8]}"
    assert c["runs"]["w8_g4"] >= 200, c
    ks.free()
