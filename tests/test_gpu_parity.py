"""Parity of the HIP engine (through its C ABI) with picotls' lib/fusion.c and the CPU oracle. Bit-exact.

Run on the MI355X box: python -m pytest tests -m gpu
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef, GcmOracle  # noqa: E402
from picotls_amd.records import RecordBatch  # noqa: E402
from vecs import check_sealed, materialise  # noqa: E402

pytestmark = pytest.mark.gpu

HAVE_REF = os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                                       "libfusion_ref.so"))


@pytest.fixture(scope="module", autouse=True)
def engine():
    assert torch.cuda.is_available(), "no GPU visible"
    pa.load_library()
    assert pa.is_supported(), "engine reports no gfx950 device"
    torch.cuda.init()


@pytest.fixture(scope="module")
def oracle():
    return GcmOracle()


@pytest.fixture(scope="module")
def ref():
    if not HAVE_REF:
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    return FusionRef()


from gpu_util import dev, empty, gpu_open, gpu_seal  # noqa: E402


def u8(b: bytes) -> np.ndarray:
    return np.frombuffer(bytes(b), dtype=np.uint8)


# ------------------------------------------------------------------------------------------------ known answers


def test_ecb_kat(kat):
    # t/fusion.c:72-86, t/picotls.c:397-413,429-437 through ptls_mi355x_ecb_batch
    for v in kat["ecb"]:
        key = bytes.fromhex(v["key"])
        if v["src"].startswith("t/picotls.c:374-376,397"):
            key = key[:16]
        ks = pa.Keyset(key, bytes(12), len(key))
        d_in, d_out = dev(u8(bytes.fromhex(v["pt"]) * 3)), empty(48)
        pa.ecb_batch(ks, 0, d_in.data_ptr(), d_out.data_ptr(), 3)
        torch.cuda.synchronize()
        assert bytes(d_out.cpu().numpy()).hex() == v["ct"] * 3, v["src"]


def test_gcm_zero_counter_kat(kat):
    # t/fusion.c:236-256,277-288
    for v in kat["gcm_zero_ctr"]:
        key, aad, pt = (bytes.fromhex(v[k]) for k in ("key", "aad", "pt"))
        ctx = pa.aead_new_direct(pa.aes128gcm, True, key, bytes(12))
        sealed = ctx.encrypt(pt, 0, aad)
        assert sealed.hex() == v["sealed"], v["src"]
        assert ctx.decrypt(sealed, 0, aad) == pt


def test_gcm_tag_vectors_and_hp_mask(kat):
    # t/fusion.c:290-344: 19 tags, then the same with the supplementary (header-protection) block
    t = kat["gcm_zero_ctr_tags"]
    ctx = pa.aead_new_direct(pa.aes128gcm, True, bytes(16), bytes(12))
    hp = pa.CtrCipher(bytes.fromhex(t["hp_key"]))
    for aadlen, ptlen, tag, mask in t["cases"]:
        sealed, m = ctx.encrypt_s(bytes(ptlen), 0, bytes(aadlen), hp, t["hp_sample_off"])
        assert sealed[ptlen:].hex() == tag, (aadlen, ptlen)
        assert m.hex() == mask
        assert ctx.decrypt(sealed, 0, bytes(aadlen)) == bytes(ptlen)


def test_gcm_seq_iv96_kat(kat):
    # t/fusion.c:258-274, :346-380 (ptls_aead_xor_iv; decrypt with the wrong IV fails, then succeeds again)
    for v in kat["gcm_seq"]:
        key, aad, pt, iv = (bytes.fromhex(v[k]) for k in ("key", "aad", "pt", "iv"))
        ctx = pa.aead_new_direct(pa.aes128gcm, False, key, iv)
        if "xor_iv" in v:
            ctx.xor_iv(bytes.fromhex(v["xor_iv"]))
        sealed = ctx.encrypt(pt, v["seq"], aad)
        assert sealed.hex() == v["sealed"]
        assert ctx.decrypt(sealed, v["seq"], aad) == pt
        if "bad_xor_iv" in v:
            ctx.xor_iv(bytes.fromhex(v["xor_iv"]))
            ctx.xor_iv(bytes.fromhex(v["bad_xor_iv"]))
            assert ctx.decrypt(sealed, v["seq"], aad) is None
            ctx.xor_iv(bytes.fromhex(v["bad_xor_iv"]))
            ctx.xor_iv(bytes.fromhex(v["xor_iv"]))
            assert ctx.decrypt(sealed, v["seq"], aad) == pt


def test_nist_vectors(kat):
    for v in kat["nist"]:
        key, iv, aad, pt = (bytes.fromhex(v[k]) for k in ("key", "iv", "aad", "pt"))
        ctx = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
        sealed = ctx.encrypt(pt, 0, aad)
        assert sealed.hex() == v["ct"] + v["tag"], v["src"]
        bad = bytearray(sealed)
        bad[-1] ^= 0xFF
        assert ctx.decrypt(bytes(bad), 0, aad) is None
        assert ctx.decrypt(sealed[:15], 0, aad) is None  # inlen < 16 -> SIZE_MAX


def test_tls12_explicit_nonce_via_iv(kat):
    # TLS 1.2 AES-GCM (RFC 5288): nonce = fixed_iv(4) || explicit(8). With the keyset IV set to fixed_iv || 0^8 the
    # engine's nonce rule iv ^ (0^32 || BE64(seq)) (lib/picotls.c:6587-6601) gives exactly that nonce for seq =
    # explicit, so TLS 1.2 records need no separate path; checked on the NIST vectors split that way, in one batch
    vs = [v for v in kat["nist"] if len(bytes.fromhex(v["iv"])) == 12]
    keys = b"".join(bytes.fromhex(v["key"]) for v in vs)
    ivs = b"".join(bytes.fromhex(v["iv"])[:4] + bytes(8) for v in vs)
    seqs = np.array([int.from_bytes(bytes.fromhex(v["iv"])[4:], "big") for v in vs], np.uint64)
    pts = [bytes.fromhex(v["pt"]) for v in vs]
    aads = [bytes.fromhex(v["aad"]) for v in vs]
    b = RecordBatch.build([len(p) for p in pts], [len(a) for a in aads], seqs=seqs, key_idx=np.arange(len(vs)))
    pt = np.zeros(max(b.pt_bytes, 1), np.uint8)
    aad = np.zeros(max(b.aad_bytes, 1), np.uint8)
    for i in range(len(vs)):
        pt[int(b.seal["in_off"][i]):int(b.seal["in_off"][i]) + len(pts[i])] = np.frombuffer(pts[i], np.uint8)
        aad[int(b.seal["aad_off"][i]):int(b.seal["aad_off"][i]) + len(aads[i])] = np.frombuffer(aads[i], np.uint8)
    ks = pa.Keyset(np.frombuffer(keys, np.uint8), np.frombuffer(ivs, np.uint8), len(bytes.fromhex(vs[0]["key"])))
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    for i, v in enumerate(vs):
        o = int(b.seal["out_off"][i])
        assert sealed[o:o + len(pts[i]) + 16].tobytes().hex() == v["ct"] + v["tag"], v["src"]


def test_fusion_vectors_one_multikey_batch(fusion_vectors):
    # every vector of lib/fusion.c's golden set in ONE launch per key size (one key per record: multi-key path)
    for key_size in (16, 32):
        vs = [v for v in fusion_vectors["vectors"] if v["key_size"] == key_size]
        mats = [materialise(v) for v in vs]
        b = RecordBatch.build([len(m[4]) for m in mats], [len(m[3]) for m in mats], seqs=[m[2] for m in mats],
                              key_idx=np.arange(len(vs)))
        keys = b"".join(m[0] for m in mats)
        ivs = b"".join(m[1] for m in mats)
        ks = pa.Keyset(keys, ivs, key_size)
        pt = np.zeros(b.pt_bytes, np.uint8)
        aad = np.zeros(max(b.aad_bytes, 1), np.uint8)
        for i, m in enumerate(mats):
            o = int(b.seal["in_off"][i])
            pt[o:o + len(m[4])] = u8(m[4])
            a = int(b.seal["aad_off"][i])
            aad[a:a + len(m[3])] = u8(m[3])
        sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
        for i, v in enumerate(vs):
            o = int(b.seal["out_off"][i])
            assert check_sealed(v, bytes(sealed[o:o + v["len"] + 16])), (key_size, v["seed"])
        back, ok = gpu_open(ks, b.open, sealed, aad, b.pt_bytes)
        assert ok.all()
        for i, m in enumerate(mats):
            o = int(b.open["out_off"][i])
            assert bytes(back[o:o + len(m[4])]) == m[4]


# ------------------------------------------------------------------------------------------------ randomized


def record_mask(recs, size, field="in_off", extra=0):
    """Byte mask of the arena bytes covered by the records (padding between 16-byte slots excluded)."""
    m = np.zeros(size, bool)
    for o, ln in zip(recs[field], recs["len"]):
        m[int(o):int(o) + int(ln) + extra] = True
    return m


def _random_batch(rng, n, max_len, max_aad, key_size, nkeys=1, sort_keys=True):
    lens = rng.integers(0, max_len + 1, n)
    aads = rng.integers(0, max_aad + 1, n)
    key_idx = rng.integers(0, nkeys, n)
    if sort_keys:
        key_idx = np.sort(key_idx)
    b = RecordBatch.build(lens, aads, seqs=rng.integers(0, 2**63, n, dtype=np.uint64), key_idx=key_idx)
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    return b, keys, ivs, pt, aad


SCHEDULES = ["lockstep", "chunked"]


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("key_size,nkeys,sort_keys", [(16, 1, True), (32, 1, True), (16, 7, True), (32, 50, False)])
def test_random_batch_vs_fusion(ref, key_size, nkeys, sort_keys, schedule):
    rng = np.random.default_rng(key_size * 1000 + nkeys)
    b, keys, ivs, pt, aad = _random_batch(rng, 3000, 3000, 64, key_size, nkeys, sort_keys)
    ks = pa.Keyset(keys, ivs, key_size)
    ks.set_schedule(schedule, allow_variable_time=True)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, key_size, b.seal, pt, aad, expect, nthreads=8)
    assert np.array_equal(sealed, expect)
    back, ok = gpu_open(ks, b.open, sealed, aad, b.pt_bytes)
    assert ok.all()
    m = record_mask(b.seal, b.pt_bytes)
    assert np.array_equal(back[m], pt[m])
    assert not back[~m].any()  # nothing outside the records was written


@pytest.mark.parametrize("key_size", [16, 32])
def test_unit_length_changes_between_runs_vs_fusion(ref, key_size):
    # every workgroup (600 records of a 256 x 600 batch) walks a block of 300 short records then 300 long ones, so its
    # runs get different unit lengths from their scans (run_unit_log2: 8-step, 1-step, then 16-step units) and the
    # combine table is rebuilt under one key between runs; plus a small batch of long records (4-step units, chains of
    # up to 36 partials)
    rng = np.random.default_rng(4242 + key_size)
    blocks = []
    for _ in range(256):
        blocks.append(rng.integers(64, 300, 300))
        blocks.append(rng.integers(4000, 16385, 300))
    for lens, ns in ((np.concatenate(blocks), 256 * 600), (rng.integers(16000, 16500, 90), 90)):
        b = RecordBatch.build(lens[:ns], rng.integers(0, 30, ns), seqs=rng.integers(0, 2**40, ns, dtype=np.uint64))
        keys, ivs = np.frombuffer(rng.bytes(key_size), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
        pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
        aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
        ks = pa.Keyset(keys, ivs, key_size)
        sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
        expect = np.zeros(b.sealed_bytes, np.uint8)
        ref.run_batch(True, keys, ivs, key_size, b.seal, pt, aad, expect, nthreads=8)
        assert np.array_equal(sealed, expect)
        bad = expect.copy()
        victims = rng.choice(ns, 5, replace=False)
        for v in victims:
            bad[int(b.seal[v]["out_off"]) + int(b.seal[v]["len"])] ^= 1
        back, ok = gpu_open(ks, b.open, bad, aad, b.pt_bytes)
        assert sorted(np.nonzero(ok != 1)[0].tolist()) == sorted(victims.tolist())
        m = record_mask(b.seal, b.pt_bytes)
        assert np.array_equal(back[m], pt[m])
        ks.free()


@pytest.mark.parametrize("schedule", SCHEDULES)
def test_every_length_0_to_300_vs_oracle(oracle, schedule):
    # all stream layouts around the G-lane boundaries (partial blocks, AAD-only, empty records)
    rng = np.random.default_rng(7)
    lens = np.arange(0, 301)
    b = RecordBatch.build(lens, (lens * 7) % 41, seqs=lens * 1000003)
    keys, ivs = np.frombuffer(rng.bytes(16), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    ks = pa.Keyset(keys, ivs, 16)
    ks.set_schedule(schedule, allow_variable_time=True)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    oracle.seal_batch(keys, ivs, 16, b.seal, pt, aad, expect)
    assert np.array_equal(sealed, expect)


@pytest.mark.parametrize("schedule", SCHEDULES)
def test_tamper_rejected_per_record(ref, schedule):
    rng = np.random.default_rng(11)
    b, keys, ivs, pt, aad = _random_batch(rng, 512, 2000, 40, 16)
    ks = pa.Keyset(keys, ivs, 16)
    ks.set_schedule(schedule, allow_variable_time=True)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    bad = sealed.copy()
    badaad = aad.copy()
    victims = rng.choice(b.n, 64, replace=False)
    for i, r in enumerate(victims):
        ln = int(b.seal["len"][r])
        kind = i % 3
        if kind == 0 or (kind == 2 and int(b.seal["aad_len"][r]) == 0):  # flip a bit of ciphertext or tag
            off = int(b.open["in_off"][r]) + int(rng.integers(0, ln + 16))
            bad[off] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1:  # flip a tag bit
            bad[int(b.open["in_off"][r]) + ln + int(rng.integers(0, 16))] ^= 0x80
        else:  # flip an AAD bit
            badaad[int(b.seal["aad_off"][r]) + int(rng.integers(0, int(b.seal["aad_len"][r])))] ^= 4
    back, ok = gpu_open(ks, b.open, bad, badaad, b.pt_bytes)
    expect_ok = np.ones(b.n, np.uint8)
    expect_ok[victims] = 0
    assert np.array_equal(ok, expect_ok)
    # like lib/fusion.c (:783-828) the plaintext is written even when the tag fails: compare with fusion's output
    ref_back = np.zeros(b.pt_bytes, np.uint8)
    ref_ok = np.zeros(b.n, np.uint8)
    ref.run_batch(False, keys, ivs, 16, b.open, bad, badaad, ref_back, ok=ref_ok, nthreads=4)
    assert np.array_equal(ref_ok, expect_ok)
    assert np.array_equal(back, ref_back)  # both leave the padding untouched (zero)


def test_unaligned_offsets_and_in_place(oracle):
    rng = np.random.default_rng(13)
    n = 200
    lens = rng.integers(0, 700, n)
    aads = rng.integers(0, 30, n)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    off = 3
    aoff = 1
    for i in range(n):
        recs[i]["in_off"] = off
        recs[i]["out_off"] = off  # in place: ciphertext over plaintext, tag right after it
        recs[i]["len"] = lens[i]
        recs[i]["aad_off"] = aoff
        recs[i]["aad_len"] = aads[i]
        recs[i]["seq"] = i * 977
        off += int(lens[i]) + 16 + int(rng.integers(0, 16))
        aoff += int(aads[i]) + int(rng.integers(0, 5))
    keys, ivs = np.frombuffer(rng.bytes(32), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    arena = np.frombuffer(rng.bytes(off + 16), np.uint8).copy()
    aad = np.frombuffer(rng.bytes(aoff + 1), np.uint8)
    expect = arena.copy()
    oracle.seal_batch(keys, ivs, 32, recs, arena, aad, expect)
    ks = pa.Keyset(keys, ivs, 32)
    d_arena = dev(arena)
    d_recs, d_aad = dev(recs), dev(aad)
    pa.seal_batch(ks, d_recs.data_ptr(), n, d_arena.data_ptr(), d_aad.data_ptr(), d_arena.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(d_arena.cpu().numpy(), expect)
    d_ok = empty(n, 0x55)
    pa.open_batch(ks, d_recs.data_ptr(), n, d_arena.data_ptr(), d_aad.data_ptr(), d_arena.data_ptr(), d_ok.data_ptr())
    torch.cuda.synchronize()
    got = d_arena.cpu().numpy()
    assert d_ok.cpu().numpy().all()
    for i in range(n):
        o, ln = int(recs[i]["in_off"]), int(lens[i])
        assert np.array_equal(got[o:o + ln], arena[o:o + ln])


def test_empty_batch_and_bad_args():
    ks = pa.Keyset(bytes(16), bytes(12), 16)
    pa.seal_batch(ks, 0, 0, 0, 0, 0)  # nrecs = 0 is a no-op
    with pytest.raises(pa.EngineError):
        pa.seal_batch(ks, 0, 5, 0, 0, 0)
    with pytest.raises(ValueError):
        pa.Keyset(bytes(24), bytes(12), 24)


@pytest.mark.parametrize("schedule", SCHEDULES)
def test_max_tls_record_and_large_records(ref, schedule):
    # PTLS_MAX_PLAINTEXT_RECORD_SIZE (lib/picotls.c:52) + the 256-byte TLS 1.3 expansion allowance, and beyond; for the
    # chunked schedule also records of exactly 64 units (the most it splits: 64 * 1 KiB of GHASH stream) and 65
    # (processed whole)
    rng = np.random.default_rng(17)
    lens = [16384, 16384 + 256, 65536, 1 << 20, 16383, 16385, 64 * 1024 - 32, 64 * 1024 - 16, 64 * 1024 - 15]
    b = RecordBatch.build(lens, [5, 5, 13, 13, 0, 32, 0, 0, 0])
    keys, ivs = np.frombuffer(rng.bytes(16), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    ks = pa.Keyset(keys, ivs, 16)
    ks.set_schedule(schedule, allow_variable_time=True)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 16, b.seal, pt, aad, expect, nthreads=4)
    assert np.array_equal(sealed, expect)


@pytest.mark.parametrize("nkeys", [1, 3])
def test_chunked_long_runs_and_key_changes(ref, nkeys):
    # chunked schedule: key runs longer than its 256-record / 1024-unit run window (runs are cut and resumed), keys
    # changing mid-window, open of the same batch, and records of every unit count 1..20
    rng = np.random.default_rng(19 + nkeys)
    n = 700
    lens = np.concatenate([np.full(300, 16384), rng.integers(0, 20 * 1024, n - 300)])
    key_idx = np.sort(rng.integers(0, nkeys, n))
    b = RecordBatch.build(lens, rng.integers(0, 30, n), seqs=rng.integers(0, 2**40, n, dtype=np.uint64),
                          key_idx=key_idx)
    keys = np.frombuffer(rng.bytes(nkeys * 32), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, 32)
    ks.set_schedule("chunked")
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 32, b.seal, pt, aad, expect, nthreads=8)
    assert np.array_equal(sealed, expect)
    back, ok = gpu_open(ks, b.open, sealed, aad, b.pt_bytes)
    assert ok.all()
    m = record_mask(b.seal, b.pt_bytes)
    assert np.array_equal(back[m], pt[m])


@pytest.mark.parametrize("length,n,nkeys", [(1200, 9000, 1), (16384, 700, 1), (1200, 3000, 5), (1201, 4500, 1)])
def test_chunked_uniform_runs_vs_fusion(ref, length, n, nkeys):
    # uniform runs take the whole-record path of the chunked schedule (one-key runs up to 4096 records)
    rng = np.random.default_rng(length + n + nkeys)
    lens = np.full(n, length)
    if length == 1201:
        lens[::97] = 1200  # within the uniformity slack
    b = RecordBatch.build(lens, 13, seqs=np.arange(n, dtype=np.uint64) * 3, key_idx=np.sort(rng.integers(0, nkeys, n)))
    keys = np.frombuffer(rng.bytes(nkeys * 16), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    ks = pa.Keyset(keys, ivs, 16)
    ks.set_schedule("chunked")
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 16, b.seal, pt, aad, expect, nthreads=8)
    assert np.array_equal(sealed, expect)
    back, ok = gpu_open(ks, b.open, sealed, aad, b.pt_bytes)
    assert ok.all()
    m = record_mask(b.seal, b.pt_bytes)
    assert np.array_equal(back[m], pt[m])


def test_hp_masks_kat_batch(kat):
    # t/fusion.c:290-344 supp vectors as ONE batch: seal 19 records, then the header-protection masks of the samples at
    # sealed + 2 (the sample covers the tag for the short records)
    t = kat["gcm_zero_ctr_tags"]
    cases = t["cases"]
    lens = [c[1] for c in cases]
    b = RecordBatch.build(lens, [c[0] for c in cases], seqs=np.zeros(len(cases), np.uint64))
    pt = np.zeros(b.pt_bytes, np.uint8)
    aad = np.zeros(max(b.aad_bytes, 1), np.uint8)
    ks = pa.Keyset(bytes(16), bytes(12), 16)
    hp_ks = pa.Keyset(bytes.fromhex(t["hp_key"]), bytes(12), 16)
    hp = np.zeros(len(cases), dtype=pa.HP_DTYPE)
    hp["sample_off"] = b.seal["out_off"] + t["hp_sample_off"]
    d_recs, d_pt, d_aad, d_hp = dev(b.seal), dev(pt), dev(aad), dev(hp)
    d_out, d_masks = empty(b.sealed_bytes), empty(16 * len(cases), 0x5A)
    pa.seal_batch_hp(ks, d_recs.data_ptr(), len(cases), d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), hp_ks,
                     d_hp.data_ptr(), d_masks.data_ptr())
    torch.cuda.synchronize()
    out, masks = d_out.cpu().numpy(), d_masks.cpu().numpy().reshape(-1, 16)
    for i, (aadlen, ptlen, tag, mask) in enumerate(cases):
        o = int(b.seal["out_off"][i])
        assert out[o + ptlen:o + ptlen + 16].tobytes().hex() == tag
        assert masks[i].tobytes().hex() == mask, i


@pytest.mark.parametrize("key_size,n,nkeys,sort_keys,schedule", [(16, 300, 5, True, "auto"), (32, 300, 5, True, "auto"),
                                                                  (16, 3000, 40, False, "auto"), (32, 700, 3, True, "lockstep"),
                                                                  (16, 20000, 1, True, "auto")])
def test_hp_masks_vs_fusion_supp(ref, key_size, n, nkeys, sort_keys, schedule):
    # random QUIC-like packets through seal_batch_hp against fusion's encrypt_s with supp (lib/fusion.c:425-430,
    # 636-651), per-connection HP keys, sample offset 4 - pn_len into the ciphertext; then the receive-side masks of
    # the same samples with hp_mask_batch. The chunked schedule computes the masks in the seal launch (each run's masks
    # after its records), also for batches regrouped by key on the device and uniform one-key batches (whole-record
    # runs); the lockstep schedule runs a second launch.
    rng = np.random.default_rng(23 + key_size + n)
    lens = rng.integers(20, 1500, n) if nkeys > 1 else np.full(n, 1200)
    key_idx = rng.integers(0, nkeys, n)
    if sort_keys:
        key_idx = np.sort(key_idx)
    b = RecordBatch.build(lens, rng.integers(8, 30, n), seqs=rng.integers(0, 2**40, n, dtype=np.uint64), key_idx=key_idx)
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    hp_keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    sample_in_ct = 4 - rng.integers(1, 5, n)
    hp = np.zeros(n, dtype=pa.HP_DTYPE)
    hp["sample_off"] = b.seal["out_off"] + sample_in_ct
    hp["key_idx"] = key_idx
    hp["key_idx"][7] = nkeys + 3  # out of range: zero mask
    ks, hp_ks = pa.Keyset(keys, ivs, key_size), pa.Keyset(hp_keys, np.zeros(nkeys * 12, np.uint8), key_size)
    ks.set_schedule(schedule, allow_variable_time=True)
    d_recs, d_pt, d_aad, d_hp = dev(b.seal), dev(pt), dev(aad), dev(hp)
    d_out, d_masks, d_masks2 = empty(b.sealed_bytes), empty(16 * n, 0x5A), empty(16 * n, 0x5A)
    pa.seal_batch_hp(ks, d_recs.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), hp_ks,
                     d_hp.data_ptr(), d_masks.data_ptr())
    pa.hp_mask_batch(hp_ks, d_hp.data_ptr(), n, d_out.data_ptr(), d_masks2.data_ptr())
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    masks = d_masks.cpu().numpy().reshape(-1, 16)
    assert np.array_equal(masks, d_masks2.cpu().numpy().reshape(-1, 16))
    for i in range(n):
        k = int(key_idx[i])
        kb, ivb, hkb = (bytes(a[k * w:(k + 1) * w]) for a, w in ((keys, key_size), (ivs, 12), (hp_keys, key_size)))
        io, oo, ln = int(b.seal["in_off"][i]), int(b.seal["out_off"][i]), int(lens[i])
        ao, al = int(b.seal["aad_off"][i]), int(b.seal["aad_len"][i])
        sealed, mask = ref.seal_with_hp(kb, ivb, int(b.seal["seq"][i]), bytes(aad[ao:ao + al]), bytes(pt[io:io + ln]), hkb,
                                        int(sample_in_ct[i]))
        assert out[oo:oo + ln + 16].tobytes() == sealed, i
        assert masks[i].tobytes() == (bytes(16) if i == 7 else mask), i


@pytest.mark.parametrize("in_place,nkeys", [(False, 1), (True, 1), (False, 30), (True, 30)])
def test_hp_masks_edges_vs_fusion(ref, in_place, nkeys):
    # seal_batch_hp with samples anywhere in the sealed record (its first byte, the middle, the last 16 bytes = the tag
    # itself), records of one unit and of several (mixed lengths to 16 KiB: cut runs, the tag written by the unit
    # combine), sealed in place (the masks' pass reads samples where the kernel read plaintext) and not, one key and
    # per-connection keys, beside rejected descriptors (nothing written) and an out-of-range header-protection key (a
    # zero mask)
    rng = np.random.default_rng(77 + 2 * nkeys + in_place)
    n = 700
    lens = rng.integers(17, 16385, n)
    lens[:100] = 1200
    key_idx = np.sort(rng.integers(0, nkeys, n))
    b = RecordBatch.build(lens, rng.integers(0, 30, n), seqs=rng.integers(0, 2**40, n, dtype=np.uint64), key_idx=key_idx)
    key_size = 16
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    hp_keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    recs = b.seal.copy()
    if in_place:  # the plaintext sits where its ciphertext goes
        arena = np.zeros(b.sealed_bytes, np.uint8)
        for i in range(n):
            io, oo, ln = int(recs["in_off"][i]), int(recs["out_off"][i]), int(lens[i])
            arena[oo:oo + ln] = pt[io:io + ln]
        recs["in_off"] = recs["out_off"]
    off = rng.integers(0, lens + 1)  # sample start inside the sealed record: [0, len]
    off[0], off[1], off[101] = 0, lens[1], lens[101]  # the first byte; the tag itself (one-unit and multi-unit records)
    hp = np.zeros(n, dtype=pa.HP_DTYPE)
    hp["sample_off"] = recs["out_off"] + off
    hp["key_idx"] = key_idx
    hp["key_idx"][7] = nkeys  # out-of-range header-protection key: a zero mask
    rejected = (8, 300)
    recs["key_idx"][8] = nkeys + 9  # rejected descriptors: nothing is written for them
    recs["len"][300] = (1 << 30) + 1  # (over PTLS_MI355X_MAX_RECORD_LEN)
    ks, hp_ks = pa.Keyset(keys, ivs, key_size), pa.Keyset(hp_keys, np.zeros(nkeys * 12, np.uint8), key_size)
    d_recs, d_aad, d_hp = dev(recs), dev(aad), dev(hp)
    d_masks = empty(16 * n, 0x5A)
    if in_place:
        d_in = d_out = dev(arena)
    else:
        d_in, d_out = dev(pt), empty(b.sealed_bytes, 0x33)
    pa.seal_batch_hp(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), hp_ks,
                     d_hp.data_ptr(), d_masks.data_ptr())
    torch.cuda.synchronize()
    out, masks = d_out.cpu().numpy(), d_masks.cpu().numpy().reshape(-1, 16)
    for i in range(n):
        io, oo, ln = int(b.seal["in_off"][i]), int(b.seal["out_off"][i]), int(lens[i])
        if i in rejected:  # untouched output
            want = arena[oo:oo + ln + 16] if in_place else np.full(ln + 16, 0x33, np.uint8)
            assert np.array_equal(out[oo:oo + ln + 16], want), i
            continue
        k = int(key_idx[i])
        kb, ivb, hkb = (bytes(a[k * w:(k + 1) * w]) for a, w in ((keys, key_size), (ivs, 12), (hp_keys, key_size)))
        ao, al = int(b.seal["aad_off"][i]), int(b.seal["aad_len"][i])
        sealed, mask = ref.seal_with_hp(kb, ivb, int(b.seal["seq"][i]), bytes(aad[ao:ao + al]), bytes(pt[io:io + ln]), hkb,
                                        int(off[i]))
        assert out[oo:oo + ln + 16].tobytes() == sealed, i
        assert masks[i].tobytes() == (bytes(16) if i == 7 else mask), i


def _tls_header(n):
    return bytes([23, 3, 3, n >> 8, n & 0xFF])


@pytest.mark.parametrize("key_size,nkeys", [(16, 1), (32, 4), (16, 97)])
def test_tls_records_seal_vs_fusion(ref, key_size, nkeys):
    # wire records equal picotls' record layer (lib/picotls.c:728-738): header || AEAD(payload || type) with the header
    # as AAD, computed here with lib/fusion.c's ptls_aead_encrypt on the same inputs (the many-key case in random key
    # order: grouped on the device)
    rng = np.random.default_rng(29 + nkeys)
    n = 400
    lens = rng.integers(0, 16385, n)
    lens[:4] = [0, 1, 15, 16384]
    types = rng.choice([21, 22, 23], n).astype(np.uint16)
    key_idx = rng.integers(0, nkeys, n)
    if nkeys < 10:
        key_idx = np.sort(key_idx)
    seqs = rng.integers(0, 2**40, n, dtype=np.uint64)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    pin, pout = 0, 0
    for i in range(n):
        recs[i]["in_off"], recs[i]["out_off"] = pin, pout
        recs[i]["len"], recs[i]["seq"], recs[i]["key_idx"], recs[i]["flags"] = lens[i], seqs[i], key_idx[i], types[i]
        pin += int(lens[i]) + int(rng.integers(0, 9))
        pout += int(lens[i]) + 22 + int(rng.integers(0, 9))
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(pin + 1), np.uint8)
    ks = pa.Keyset(keys, ivs, key_size)
    d_recs, d_pt, d_out = dev(recs), dev(pt), empty(pout + 1, 0xEE)
    pa.seal_tls_records(ks, d_recs.data_ptr(), n, d_pt.data_ptr(), d_out.data_ptr())
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i in range(n):
        k, ln = int(key_idx[i]), int(lens[i])
        io, oo = int(recs[i]["in_off"]), int(recs[i]["out_off"])
        hdr = _tls_header(ln + 17)
        inner = bytes(pt[io:io + ln]) + bytes([int(types[i])])
        expect = hdr + ref.seal(bytes(keys[k * key_size:(k + 1) * key_size]), bytes(ivs[k * 12:(k + 1) * 12]),
                                int(seqs[i]), hdr, inner)
        assert out[oo:oo + ln + 22].tobytes() == expect, i
    # nothing outside the wire records was written
    m = np.zeros(out.size, bool)
    for i in range(n):
        m[int(recs[i]["out_off"]):int(recs[i]["out_off"]) + int(lens[i]) + 22] = True
    assert (out[~m] == 0xEE).all()


def test_tls_records_open_strip_and_reject(ref):
    # receive side (lib/picotls.c:5952-5974): padding strip, inner type, and the failure classes
    rng = np.random.default_rng(31)
    key, iv = rng.bytes(16), rng.bytes(12)
    cases = []  # (inner plaintext, tamper kind)
    for i in range(120):
        body = rng.bytes(int(rng.integers(0, 3000)))
        inner = body + bytes([int(rng.choice([21, 22, 23]))]) + bytes(int(rng.integers(0, 300)))
        cases.append((inner, None))
    cases += [(bytes(40), None), (bytes([21]), None), (bytes([22]) + bytes(9), None), (bytes([23]), None),
              (b"hello" + bytes([23]), "ct"), (b"hello" + bytes([23]), "tag"), (b"hello" + bytes([23]), "hdr_type"),
              (b"hello" + bytes([23]), "hdr_len"), (b"x" * 5000 + bytes([23]) + bytes(100), None)]
    n = len(cases)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    wire = bytearray()
    pout = 0
    for i, (inner, kind) in enumerate(cases):
        L = len(inner)
        hdr = _tls_header(L + 16)
        rec = bytearray(hdr + ref.seal(key, iv, 1000 + i, hdr, inner))
        if kind == "ct":
            rec[5] ^= 1
        elif kind == "tag":
            rec[-1] ^= 0x80
        elif kind == "hdr_type":
            rec[0] = 22
        elif kind == "hdr_len":
            rec[4] ^= 1
        recs[i]["in_off"], recs[i]["out_off"], recs[i]["len"], recs[i]["seq"] = len(wire), pout, L, 1000 + i
        wire += rec + bytes(int(rng.integers(0, 7)))
        pout += L + 3
    ks = pa.Keyset(key, iv, 16)
    d_recs, d_in, d_out = dev(recs), dev(np.frombuffer(bytes(wire), np.uint8)), empty(pout + 1)
    d_ok, d_res = empty(n, 0x77), empty(8 * n, 0x77)
    pa.open_tls_records(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_out.data_ptr(), d_ok.data_ptr(), d_res.data_ptr())
    torch.cuda.synchronize()
    ok = d_ok.cpu().numpy()
    res = d_res.cpu().numpy().view(pa.TLS_RESULT_DTYPE)
    out = d_out.cpu().numpy()
    for i, (inner, kind) in enumerate(cases):
        if kind in ("ct", "tag", "hdr_len"):  # a wrong length field changes the AAD, so the tag fails first
            assert res[i]["status"] == pa.TLS_BAD_MAC and ok[i] == 0, i
            continue
        if kind == "hdr_type":  # the header is authenticated too
            assert res[i]["status"] == pa.TLS_BAD_MAC and ok[i] == 0, i
            continue
        stripped = inner.rstrip(b"\x00")
        if not stripped or (len(stripped) == 1 and stripped[0] in (21, 22)):
            assert res[i]["status"] == pa.TLS_UNEXPECTED_MESSAGE and ok[i] == 0, i
            continue
        assert res[i]["status"] == pa.TLS_OK and ok[i] == 1, i
        assert res[i]["content_type"] == stripped[-1]
        assert res[i]["plain_len"] == len(stripped) - 1
        o = int(recs[i]["out_off"])
        assert out[o:o + len(inner)].tobytes() == inner


def test_tls_records_round_trip_bad_header_after_valid_tag():
    # a record whose tag verifies under a header that is not {23,3,3,len+16}: sealed by the engine with a
    # non-application outer type is impossible, so build one with seal_batch and a custom 5-byte AAD
    rng = np.random.default_rng(37)
    key, iv = rng.bytes(16), rng.bytes(12)
    inner = b"abc" + bytes([23])
    hdr = bytes([22, 3, 3, 0, len(inner) + 16])
    b = RecordBatch.build([len(inner)], [5], seqs=np.array([5], np.uint64))
    ks = pa.Keyset(key, iv, 16)
    sealed = gpu_seal(ks, b.seal, np.frombuffer(inner, np.uint8), np.frombuffer(hdr, np.uint8), b.sealed_bytes)
    wire = hdr + sealed[:len(inner) + 16].tobytes()
    recs = np.zeros(1, dtype=pa.RECORD_DTYPE)
    recs[0]["len"], recs[0]["seq"] = len(inner), 5
    d_recs, d_in, d_out, d_ok, d_res = dev(recs), dev(np.frombuffer(wire, np.uint8)), empty(16), empty(1), empty(8)
    pa.open_tls_records(ks, d_recs.data_ptr(), 1, d_in.data_ptr(), d_out.data_ptr(), d_ok.data_ptr(), d_res.data_ptr())
    torch.cuda.synchronize()
    res = d_res.cpu().numpy().view(pa.TLS_RESULT_DTYPE)
    assert res[0]["status"] == pa.TLS_BAD_HEADER and d_ok.cpu().numpy()[0] == 0


def test_schedule_argument_checked():
    ks = pa.Keyset(bytes(16), bytes(12), 16)
    with pytest.raises(ValueError):
        ks.set_schedule("fastest")
    assert pa.load_library().ptls_mi355x_keyset_set_schedule(ks.handle, 7) == -1


@pytest.mark.parametrize("combine", [None, "1", "4"])
def test_picotls_vtable_pairs(combine):
    # cross-backend pairs in the reference's style (t/picotls.c:224-370): seal with fusion / open with MI355X and back,
    # through ptls_aead_new_direct + the ptls_aead_algorithm_t objects (tests/c/test_vtable.c); its thread tests run the
    # per-record calls each on its own (the default) and combined across threads with 1 (the largest batches) and 4
    # launches in flight per kind (PTLS_MI355X_COMBINE)
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "_bin", "test_vtable")
    if not os.path.exists(exe):
        pytest.skip("tests/c/_bin/test_vtable not built (needs picotls headers at build time)")
    env = dict(os.environ)
    if combine is not None:
        env["PTLS_MI355X_COMBINE"] = combine
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "not ok" not in r.stdout


@pytest.mark.parametrize("copy_path", [False, True])
def test_picotls_vtable_fail_closed(copy_path):
    # an engine failure inside ptls_aead_encrypt (here: a record above the staging cap set for this process) leaves
    # zeros in the output, never the plaintext (sealed in place), and the process keeps working; the same binary also
    # checks that ptls_mi355x_last_error() names the cause. copy_path: the staging round trip through device memory
    # (PTLS_MI355X_STAGE_COPY=1) instead of the mapped pinned buffer.
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "_bin", "test_vtable")
    if not os.path.exists(exe):
        pytest.skip("tests/c/_bin/test_vtable not built (needs picotls headers at build time)")
    env = dict(os.environ, PTLS_MI355X_MAX_STAGE_BYTES="65536")
    if copy_path:
        env["PTLS_MI355X_STAGE_COPY"] = "1"
    r = subprocess.run([exe, "failclosed"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "not ok" not in r.stdout


def test_picotls_vtable_tls12_with_handled_errors_left_on_the_thread():
    """Regression test of the round-3 TLS 1.2 failure's demonstrated mechanism (VERDICT round 4, weak
    item 1): in a fresh process, before every engine call of picotls' TLS 1.2 ptls_send (16384 + 16384 + 7232 bytes: the
    first uses of two staging size classes) and of each ptls_receive of fusion's records, and before per-record seals
    and opens of those lengths, the thread is left holding the HIP error a handled hipHostGetDevicePointer failure leaves
    (ptls_mi355x_debug_inject_error). Every wire byte, receive and plaintext equals fusion's. (The same binary fails
    these checks against an engine built with -DLAUNCH_CLEAR_NOOP=1: profiles/r5/lasterr_regression.txt.)"""
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "_bin", "test_vtable")
    if not os.path.exists(exe):
        pytest.skip("tests/c/_bin/test_vtable not built (needs picotls headers at build time)")
    r = subprocess.run([exe, "lasterr"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "not ok" not in r.stdout and "# 0 failed" in r.stdout


def test_raw_context_api_vs_fusion():
    """The counterparts of fusion's raw context API (include/picotls/mi355x_picotls.h ptls_mi355x_aesgcm_* /
    ptls_mi355x_aesecb_*; include/picotls/fusion.h:40-94), driven beside ptls_fusion_aesgcm_* with the same __m128i
    counter: records of 0-69,999 bytes with AADs to 290 bytes, both key sizes, capacity growth, decryption of each
    other's records, bad tags and tampered ciphertext (plaintext written as fusion's), AES-ECB blocks (tests/c/test_vtable.c
    raw_context_test)."""
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "_bin", "test_vtable")
    if not os.path.exists(exe):
        pytest.skip("tests/c/_bin/test_vtable not built (needs picotls headers at build time)")
    r = subprocess.run([exe, "raw"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "not ok" not in r.stdout and "# 0 failed" in r.stdout


def test_picotls_vtable_pairs_copy_path():
    # the whole vtable suite with the staging round trip copying through device memory (PTLS_MI355X_STAGE_COPY=1)
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "_bin", "test_vtable")
    if not os.path.exists(exe):
        pytest.skip("tests/c/_bin/test_vtable not built (needs picotls headers at build time)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=dict(os.environ, PTLS_MI355X_STAGE_COPY="1"))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "not ok" not in r.stdout


@pytest.mark.parametrize("key_size", [16, 32])
def test_per_record_path_every_unit_size_vs_fusion(ref, key_size):
    # the per-record path (ptls_aead_encrypt / decrypt through the vtable = a launch of one record) cuts the record into
    # units of 1, 2, 4, 8 or 16 steps by its length, each recombined with its own power H^(8 * steps); lengths across
    # every choice and its boundaries, against fusion, plus a tampered tag
    rng = np.random.default_rng(600 + key_size)
    key, iv = rng.bytes(key_size), rng.bytes(12)
    alg = pa.aes128gcm if key_size == 16 else pa.aes256gcm
    enc = pa.aead_new_direct(alg, True, key, iv)
    dec = pa.aead_new_direct(alg, False, key, iv)
    # steps = ceil((ceil(A/16) + ceil(L/16) + 1) / 8) with A = 13: switch points 24 / 96 / 400 / 1600 steps
    lens = [0, 1, 100, 1200, 2900, 2950, 3000, 12000, 12300, 16384, 16640, 51000, 51300, 60000, 204700, 204900, 300000,
            1 << 20]
    for ln in lens:
        pt, aad, seq = rng.bytes(ln), rng.bytes(13), int(rng.integers(0, 2**48))
        want = ref.seal(key, iv, seq, aad, pt)
        got = enc.encrypt(pt, seq, aad)
        assert got == want, ln
        assert dec.decrypt(want, seq, aad) == pt, ln
        bad = bytearray(want)
        bad[-1] ^= 0x40
        assert dec.decrypt(bytes(bad), seq, aad) is None, ln


@pytest.mark.parametrize("schedule", ["lockstep", "chunked"])
def test_invalid_descriptor_rejected(ref, schedule):
    # a descriptor whose len exceeds PTLS_MI355X_MAX_RECORD_LEN (corrupt, or up to 2^32 - 1) or whose key_idx is not in
    # the keyset is rejected as a whole: nothing is written for it, open reports ok = 0, and the other records of the
    # batch are unaffected
    rng = np.random.default_rng(610)
    n = 40
    lens = rng.integers(0, 3000, n)
    b = RecordBatch.build(lens, rng.integers(0, 30, n), seqs=rng.integers(0, 2**40, n, dtype=np.uint64))
    keys, ivs = np.frombuffer(rng.bytes(16), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 16, b.seal, pt, aad, expect, nthreads=2)
    bad = [3, 17, 39, 25, 8]
    seal, opn = b.seal.copy(), b.open.copy()
    for i, v in zip(bad, [(1 << 30) + 1, 0xFFFFFFFF, 0xFFFFFFF0]):  # PTLS_MI355X_MAX_RECORD_LEN = 2^30
        seal[i]["len"] = opn[i]["len"] = v
    seal[25]["key_idx"] = opn[25]["key_idx"] = 5  # a one-key keyset: key 5 does not exist
    seal[8]["flags"] = opn[8]["flags"] = 0x4001  # AAD length above PTLS_MI355X_MAX_AAD_LEN (bits 16..31 in flags)
    ks = pa.Keyset(keys, ivs, 16)
    ks.set_schedule(schedule, allow_variable_time=True)
    sealed = gpu_seal(ks, seal, pt, aad, b.sealed_bytes, out_fill=0xEE)
    for i, r in enumerate(b.seal):
        o, ln = int(r["out_off"]), int(r["len"]) + 16
        if i in bad:
            assert (sealed[o:o + ln] == 0xEE).all(), i
        else:
            assert np.array_equal(sealed[o:o + ln], expect[o:o + ln]), i
    plain, ok = gpu_open(ks, opn, expect, aad, b.pt_bytes, out_fill=0x55)
    assert [int(x) for x in ok] == [0 if i in bad else 1 for i in range(n)]
    for i, r in enumerate(b.open):
        o, ln = int(r["out_off"]), int(r["len"])
        want = np.full(ln, 0x55, np.uint8) if i in bad else pt[int(b.seal[i]["in_off"]):int(b.seal[i]["in_off"]) + ln]
        assert np.array_equal(plain[o:o + ln], want), i


def test_records_beyond_1024_units_chunked(ref):
    # records needing more than 1024 units of 2 KiB (> 2 MiB) take units of a multiple length (their partials combined
    # with the unit power applied that many times) instead of running whole on one group; up to
    # PTLS_MI355X_MAX_RECORD_LEN, next to ordinary records in the same run, sealed and opened (one tampered)
    rng = np.random.default_rng(620)
    lens = [3 << 20, 16384, (5 << 20) + 7, (2 << 20) + 1, 1 << 24, 1200, (2 << 20) - 40]
    n = len(lens)
    b = RecordBatch.build(lens, [13] * n, seqs=rng.integers(0, 2**40, n, dtype=np.uint64))
    keys, ivs = np.frombuffer(rng.bytes(32), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    ks = pa.Keyset(keys, ivs, 32)
    ks.set_schedule("chunked")
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 32, b.seal, pt, aad, expect, nthreads=4)
    assert np.array_equal(sealed, expect)
    bad = expect.copy()
    bad[int(b.seal[4]["out_off"]) + 12345] ^= 1
    plain, ok = gpu_open(ks, b.open, bad, aad, b.pt_bytes)
    assert [int(x) for x in ok] == [1, 1, 1, 1, 0, 1, 1]
    want = pt.copy()
    want[int(b.seal[4]["in_off"]) + 12345] ^= 1  # plaintext is written regardless, like fusion (CTR: the flipped bit)
    for r in b.open:
        o, ln = int(r["out_off"]), int(r["len"])
        assert np.array_equal(plain[o:o + ln], want[o:o + ln]), ln


@pytest.mark.parametrize("nkeys,frac_bad", [(300, 0.0), (4096, 0.02)])
def test_ungrouped_many_key_batch_regrouped_on_device(ref, nkeys, frac_bad):
    # records of many connections in random order (SURVEY 8(d) config 4 as written) are grouped by key on the device
    # before the chunked kernel (key_hist / key_scan / key_scatter); results and ok bytes stay at each record's own
    # index, out-of-range keys are rejected wherever they sit, and a second batch on the same keyset reuses the scratch
    rng = np.random.default_rng(630 + nkeys)
    n = 6000
    lens = rng.integers(0, 5000, n)
    key_idx = rng.integers(0, nkeys, n)
    bad = rng.random(n) < frac_bad
    key_idx[bad] = nkeys + rng.integers(0, 5, int(bad.sum()))
    b = RecordBatch.build(lens, rng.integers(0, 40, n), seqs=rng.integers(0, 2**48, n, dtype=np.uint64), key_idx=key_idx)
    keys = np.frombuffer(rng.bytes(nkeys * 32), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, 32)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    good = np.flatnonzero(~bad)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 32, b.seal[good], pt, aad, expect, nthreads=8)
    for i in range(n):
        o, ln = int(b.seal[i]["out_off"]), int(b.seal[i]["len"]) + 16
        if bad[i]:
            assert not sealed[o:o + ln].any(), i  # nothing written (the arena starts zeroed)
        else:
            assert np.array_equal(sealed[o:o + ln], expect[o:o + ln]), i
    back, ok = gpu_open(ks, b.open, expect, aad, b.pt_bytes)
    assert np.array_equal(ok.astype(bool), ~bad)
    for i in good:
        o, ln = int(b.open[i]["out_off"]), int(b.open[i]["len"])
        assert np.array_equal(back[o:o + ln], pt[o:o + ln]), i
    # the same keyset again, grouped order this time (no regrouping needed)
    order = np.argsort(key_idx, kind="stable")
    sealed2 = gpu_seal(ks, b.seal[order], pt, aad, b.sealed_bytes)
    assert np.array_equal(sealed2, sealed)


def test_many_key_batch_in_bursts_regrouped_on_device(ref):
    # (round 5) connections sending bursts of 6-20 records, the bursts in random order: runs average ~13 records, above
    # the 8-record rule, but outnumber the 1000 keys more than twice (and reach KEY_REGROUP_MIN_RUNS), so key_regroup
    # groups the batch (aux_kernels.h); a W8-sized batch with every key's bursts spread over it, against fusion, seal
    # and open
    rng = np.random.default_rng(655)
    nkeys, bursts = 1000, []
    for k in range(nkeys):
        left = 120
        while left > 0:
            m = min(left, int(rng.integers(6, 21)))
            bursts.append((k, m))
            left -= m
    rng.shuffle(bursts)
    key_idx = np.concatenate([np.full(m, k, np.int64) for k, m in bursts])
    n = len(key_idx)
    changes = int((key_idx[1:] != key_idx[:-1]).sum())
    assert changes * 8 <= n and changes >= 2 * nkeys and changes * 32 > n and changes >= 8192  # only the burst rule
    lens = rng.integers(0, 1500, n)
    b = RecordBatch.build(lens, rng.integers(0, 30, n), seqs=rng.integers(0, 2**48, n, dtype=np.uint64), key_idx=key_idx)
    keys = np.frombuffer(rng.bytes(nkeys * 16), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, 16)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 16, b.seal, pt, aad, expect, nthreads=8)
    assert np.array_equal(sealed, expect)
    bad = expect.copy()
    tamper = rng.choice(n, 7, replace=False)
    for i in tamper:
        bad[int(b.seal[i]["out_off"]) + int(b.seal[i]["len"])] ^= 0x40  # the tag's first byte
    back, ok = gpu_open(ks, b.open, bad, aad, b.pt_bytes)
    want_ok = np.ones(n, bool)
    want_ok[tamper] = False
    assert np.array_equal(ok.astype(bool), want_ok)
    for i in range(n):
        o, ln = int(b.open[i]["out_off"]), int(b.open[i]["len"])
        assert np.array_equal(back[o:o + ln], pt[o:o + ln]), i


# n = 1, 2, 33: one workgroup or a few; n = 256 * k: k records per workgroup on a 256-CU MI355X (one persistent
# workgroup per CU once a batch has >= 32 records per CU)
@pytest.mark.parametrize("n", [1, 2, 33, 300, 1000, 256 * 63, 256 * 64, 256 * 65, 256 * 129, 256 * 256])
def test_first_run_sizes(ref, n):
    # a launch's first run is scanned by the guarded scan (scan_run<..., FIRST>): its loops stop at the run's last
    # 64-record block, a lone record skips the front-unit sort and a run of at most 64 records is ranked directly;
    # workgroup shares around those edges, with mixed lengths so that runs are cut into units (not whole-record mode),
    # one record longer than 1024 units
    rng = np.random.default_rng(640 + n)
    lens = rng.integers(0, 40000 if n < 64 else 3000, n)
    lens[int(rng.integers(0, n))] = (3 << 20) + 5
    b = RecordBatch.build(lens, rng.integers(0, 30, n), seqs=rng.integers(0, 2**48, n, dtype=np.uint64))
    keys, ivs = np.frombuffer(rng.bytes(16), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, 16)
    ks.set_schedule("chunked")
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 16, b.seal, pt, aad, expect, nthreads=8)
    assert np.array_equal(sealed, expect)
    victim = int(rng.integers(0, n))
    bad = expect.copy()
    bad[int(b.seal[victim]["out_off"]) + int(lens[victim])] ^= 0x01  # first tag byte
    plain, ok = gpu_open(ks, b.open, bad, aad, b.pt_bytes)
    want_ok = np.ones(n, np.uint8)
    want_ok[victim] = 0
    assert np.array_equal(ok, want_ok)
    mask = record_mask(b.open, b.pt_bytes, field="out_off")
    assert np.array_equal(plain[mask], pt[mask])
    ks.free()


def test_lone_huge_record_per_record_path(ref):
    # the picotls vtable's batch of one with a record beyond 1024 units (the lone-record scan marks it huge)
    rng = np.random.default_rng(650)
    key, iv = rng.bytes(16), rng.bytes(12)
    enc = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
    dec = pa.aead_new_direct(pa.aes128gcm, False, key, iv)
    for ln in [(3 << 20) + 5, 1 << 24]:
        pt, aad, seq = rng.bytes(ln), rng.bytes(13), int(rng.integers(0, 2**48))
        want = ref.seal(key, iv, seq, aad, pt)
        assert enc.encrypt(pt, seq, aad) == want, ln
        assert dec.decrypt(want, seq, aad) == pt, ln
        bad = bytearray(want)
        bad[ln // 2] ^= 0x10
        assert dec.decrypt(bytes(bad), seq, aad) is None, ln


def test_batch_on_pinned_host_arenas(ref):
    # the batch calls take pinned (device-mapped) host memory for every arena, descriptors and ok bytes included: the
    # kernels read and write it over PCIe (bench.py --e2e "in_place"); bit-exact vs fusion, one tampered record
    rng = np.random.default_rng(660)
    n = 3000
    lens = rng.integers(0, 20000, n)
    b = RecordBatch.build(lens, rng.integers(0, 30, n), seqs=rng.integers(0, 2**48, n, dtype=np.uint64))
    keys, ivs = np.frombuffer(rng.bytes(32), np.uint8), np.frombuffer(rng.bytes(12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)

    def pinned(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).pin_memory()

    h_seal, h_open, h_pt, h_aad = pinned(b.seal), pinned(b.open), pinned(pt), pinned(aad)
    h_sealed = torch.zeros(b.sealed_bytes, dtype=torch.uint8).pin_memory()
    ks = pa.Keyset(keys, ivs, 32)
    s = torch.cuda.current_stream().cuda_stream
    pa.seal_batch(ks, h_seal.data_ptr(), n, h_pt.data_ptr(), h_aad.data_ptr(), h_sealed.data_ptr(), s)
    torch.cuda.synchronize()
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 32, b.seal, pt, aad, expect, nthreads=8)
    assert np.array_equal(h_sealed.numpy(), expect)
    victim = 1234
    h_sealed[int(b.seal[victim]["out_off"]) + 7] ^= 0x20
    h_back = torch.zeros(b.pt_bytes, dtype=torch.uint8).pin_memory()
    h_ok = torch.full((n,), 0xAA, dtype=torch.uint8).pin_memory()
    pa.open_batch(ks, h_open.data_ptr(), n, h_sealed.data_ptr(), h_aad.data_ptr(), h_back.data_ptr(), h_ok.data_ptr(), s)
    torch.cuda.synchronize()
    want_ok = np.ones(n, np.uint8)
    want_ok[victim] = 0
    assert np.array_equal(h_ok.numpy(), want_ok)
    want = pt.copy()
    want[int(b.seal[victim]["in_off"]) + 7] ^= 0x20  # CTR: the flipped ciphertext bit flips the plaintext bit
    mask = record_mask(b.open, b.pt_bytes, field="out_off")
    assert np.array_equal(h_back.numpy()[mask], want[mask])
    ks.free()
