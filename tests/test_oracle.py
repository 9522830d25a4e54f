"""Pins the CPU oracle (oracle/gcm_ref.c) to the reference's own known answers and to lib/fusion.c.

CPU only. The oracle is test infrastructure; the HIP engine is checked against it in test_gpu_parity.py.
"""
import os

import numpy as np
import pytest

from oracle import FusionRef, GcmOracle
from vecs import check_sealed, h_from_fusion_internal, materialise

HAVE_REF = os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                                       "libfusion_ref.so"))


@pytest.fixture(scope="module")
def oracle():
    return GcmOracle()


def test_ecb_kat(oracle, kat):
    # t/fusion.c:72-86, t/picotls.c:397-413,429-437
    for v in kat["ecb"]:
        key = bytes.fromhex(v["key"])
        if v["src"].startswith("t/picotls.c:374-376,397"):
            key = key[:16]
        assert oracle.aes_encrypt(key, bytes.fromhex(v["pt"])).hex() == v["ct"], v["src"]


def test_ghash_kat(oracle, kat):
    # t/fusion.c:88-234, H and results held in fusion's internal form
    h = h_from_fusion_internal(bytes.fromhex(kat["ghash"]["h_fusion_internal"]))
    for c in kat["ghash"]["cases"]:
        data = bytes.fromhex(c["data"])[:16 * c["nblocks"]]
        assert oracle.ghash(h, data) == bytes.fromhex(c["out_fusion_internal"])[::-1], c["nblocks"]


def test_gcm_zero_counter_kat(oracle, kat):
    # t/fusion.c:236-256,277-288: raw API with counter 0 == IV 0^96, seq 0
    for v in kat["gcm_zero_ctr"]:
        key, aad, pt = (bytes.fromhex(v[k]) for k in ("key", "aad", "pt"))
        sealed = oracle.seal(key, bytes(12), 0, aad, pt)
        assert sealed.hex() == v["sealed"], v["src"]
        assert oracle.open(key, bytes(12), 0, aad, sealed) == pt


def test_gcm_tag_vectors(oracle, kat):
    # t/fusion.c:290-344 (19 tags over zero inputs) and the supp mask (AES-ECB(01*16, sealed[2:18]))
    t = kat["gcm_zero_ctr_tags"]
    hp_key = bytes.fromhex(t["hp_key"])
    for aadlen, ptlen, tag, mask in t["cases"]:
        sealed = oracle.seal(bytes(16), bytes(12), 0, bytes(aadlen), bytes(ptlen))
        assert sealed[ptlen:].hex() == tag, (aadlen, ptlen)
        off = t["hp_sample_off"]
        assert oracle.aes_encrypt(hp_key, sealed[off:off + 16]).hex() == mask
        assert oracle.open(bytes(16), bytes(12), 0, bytes(aadlen), sealed) == bytes(ptlen)


def test_gcm_seq_and_iv96(oracle, kat):
    # t/fusion.c:258-274 and gcm_iv96 :346-380 (ptls_aead_xor_iv, wrong IV rejected)
    for v in kat["gcm_seq"]:
        key, aad, pt, iv = (bytes.fromhex(v[k]) for k in ("key", "aad", "pt", "iv"))
        if "xor_iv" in v:
            iv = bytes(a ^ b for a, b in zip(iv, bytes.fromhex(v["xor_iv"]) + bytes(8)))
        sealed = oracle.seal(key, iv, v["seq"], aad, pt)
        assert sealed.hex() == v["sealed"]
        assert oracle.open(key, iv, v["seq"], aad, sealed) == pt
        if "bad_xor_iv" in v:
            bad = bytes(a ^ b for a, b in zip(iv, bytes.fromhex(v["bad_xor_iv"]) + bytes(8)))
            assert oracle.open(key, bad, v["seq"], aad, sealed) is None


def test_nist_vectors(oracle, kat):
    # deps/cifra/src/testmodes.c:395-433
    for v in kat["nist"]:
        key, iv, aad, pt = (bytes.fromhex(v[k]) for k in ("key", "iv", "aad", "pt"))
        sealed = oracle.seal(key, iv, 0, aad, pt)
        assert sealed.hex() == v["ct"] + v["tag"], v["src"]
        bad = bytearray(sealed)
        bad[-1] ^= 0xFF
        assert oracle.open(key, iv, 0, aad, bytes(bad)) is None


def test_fusion_vectors(oracle, fusion_vectors):
    # 528 vectors produced by lib/fusion.c itself (tests/golden/gen_golden.py)
    for v in fusion_vectors["vectors"]:
        key, iv, seq, aad, pt = materialise(v)
        sealed = oracle.seal(key, iv, seq, aad, pt)
        assert check_sealed(v, sealed), v["seed"]


def test_open_rejects_short_and_tampered(oracle):
    key, iv = bytes(range(16)), bytes(range(12))
    assert oracle.open(key, iv, 0, b"", b"\0" * 15) is None  # inlen < 16 -> SIZE_MAX (lib/fusion.c:1160-1161)
    sealed = oracle.seal(key, iv, 7, b"hdr", b"payload!")
    for i in range(len(sealed)):
        bad = bytearray(sealed)
        bad[i] ^= 1
        assert oracle.open(key, iv, 7, b"hdr", bytes(bad)) is None
    assert oracle.open(key, iv, 8, b"hdr", sealed) is None  # wrong seq
    assert oracle.open(key, iv, 7, b"hdx", sealed) is None  # wrong AAD


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref/libfusion_ref.so not built (needs /root/reference)")
def test_random_differential_vs_fusion(oracle):
    # t/fusion.c:385-466 shape: random (key, iv, seq, aadlen < 256, textlen < 256), both directions
    ref = FusionRef()
    rng = np.random.default_rng(1234)
    for i in range(1500):
        ks = 16 if i % 2 == 0 else 32
        key, iv = rng.bytes(ks), rng.bytes(12)
        seq = int(rng.integers(0, 2**63))
        aad, pt = rng.bytes(int(rng.integers(0, 256))), rng.bytes(int(rng.integers(0, 256)))
        a = oracle.seal(key, iv, seq, aad, pt)
        assert a == ref.seal(key, iv, seq, aad, pt)
        assert ref.open(key, iv, seq, aad, a) == pt
        assert oracle.open(key, iv, seq, aad, a) == pt


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref/libfusion_ref.so not built (needs /root/reference)")
def test_batch_helpers_match_fusion(oracle):
    # the batch layout used by the GPU tests, checked between both checkers
    from picotls_amd.records import RecordBatch

    ref = FusionRef()
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 3000, 64)
    lens[:4] = [0, 1, 16, 4096]
    b = RecordBatch.build(lens, rng.integers(0, 40, 64), seqs=rng.integers(0, 2**40, 64), key_idx=rng.integers(0, 3, 64))
    keys, ivs = np.frombuffer(rng.bytes(3 * 32), np.uint8), np.frombuffer(rng.bytes(3 * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    out_o, out_r = np.zeros(b.sealed_bytes, np.uint8), np.zeros(b.sealed_bytes, np.uint8)
    oracle.seal_batch(keys, ivs, 32, b.seal, pt, aad, out_o)
    ref.run_batch(True, keys, ivs, 32, b.seal, pt, aad, out_r, nthreads=2)
    assert np.array_equal(out_o, out_r)
    back_o, back_r = np.zeros(b.pt_bytes, np.uint8), np.zeros(b.pt_bytes, np.uint8)
    ok_o, ok_r = np.zeros(b.n, np.uint8), np.zeros(b.n, np.uint8)
    oracle.open_batch(keys, ivs, 32, b.open, out_o, aad, back_o, ok_o)
    _, fails = ref.run_batch(False, keys, ivs, 32, b.open, out_r, aad, back_r, ok=ok_r, nthreads=3)
    assert fails == 0 and ok_o.all() and ok_r.all()
    assert np.array_equal(back_o, back_r)
    for i in range(b.n):
        s, ln = int(b.seal["in_off"][i]), int(lens[i])
        assert np.array_equal(back_o[s:s + ln], pt[s:s + ln])


# ------------------------------------------------------------------------------------------------ QUIC-LB (lib/quiclb-impl.h)


def _quiclb_vectors():
    import json

    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "quiclb_vectors.json")) as f:
        return json.load(f)["vectors"]


def test_quiclb_kat(oracle, kat):
    # t/quiclb.c:27-46: the draft vector at len 7, and a round trip for every length 7..19
    v = kat["quiclb"]
    key, pt19 = bytes.fromhex(v["key"]), bytes.fromhex(v["pt19"])
    for ln in range(7, 20):
        ct = oracle.quiclb(key, pt19[:ln], True)
        if ln == 7:
            assert ct.hex() == v["ct7"]
        assert oracle.quiclb(key, ct, False) == pt19[:ln]
    with pytest.raises(ValueError):
        oracle.quiclb(key, bytes(6), True)
    with pytest.raises(ValueError):
        oracle.quiclb(key, bytes(20), True)


def test_quiclb_fusion_vectors(oracle):
    # tests/golden/quiclb_vectors.json: written by ptls_fusion_quiclb (tests/golden/gen_quiclb.py)
    from vectors import splitmix_bytes

    vecs = _quiclb_vectors()
    assert len(vecs) == 78 and {v["len"] for v in vecs} == set(range(7, 20))
    for v in vecs:
        blob = splitmix_bytes(v["seed"], 16 + v["len"])
        key, pt = blob[:16], blob[16:]
        assert oracle.quiclb(key, pt, True).hex() == v["ct"], v["seed"]
        assert oracle.quiclb(key, bytes.fromhex(v["ct"]), False) == pt


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref/libfusion_ref.so not built")
def test_quiclb_oracle_vs_fusion_random(oracle):
    ref = FusionRef()
    rng = np.random.default_rng(31337)
    for _ in range(400):
        key, ln = rng.bytes(16), int(rng.integers(7, 20))
        data = rng.bytes(ln)
        for enc in (True, False):
            assert oracle.quiclb(key, data, enc) == ref.quiclb(key, data, enc), (ln, enc)


# ------------------------------------------------------------------------------------------------ TLS 1.2 framing

HAVE_TLS12_REF = os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                                             "libtls12_ref.so"))


def parse_tls12_records(wire: bytes):
    """(type, explicit nonce, ciphertext||tag) per record: header {type, 3, 3, BE16(n)} || nonce (8) || body."""
    out, off = [], 0
    while off < len(wire):
        t, v0, v1, n = wire[off], wire[off + 1], wire[off + 2], int.from_bytes(wire[off + 3:off + 5], "big")
        assert (v0, v1) == (3, 3)
        out.append((t, int.from_bytes(wire[off + 5:off + 13], "big"), wire[off + 13:off + 5 + n]))
        off += 5 + n
    return out


@pytest.mark.skipif(not HAVE_TLS12_REF, reason="oracle/_ref/libtls12_ref.so not built")
@pytest.mark.parametrize("key_size", [16, 32])
def test_tls12_record_layer_matches_oracle_framing(oracle, key_size):
    # picotls' own TLS 1.2 send path (lib/picotls.c:779-799) decoded with the framing the engine implements:
    # nonce = fixed IV || explicit nonce, AAD = BE64(seq) || type || 3 || 3 || BE16(len) (build_tls12_aad :753-762)
    from oracle import Tls12Ref

    t = Tls12Ref()
    rng = np.random.default_rng(key_size)
    ms, randoms = rng.bytes(48), rng.bytes(64)
    key, fixed = t.server_keys(key_size, ms, randoms)
    data = rng.bytes(40000)  # three records: 16384, 16384, 7232
    rec_iv = 0x0102030405060708
    wire = t.send(key_size, ms, randoms, rec_iv, data)
    recs = parse_tls12_records(wire)
    assert [len(b) - 16 for _, _, b in recs] == [16384, 16384, 40000 - 32768]
    pos = 0
    for i, (typ, nonce, body) in enumerate(recs):
        assert typ == 23 and nonce == rec_iv + i
        ln = len(body) - 16
        aad = (1 + i).to_bytes(8, "big") + bytes([typ, 3, 3]) + ln.to_bytes(2, "big")
        assert oracle.open(key, fixed + bytes(8), nonce, aad, body) == data[pos:pos + ln]
        pos += ln
    assert t.receive(key_size, ms, randoms, wire) == data
    bad = bytearray(wire)
    bad[20] ^= 1
    assert t.receive(key_size, ms, randoms, bytes(bad)) == -20  # PTLS_ALERT_BAD_RECORD_MAC


def parse_tls13_records(wire: bytes):
    """(header, ciphertext||tag) per record: header {23, 3, 3, BE16(n)}."""
    out, off = [], 0
    while off < len(wire):
        n = int.from_bytes(wire[off + 3:off + 5], "big")
        assert wire[off:off + 3] == bytes([23, 3, 3])
        out.append((wire[off:off + 5], wire[off + 5:off + 5 + n]))
        off += 5 + n
    return out


@pytest.mark.skipif(not HAVE_TLS12_REF, reason="oracle/_ref/libtls12_ref.so not built")
@pytest.mark.parametrize("key_size", [16, 32])
def test_tls13_record_layer_matches_oracle_framing(oracle, key_size):
    # picotls' own TLS 1.3 send path (aead_encrypt lib/picotls.c:728-738) decoded with the framing the engine
    # implements: AAD = the 5-byte header, plaintext = payload || inner type (23), nonce = iv ^ seq
    from oracle import Tls12Ref

    t = Tls12Ref()
    rng = np.random.default_rng(300 + key_size)
    secret = rng.bytes(32 if key_size == 16 else 48)
    key, iv = t.tls13_keys(key_size, secret)
    data = rng.bytes(40000)
    seq0 = 12345
    wire = t.tls13_send(key_size, secret, seq0, data)
    recs = parse_tls13_records(wire)
    assert [len(b) - 17 for _, b in recs] == [16384, 16384, 40000 - 32768]
    pos = 0
    for i, (hdr, body) in enumerate(recs):
        inner = oracle.open(key, iv, seq0 + i, hdr, body)
        ln = len(body) - 17
        assert inner == data[pos:pos + ln] + bytes([23])
        pos += ln
    assert t.tls13_receive(key_size, secret, seq0, wire) == data


@pytest.mark.skipif(not HAVE_TLS12_REF, reason="oracle/_ref/libtls12_ref.so not built")
@pytest.mark.parametrize("key_size", [16, 32])
def test_tls13_key_update_at_2_24_records(oracle, key_size):
    # from enc.seq >= 2^24 ptls_send emits a KeyUpdate (handshake 24, request_update 0) under the old key at that seq,
    # then seals the data under the next traffic secret from seq 0 (lib/picotls.c:6220-6232, :6193-6211)
    from oracle import Tls12Ref

    t = Tls12Ref()
    rng = np.random.default_rng(310 + key_size)
    secret = rng.bytes(32 if key_size == 16 else 48)
    key, iv = t.tls13_keys(key_size, secret)
    data = rng.bytes(20000)
    seq0 = 2**24 + 7
    wire, key2, iv2, seq_after = t.tls13_send_rekeyed(key_size, secret, seq0, data)
    assert (key2, iv2) != (key, iv) and seq_after == 2
    recs = parse_tls13_records(wire)
    assert len(recs) == 3
    assert oracle.open(key, iv, seq0, *recs[0]) == bytes([24, 0, 0, 1, 0, 22])
    assert oracle.open(key2, iv2, 0, *recs[1]) + oracle.open(key2, iv2, 1, *recs[2]) == data[:16384] + b"\x17" + data[16384:] + b"\x17"
    assert t.tls13_receive(key_size, secret, seq0, wire) == data
    # below 2^24 nothing changes
    w, k, v, s = t.tls13_send_rekeyed(key_size, secret, 2**24 - 1, data)
    assert (k, v, s) == (key, iv, 2**24 + 1) and len(parse_tls13_records(w)) == 2
