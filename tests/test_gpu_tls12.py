"""Record framing on the GPU against picotls' own record layer (oracle/_ref/libtls12_ref.so: ptls_import + ptls_send /
ptls_receive over fusion's non-temporal AEADs). TLS 1.2 (ptls_mi355x_seal_tls12_records / _open_tls12_records,
lib/picotls.c:779-799, :6019-6060), and, for arbitrary descriptors, lib/fusion.c's ptls_aead_encrypt with the
record-layer nonce and AAD; TLS 1.3 (ptls_mi355x_seal_tls_records / _open_tls_records, :728-738, :5952-5974) against
ptls_send after ptls_import of a traffic secret. Bit-exact.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef  # noqa: E402

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(os.path.dirname(HERE), "oracle", "_ref")

from gpu_util import dev, empty  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def engine():
    assert torch.cuda.is_available(), "no GPU visible"
    pa.load_library()
    assert pa.is_supported(), "engine reports no gfx950 device"


@pytest.fixture(scope="module")
def tls12ref():
    if not os.path.exists(os.path.join(REF_DIR, "libtls12_ref.so")):
        pytest.skip("oracle/_ref/libtls12_ref.so not shipped")
    from oracle import Tls12Ref

    return Tls12Ref()


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(os.path.join(REF_DIR, "libfusion_ref.so")):
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    return FusionRef()


def _seal(ks, recs, arena, out_bytes, fill=0xEE):
    d_recs, d_in, d_out = dev(recs), dev(arena), empty(out_bytes, fill)
    pa.seal_tls12_records(ks, d_recs.data_ptr(), len(recs), d_in.data_ptr(), d_out.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_out.cpu().numpy()


def _open(ks, recs, wire, out_bytes):
    n = len(recs)
    d_recs, d_in, d_out = dev(recs), dev(np.frombuffer(bytes(wire), np.uint8)), empty(out_bytes + 1)
    d_ok, d_res = empty(n, 0x77), empty(8 * n, 0x77)
    pa.open_tls12_records(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_out.data_ptr(), d_ok.data_ptr(), d_res.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_out.cpu().numpy(), d_ok.cpu().numpy(), d_res.cpu().numpy().view(pa.TLS_RESULT_DTYPE)


@pytest.mark.parametrize("key_size", [16, 32])
def test_tls12_seal_equals_picotls_send_and_open_its_records(tls12ref, key_size):
    # one connection: picotls' ptls_send cuts 60000 bytes into records of 16384 (sequence numbers from 1, explicit
    # nonces from the imported record IV); the batch seals the same records and must give the same wire bytes
    rng = np.random.default_rng(100 + key_size)
    ms, randoms = rng.bytes(48), rng.bytes(64)
    key, fixed = tls12ref.server_keys(key_size, ms, randoms)
    data = rng.bytes(60000)
    rec_iv = int(rng.integers(0, 2**62))
    wire = tls12ref.send(key_size, ms, randoms, rec_iv, data)
    chunks = [data[o:o + 16384] for o in range(0, len(data), 16384)]
    n = len(chunks)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    arena, pin, pout = bytearray(), 0, 0
    for i, c in enumerate(chunks):
        arena += (rec_iv + i).to_bytes(8, "big") + c
        recs[i]["in_off"], recs[i]["out_off"], recs[i]["len"] = pin, pout, len(c)
        recs[i]["seq"], recs[i]["flags"] = 1 + i, 23
        pin += 8 + len(c)
        pout += 13 + len(c) + 16
    ks = pa.Keyset(key, fixed + bytes(8), key_size)
    out = _seal(ks, recs, np.frombuffer(bytes(arena), np.uint8), pout)
    assert out.tobytes() == wire
    # and the engine opens picotls' records
    precs = recs.copy()
    precs["in_off"], precs["out_off"] = recs["out_off"], np.cumsum([0] + [len(c) for c in chunks[:-1]])
    plain, ok, res = _open(ks, precs, wire, len(data))
    assert ok.all() and (res["status"] == pa.TLS_OK).all() and (res["content_type"] == 23).all()
    assert list(res["plain_len"]) == [len(c) for c in chunks]
    assert plain[:len(data)].tobytes() == data
    # picotls' client side accepts the engine's records (identical bytes, but through ptls_receive)
    assert tls12ref.receive(key_size, ms, randoms, out.tobytes()) == data
    ks.free()


@pytest.mark.parametrize("key_size,nkeys", [(16, 1), (32, 5)])
def test_tls12_random_records_vs_fusion(ref, key_size, nkeys):
    # arbitrary lengths 0..16384, types, sequence numbers and explicit nonces; expected = header || nonce ||
    # ptls_aead_encrypt(fixed IV || 0^64 static IV, seq = nonce, AAD = BE64(seq) || type || 3 || 3 || BE16(len))
    rng = np.random.default_rng(7 * nkeys + key_size)
    n = 300
    lens = rng.integers(0, 16385, n)
    lens[:5] = [0, 1, 15, 16, 16384]
    types = rng.choice([21, 22, 23], n)
    key_idx = np.sort(rng.integers(0, nkeys, n))
    seqs = rng.integers(0, 2**63, n, dtype=np.uint64)
    nonces = rng.integers(0, 2**63, n, dtype=np.uint64)
    keys = rng.bytes(nkeys * key_size)
    fixed = rng.bytes(nkeys * 4)
    ivs = b"".join(fixed[4 * k:4 * k + 4] + bytes(8) for k in range(nkeys))
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    arena, pin, pout = bytearray(), 0, 0
    payloads = []
    for i in range(n):
        p = rng.bytes(int(lens[i]))
        payloads.append(p)
        gap = int(rng.integers(0, 5))
        arena += bytes(gap) + int(nonces[i]).to_bytes(8, "big") + p
        recs[i]["in_off"], recs[i]["out_off"], recs[i]["len"] = pin + gap, pout, lens[i]
        recs[i]["seq"], recs[i]["flags"], recs[i]["key_idx"] = seqs[i], types[i], key_idx[i]
        pin += gap + 8 + int(lens[i])
        pout += 13 + int(lens[i]) + 16 + int(rng.integers(0, 5))
    ks = pa.Keyset(keys, ivs, key_size)
    out = _seal(ks, recs, np.frombuffer(bytes(arena), np.uint8), pout + 1)
    m = np.zeros(out.size, bool)
    for i in range(n):
        k, ln = int(key_idx[i]), int(lens[i])
        t = int(types[i])
        aad = int(seqs[i]).to_bytes(8, "big") + bytes([t, 3, 3]) + ln.to_bytes(2, "big")
        expect = (bytes([t, 3, 3]) + (ln + 24).to_bytes(2, "big") + int(nonces[i]).to_bytes(8, "big") +
                  ref.seal(keys[k * key_size:(k + 1) * key_size], ivs[12 * k:12 * k + 12], int(nonces[i]), aad, payloads[i]))
        o = int(recs[i]["out_off"])
        assert out[o:o + ln + 29].tobytes() == expect, i
        m[o:o + ln + 29] = True
    assert (out[~m] == 0xEE).all()  # nothing outside the wire records is written
    # open them back (in place of a receiver), then tamper: tag, ciphertext, explicit nonce, header type / length
    wire = out.tobytes()
    precs = recs.copy()
    precs["in_off"] = recs["out_off"]
    precs["out_off"] = np.concatenate([[0], np.cumsum(lens[:-1] + 3)])
    plain, ok, res = _open(ks, precs, wire, int(precs["out_off"][-1]) + int(lens[-1]))
    assert ok.all() and (res["status"] == pa.TLS_OK).all()
    assert list(res["content_type"]) == list(types)
    for i in range(n):
        o = int(precs["out_off"][i])
        assert plain[o:o + int(lens[i])].tobytes() == payloads[i], i
    bad = bytearray(wire)
    idx = {}
    for kind, i in zip(("tag", "ct", "nonce", "type", "len", "ver"), (5, 6, 7, 8, 9, 10)):
        o = int(recs[i]["out_off"])
        if kind == "tag":
            bad[o + 13 + int(lens[i]) + 15] ^= 1
        elif kind == "ct":
            bad[o + 13] ^= 0x40
        elif kind == "nonce":
            bad[o + 5 + 7] ^= 1
        elif kind == "type":
            bad[o] ^= 3
        elif kind == "len":
            bad[o + 4] ^= 1
        else:
            bad[o + 2] = 1  # version 3.1: not authenticated (the AAD carries 3.3), rejected by the header check
        idx[kind] = i
    plain, ok, res = _open(ks, precs, bytes(bad), int(precs["out_off"][-1]) + int(lens[-1]))
    for kind, i in idx.items():
        # the type is in the AAD as received; the AAD length and version come from the descriptor / constants, so a
        # wrong length or version field is caught by the header check
        want = pa.TLS_BAD_HEADER if kind in ("ver", "len") else pa.TLS_BAD_MAC
        assert ok[i] == 0 and res[i]["status"] == want, kind
    assert ok.sum() == n - len(idx)
    ks.free()


def test_tls12_empty_batch():
    ks = pa.Keyset(bytes(16), bytes(12), 16)
    pa.seal_tls12_records(ks, 0, 0, 0, 0)
    pa.open_tls12_records(ks, 0, 0, 0, 0, 0)
    ks.free()


@pytest.mark.parametrize("key_size", [16, 32])
def test_tls13_seal_equals_picotls_send_and_open_its_records(tls12ref, key_size):
    # TLS 1.3: picotls' own ptls_send (aead_encrypt, lib/picotls.c:728-738) after ptls_import of a traffic secret; the
    # batch (ptls_mi355x_seal_tls_records) with the key / IV of ptls_get_traffic_keys must give the same wire bytes,
    # open_tls_records must recover the data from picotls' records, and ptls_receive must accept the engine's
    rng = np.random.default_rng(500 + key_size)
    secret = rng.bytes(32 if key_size == 16 else 48)
    key, iv = tls12ref.tls13_keys(key_size, secret)
    data = rng.bytes(70000)
    # below 2^24: from there ptls_send first emits a KeyUpdate and rekeys (lib/picotls.c:6220-6232)
    seq0 = int(rng.integers(0, 2**24 - 16))
    wire = tls12ref.tls13_send(key_size, secret, seq0, data)
    chunks = [data[o:o + 16384] for o in range(0, len(data), 16384)]
    n = len(chunks)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    pin = pout = 0
    for i, c in enumerate(chunks):
        recs[i]["in_off"], recs[i]["out_off"], recs[i]["len"] = pin, pout, len(c)
        recs[i]["seq"], recs[i]["flags"] = seq0 + i, 23
        pin += len(c)
        pout += 5 + len(c) + 1 + 16
    ks = pa.Keyset(key, iv, key_size)
    d_recs, d_in, d_out = dev(recs), dev(np.frombuffer(data, np.uint8)), empty(pout, 0xEE)
    pa.seal_tls_records(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy().tobytes()
    assert out == wire
    orecs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    orecs["in_off"] = recs["out_off"]
    orecs["out_off"] = np.cumsum([0] + [len(c) + 1 for c in chunks[:-1]])
    orecs["len"] = [len(c) + 1 for c in chunks]
    orecs["seq"] = recs["seq"]
    d_recs2, d_wire, d_plain = dev(orecs), dev(np.frombuffer(wire, np.uint8)), empty(len(data) + n + 1)
    d_ok, d_res = empty(n, 0x77), empty(8 * n, 0x77)
    pa.open_tls_records(ks, d_recs2.data_ptr(), n, d_wire.data_ptr(), d_plain.data_ptr(), d_ok.data_ptr(), d_res.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ok, res, plain = d_ok.cpu().numpy(), d_res.cpu().numpy().view(pa.TLS_RESULT_DTYPE), d_plain.cpu().numpy()
    assert ok.all() and (res["status"] == pa.TLS_OK).all() and (res["content_type"] == 23).all()
    assert b"".join(plain[int(o):int(o) + int(r["plain_len"])].tobytes() for o, r in zip(orecs["out_off"], res)) == data
    assert tls12ref.tls13_receive(key_size, secret, seq0, out) == data
    ks.free()


@pytest.mark.gpu
@pytest.mark.parametrize("key_size", [16, 32])
def test_tls13_key_update_via_keyset_update(tls12ref, key_size):
    # picotls rekeys its send side once enc.seq reaches 2^24 (lib/picotls.c:6220-6232): the KeyUpdate record goes out
    # under the old key, the data under the next traffic secret from seq 0. The engine does the same with one keyset:
    # seal the KeyUpdate, ptls_mi355x_keyset_update to the new key / IV, seal the data; the wire bytes must match
    rng = np.random.default_rng(520 + key_size)
    secret = rng.bytes(32 if key_size == 16 else 48)
    key, iv = tls12ref.tls13_keys(key_size, secret)
    data = rng.bytes(50000)
    seq0 = 2**24 + int(rng.integers(0, 1000))
    wire, key2, iv2, seq_after = tls12ref.tls13_send_rekeyed(key_size, secret, seq0, data)
    stream = torch.cuda.current_stream().cuda_stream
    ks = pa.Keyset(key, iv, key_size)
    # the KeyUpdate handshake message (type 24, length 1, request_update 0), content type 22
    ku = np.zeros(1, dtype=pa.RECORD_DTYPE)
    ku[0]["len"], ku[0]["seq"], ku[0]["flags"] = 5, seq0, 22
    d_ku, d_kin, d_kout = dev(ku), dev(np.frombuffer(bytes([24, 0, 0, 1, 0]), np.uint8)), empty(27, 0xEE)
    pa.seal_tls_records(ks, d_ku.data_ptr(), 1, d_kin.data_ptr(), d_kout.data_ptr(), stream)
    torch.cuda.synchronize()
    ks.update([0], key2, iv2)
    chunks = [data[o:o + 16384] for o in range(0, len(data), 16384)]
    n = len(chunks)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    recs["in_off"] = np.arange(n) * 16384
    recs["out_off"] = np.arange(n) * (16384 + 22)
    recs["len"] = [len(c) for c in chunks]
    recs["seq"], recs["flags"] = np.arange(n), 23
    d_recs, d_in, d_out = dev(recs), dev(np.frombuffer(data, np.uint8)), empty(len(data) + 22 * n, 0xEE)
    pa.seal_tls_records(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_out.data_ptr(), stream)
    torch.cuda.synchronize()
    assert seq_after == n
    assert d_kout.cpu().numpy().tobytes() + d_out.cpu().numpy().tobytes() == wire
    ks.free()


@pytest.mark.gpu
def test_keyset_update_rekeys_only_the_named_entries(ref):
    # rekey entries 2 and 5 of a 7-key keyset (key schedule + H powers rebuilt on the GPU); every record of a batch
    # over all keys must then equal fusion under the current key of its entry
    rng = np.random.default_rng(530)
    nkeys, n = 7, 70
    keys = [rng.bytes(16) for _ in range(nkeys)]
    ivs = [rng.bytes(12) for _ in range(nkeys)]
    ks = pa.Keyset(b"".join(keys), b"".join(ivs), 16)
    new = {2: (rng.bytes(16), rng.bytes(12)), 5: (rng.bytes(16), rng.bytes(12))}
    ks.update([5, 2], new[5][0] + new[2][0], new[5][1] + new[2][1])
    for i, (k, v) in new.items():
        keys[i], ivs[i] = k, v
    lens = rng.integers(0, 3000, n)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    recs["in_off"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    recs["out_off"] = recs["in_off"] + 16 * np.arange(n)
    recs["len"], recs["seq"] = lens, rng.integers(0, 2**48, n)
    recs["key_idx"] = np.sort(rng.integers(0, nkeys, n))
    recs["aad_off"], recs["aad_len"] = 0, 13
    pt = rng.bytes(int(lens.sum()))
    aad = rng.bytes(13)
    d_recs, d_in, d_aad, d_out = dev(recs), dev(np.frombuffer(pt, np.uint8)), dev(np.frombuffer(aad, np.uint8)), \
        empty(int(lens.sum()) + 16 * n, 0xEE)
    pa.seal_batch(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy().tobytes()
    for r in recs:
        o, ln, k = int(r["out_off"]), int(r["len"]), int(r["key_idx"])
        want = ref.seal(keys[k], ivs[k], int(r["seq"]), aad, pt[int(r["in_off"]):int(r["in_off"]) + ln])
        assert out[o:o + ln + 16] == want, (k, ln)
    # an index outside the keyset is refused and leaves the keyset usable
    with pytest.raises(pa.EngineError):
        ks.update([7], rng.bytes(16), rng.bytes(12))
    with pytest.raises(pa.EngineError):
        ks.update([3, 3], rng.bytes(32), rng.bytes(24))
    with pytest.raises(ValueError):
        ks.update([1], rng.bytes(32), rng.bytes(12))
    ks.free()


@pytest.mark.gpu
def test_tls13_many_key_large_framed_batch_balanced():
    # a framed many-key batch large enough for the work-balanced workgroup ranges (the weights then take the 5-byte
    # record header as AAD, not the flags field): 140,000 TLS 1.3 records of 0-200 B over 70 connections; sampled
    # records equal header || fusion's seal of payload || type under the header as AAD, and every record opens back
    from oracle import FusionRef

    ref_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref")
    if not os.path.exists(os.path.join(ref_dir, "libfusion_ref.so")):
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    ref = FusionRef()
    rng = np.random.default_rng(909)
    n, nkeys = 140000, 70
    lens = rng.integers(0, 201, n)
    keys, ivs = rng.bytes(16 * nkeys), rng.bytes(12 * nkeys)
    data = np.frombuffer(rng.bytes(int(lens.sum())), np.uint8)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    recs["len"] = lens
    recs["in_off"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    recs["out_off"] = np.concatenate([[0], np.cumsum(lens + 5 + 1 + 16)[:-1]])
    recs["key_idx"] = np.arange(n) * nkeys // n
    recs["seq"] = rng.integers(0, 2**40, n)
    recs["flags"] = 23
    wire_len = int((lens + 5 + 1 + 16).sum())
    ks = pa.Keyset(keys, ivs, 16)
    s = torch.cuda.current_stream().cuda_stream
    d_recs, d_in, d_out = dev(recs), dev(data), empty(wire_len, 0xEE)
    pa.seal_tls_records(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_out.data_ptr(), s)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i in list(rng.choice(n, 300, replace=False)) + [0, n - 1]:
        k = int(recs["key_idx"][i])
        o, ln, p = int(recs["out_off"][i]), int(lens[i]), int(recs["in_off"][i])
        hdr = bytes([23, 3, 3, (ln + 17) >> 8, (ln + 17) & 0xFF])
        want = hdr + ref.seal(keys[16 * k:16 * k + 16], ivs[12 * k:12 * k + 12], int(recs["seq"][i]), hdr,
                              data[p:p + ln].tobytes() + b"\x17")
        assert out[o:o + len(want)].tobytes() == want, i
    orecs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    orecs["in_off"], orecs["len"], orecs["seq"], orecs["key_idx"] = recs["out_off"], lens + 1, recs["seq"], recs["key_idx"]
    orecs["out_off"] = np.concatenate([[0], np.cumsum(lens + 1)[:-1]])
    d_recs2, d_plain = dev(orecs), empty(int((lens + 1).sum()) + 1)
    d_ok, d_res = empty(n, 0x77), empty(8 * n, 0x77)
    pa.open_tls_records(ks, d_recs2.data_ptr(), n, d_out.data_ptr(), d_plain.data_ptr(), d_ok.data_ptr(), d_res.data_ptr(), s)
    torch.cuda.synchronize()
    ok, res, plain = d_ok.cpu().numpy(), d_res.cpu().numpy().view(pa.TLS_RESULT_DTYPE), d_plain.cpu().numpy()
    assert ok.all() and (res["status"] == pa.TLS_OK).all() and (res["content_type"] == 23).all()
    assert np.array_equal(res["plain_len"].astype(np.int64), lens)
    got = np.concatenate([plain[int(o):int(o) + int(ln)] for o, ln in zip(orecs["out_off"], lens)])
    assert np.array_equal(got, data)
    ks.free()


def _tls12_batch(rng, lens, nkeys, key_size):
    """TLS 1.2 records back to back: explicit nonce || payload in, header || nonce || ciphertext || tag out."""
    n = len(lens)
    keys = rng.bytes(nkeys * key_size)
    fixed = rng.bytes(nkeys * 4)
    ivs = b"".join(fixed[4 * k:4 * k + 4] + bytes(8) for k in range(nkeys))
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    recs["len"] = lens
    recs["in_off"] = np.concatenate([[0], np.cumsum(lens + 8)[:-1]])
    recs["out_off"] = np.concatenate([[0], np.cumsum(lens + 29)[:-1]])
    recs["seq"] = rng.integers(0, 2**62, n, dtype=np.uint64)
    recs["flags"] = 23
    recs["key_idx"] = np.arange(n) * nkeys // n
    arena = np.frombuffer(rng.bytes(int((lens + 8).sum())), np.uint8).copy()
    return keys, ivs, recs, arena


def _tls12_expect(ref, keys, ivs, key_size, recs, arena, i):
    k, ln, p = int(recs["key_idx"][i]), int(recs["len"][i]), int(recs["in_off"][i])
    nonce = arena[p:p + 8].tobytes()
    aad = int(recs["seq"][i]).to_bytes(8, "big") + bytes([23, 3, 3]) + ln.to_bytes(2, "big")
    return (bytes([23, 3, 3]) + (ln + 24).to_bytes(2, "big") + nonce +
            ref.seal(keys[k * key_size:(k + 1) * key_size], ivs[12 * k:12 * k + 12], int.from_bytes(nonce, "big"), aad,
                     arena[p + 8:p + 8 + ln].tobytes()))


@pytest.mark.parametrize("key_size,nkeys,n,uniform", [(16, 3, 2600, 0), (32, 1, 2100, 0), (16, 1, 256 * 130, 16384),
                                                       (32, 2, 256 * 130, 1200), (16, 1, 256 * 130, 3001)])
def test_tls12_w8_kernels_vs_fusion(ref, key_size, nkeys, n, uniform):
    """TLS 1.2 framing in the W8 kernels (batches of at least W8_MIN_RECS records: 256 since round 5): random lengths (EXT 4's cut
    runs), 33,280 records of 16 KiB, 130 per workgroup (EXT 3's whole runs of long records), and 33,280 records of 1200
    or 3001 bytes (EXT 4's whole runs, in 4-lane groups since round 5). Every record (the uniform batches: 400 sampled
    and the ends) equals lib/fusion.c's seal with the record-layer nonce and AAD, nothing outside the wire records is
    written, and every record opens back to its payload."""
    long_runs = uniform != 0
    rng = np.random.default_rng(1200 + n + key_size + uniform)
    lens = np.full(n, uniform) if long_runs else rng.integers(0, 16385, n)
    keys, ivs, recs, arena = _tls12_batch(rng, lens, nkeys, key_size)
    ks = pa.Keyset(keys, ivs, key_size)
    wire_len = int((lens + 29).sum())
    out = _seal(ks, recs, arena, wire_len + 3)
    check = list(rng.choice(n, 400, replace=False)) + [0, n - 1] if long_runs else range(n)
    for i in check:
        o = int(recs["out_off"][i])
        want = _tls12_expect(ref, keys, ivs, key_size, recs, arena, i)
        assert out[o:o + len(want)].tobytes() == want, i
    assert (out[wire_len:] == 0xEE).all()
    precs = recs.copy()
    precs["in_off"] = recs["out_off"]
    precs["out_off"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    plain, ok, res = _open(ks, precs, out[:wire_len].tobytes(), int(lens.sum()))
    assert ok.all() and (res["status"] == pa.TLS_OK).all()
    src = arena.reshape(n, 8 + uniform)[:, 8:].reshape(-1) if long_runs else np.concatenate(
        [arena[int(recs["in_off"][i]) + 8:int(recs["in_off"][i]) + 8 + int(lens[i])] for i in range(n)])
    assert np.array_equal(plain[:int(lens.sum())], src)
    ks.free()


@pytest.mark.parametrize("ln", [16384, 1200, 37])
def test_tls13_w8_whole_runs_vs_fusion(ref, ln):
    """TLS 1.3 framing in the W8 kernels' whole runs: 33,280 records (130 per workgroup) of two connections, of 16 KiB
    (EXT 3: long records) or 1200 / 37 bytes (EXT 4, in 4-lane groups since round 5); sampled records equal header ||
    fusion's seal of payload || type under the header as AAD, and every record opens back."""
    rng = np.random.default_rng(1313 + ln)
    n, nkeys = 256 * 130, 2
    keys, ivs = rng.bytes(16 * nkeys), rng.bytes(12 * nkeys)
    data = np.frombuffer(rng.bytes(n * ln), np.uint8)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    recs["len"] = ln
    recs["in_off"] = np.arange(n, dtype=np.uint64) * ln
    recs["out_off"] = np.arange(n, dtype=np.uint64) * (ln + 22)
    recs["key_idx"] = np.arange(n) * nkeys // n
    recs["seq"] = rng.integers(0, 2**40, n)
    recs["flags"] = 23
    ks = pa.Keyset(keys, ivs, 16)
    s = torch.cuda.current_stream().cuda_stream
    d_recs, d_in, d_out = dev(recs), dev(data), empty(n * (ln + 22), 0xEE)
    pa.seal_tls_records(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_out.data_ptr(), s)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    hdr = bytes([23, 3, 3, (ln + 17) >> 8, (ln + 17) & 0xFF])
    for i in list(rng.choice(n, 400, replace=False)) + [0, n - 1]:
        k, o, p = int(recs["key_idx"][i]), int(recs["out_off"][i]), int(recs["in_off"][i])
        want = hdr + ref.seal(keys[16 * k:16 * k + 16], ivs[12 * k:12 * k + 12], int(recs["seq"][i]), hdr,
                              data[p:p + ln].tobytes() + b"\x17")
        assert out[o:o + len(want)].tobytes() == want, i
    orecs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    orecs["in_off"], orecs["len"], orecs["seq"], orecs["key_idx"] = recs["out_off"], ln + 1, recs["seq"], recs["key_idx"]
    orecs["out_off"] = np.arange(n, dtype=np.uint64) * (ln + 1)
    d_recs2, d_plain = dev(orecs), empty(n * (ln + 1) + 1)
    d_ok, d_res = empty(n, 0x77), empty(8 * n, 0x77)
    pa.open_tls_records(ks, d_recs2.data_ptr(), n, d_out.data_ptr(), d_plain.data_ptr(), d_ok.data_ptr(), d_res.data_ptr(), s)
    torch.cuda.synchronize()
    assert d_ok.cpu().numpy().all()
    res = d_res.cpu().numpy().view(pa.TLS_RESULT_DTYPE)
    assert (res["status"] == pa.TLS_OK).all() and (res["plain_len"] == ln).all()
    plain = d_plain.cpu().numpy()[:n * (ln + 1)].reshape(n, ln + 1)
    assert np.array_equal(plain[:, :ln].reshape(-1), data)
    ks.free()


def test_tls13_w8_cut_runs_random_lengths_vs_fusion(ref):
    """TLS 1.3 framing in the EXT 4 kernel's cut runs: 2,500 records of 0-16,383 payload bytes over three connections,
    AES-256; every record equals header || fusion's seal of payload || type under the header as AAD, and every record
    opens back with its content type."""
    rng = np.random.default_rng(1314)
    n, nkeys = 2500, 3
    lens = rng.integers(0, 16384, n)
    keys, ivs = rng.bytes(32 * nkeys), rng.bytes(12 * nkeys)
    data = np.frombuffer(rng.bytes(int(lens.sum())), np.uint8)
    recs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    recs["len"] = lens
    recs["in_off"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    recs["out_off"] = np.concatenate([[0], np.cumsum(lens + 22)[:-1]])
    recs["key_idx"] = np.arange(n) * nkeys // n
    recs["seq"] = rng.integers(0, 2**40, n)
    recs["flags"] = rng.choice([21, 22, 23], n)
    wire_len = int((lens + 22).sum())
    ks = pa.Keyset(keys, ivs, 32)
    s = torch.cuda.current_stream().cuda_stream
    d_recs, d_in, d_out = dev(recs), dev(data), empty(wire_len + 3, 0xEE)
    pa.seal_tls_records(ks, d_recs.data_ptr(), n, d_in.data_ptr(), d_out.data_ptr(), s)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i in range(n):
        k, o, ln, p = int(recs["key_idx"][i]), int(recs["out_off"][i]), int(lens[i]), int(recs["in_off"][i])
        hdr = bytes([23, 3, 3, (ln + 17) >> 8, (ln + 17) & 0xFF])
        want = hdr + ref.seal(keys[32 * k:32 * k + 32], ivs[12 * k:12 * k + 12], int(recs["seq"][i]), hdr,
                              data[p:p + ln].tobytes() + bytes([int(recs["flags"][i])]))
        assert out[o:o + len(want)].tobytes() == want, i
    assert (out[wire_len:] == 0xEE).all()
    orecs = np.zeros(n, dtype=pa.RECORD_DTYPE)
    orecs["in_off"], orecs["len"], orecs["seq"], orecs["key_idx"] = recs["out_off"], lens + 1, recs["seq"], recs["key_idx"]
    orecs["out_off"] = np.concatenate([[0], np.cumsum(lens + 1)[:-1]])
    d_recs2, d_plain = dev(orecs), empty(int((lens + 1).sum()) + 1)
    d_ok, d_res = empty(n, 0x77), empty(8 * n, 0x77)
    pa.open_tls_records(ks, d_recs2.data_ptr(), n, d_out.data_ptr(), d_plain.data_ptr(), d_ok.data_ptr(), d_res.data_ptr(), s)
    torch.cuda.synchronize()
    assert d_ok.cpu().numpy().all()
    res = d_res.cpu().numpy().view(pa.TLS_RESULT_DTYPE)
    assert (res["status"] == pa.TLS_OK).all() and (res["plain_len"] == lens).all()
    assert (res["content_type"] == recs["flags"]).all()
    plain = d_plain.cpu().numpy()
    for i in range(0, n, 7):
        o, ln, p = int(orecs["out_off"][i]), int(lens[i]), int(recs["in_off"][i])
        assert np.array_equal(plain[o:o + ln], data[p:p + ln]), i
    ks.free()
