"""Context lifecycle, concurrency and the per-record path's edges, through the engine's C ABI, bit-exact vs lib/fusion.c.

  * contexts are independent (SURVEY 8(b) Threading, lib/picotls.c:6553-6568): threads with their own contexts seal and
    open concurrently while others are created and freed;
  * teardown is stream-ordered: freeing a keyset right after launching a batch on it leaves that batch intact, and the
    slab entry it frees is only reused once cleared;
  * records and AADs beyond the descriptor's 16-bit AAD field (flags carries bits 16..31) and the per-record path's
    gather (encrypt_v) and fused header protection (encrypt_s);
  * the batch calls on pinned host arenas for a many-key keyset in random key order and for TLS 1.3 records.
"""
import os
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef  # noqa: E402
from picotls_amd.records import RecordBatch  # noqa: E402

pytestmark = pytest.mark.gpu

HAVE_REF = os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                                       "libfusion_ref.so"))


@pytest.fixture(scope="module", autouse=True)
def engine():
    assert torch.cuda.is_available(), "no GPU visible"
    pa.load_library()
    assert pa.is_supported(), "engine reports no gfx950 device"


@pytest.fixture(scope="module")
def ref():
    if not HAVE_REF:
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    return FusionRef()


def pinned(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).pin_memory()


def test_threads_with_own_contexts_and_churn(ref):
    # 8 threads (ctypes drops the GIL inside each engine call): each owns a send and a receive context and, every few
    # records, creates, uses and frees a short-lived one; everything equals fusion
    errors = []

    def worker(t):
        rng = np.random.default_rng(1000 + t)
        ks_size = 16 if t % 2 == 0 else 32
        alg = pa.aes128gcm if ks_size == 16 else pa.aes256gcm
        key, iv = rng.bytes(ks_size), rng.bytes(12)
        enc, dec = pa.aead_new_direct(alg, True, key, iv), pa.aead_new_direct(alg, False, key, iv)
        try:
            for i in range(40):
                ln, al = int(rng.integers(0, 3000)), int(rng.integers(0, 40))
                pt, aad, seq = rng.bytes(ln), rng.bytes(al), int(rng.integers(0, 2**62))
                want = ref.seal(key, iv, seq, aad, pt)
                if enc.encrypt(pt, seq, aad) != want or dec.decrypt(want, seq, aad) != pt:
                    errors.append((t, i))
                if i % 5 == 0:
                    k2, v2 = rng.bytes(ks_size), rng.bytes(12)
                    tmp = pa.aead_new_direct(alg, True, k2, v2)
                    if tmp.encrypt(pt, seq, aad) != ref.seal(k2, v2, seq, aad, pt):
                        errors.append((t, i, "tmp"))
                    tmp.free()
        finally:
            enc.free()
            dec.free()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert errors == []


def test_combined_per_record_calls_across_threads(ref):
    # per-record calls of many threads arriving together (each on its own launch by default; combined into shared
    # launches under PTLS_MI355X_COMBINE, which the C vtable suite runs): 16 threads, AES-128 and AES-256 contexts,
    # seal, open (a quarter tampered), seal with the header-protection mask (encrypt_s) and records above the combining
    # cap (64 KiB), released in bursts by a barrier; every output, ok result and mask equals fusion's
    nthreads, nops = 16, 48
    barrier = threading.Barrier(nthreads)
    errors = []
    plans = []
    for t in range(nthreads):
        rng = np.random.default_rng(5000 + t)
        ks_size = 16 if t % 2 == 0 else 32
        key, iv, hpkey = rng.bytes(ks_size), rng.bytes(12), rng.bytes(ks_size)
        ops = []
        for i in range(nops):
            ln = int(rng.choice([0, 1, 15, 16, 17, 100, 1200, 1500, 4096, 16384])) if i != 7 else 70000
            aad, seq, pt = rng.bytes(int(rng.integers(0, 40))), int(rng.integers(0, 2**62)), None
            pt = rng.bytes(ln)
            kind = ["enc", "dec", "dec_bad", "enc_s"][i % 4]
            if kind == "enc_s":
                so = int(rng.integers(0, ln + 1))
                want, mask = ref.seal_with_hp(key, iv, seq, aad, pt, hpkey, so)
                ops.append((kind, pt, seq, aad, (want, mask, so)))
            else:
                want = ref.seal(key, iv, seq, aad, pt)
                if kind == "dec_bad":
                    want = bytearray(want)
                    want[int(rng.integers(0, len(want)))] ^= 0x40
                    want = bytes(want)
                ops.append((kind, pt, seq, aad, want))
        plans.append((ks_size, key, iv, hpkey, ops))

    def worker(t):
        ks_size, key, iv, hpkey, ops = plans[t]
        alg = pa.aes128gcm if ks_size == 16 else pa.aes256gcm
        enc, dec, hp = pa.aead_new_direct(alg, True, key, iv), pa.aead_new_direct(alg, False, key, iv), pa.CtrCipher(hpkey)
        try:
            for i, (kind, pt, seq, aad, want) in enumerate(ops):
                if i % 8 == 0:
                    barrier.wait()
                if kind == "enc":
                    ok = enc.encrypt(pt, seq, aad) == want
                elif kind == "dec":
                    ok = dec.decrypt(want, seq, aad) == pt
                elif kind == "dec_bad":
                    ok = dec.decrypt(want, seq, aad) is None
                else:
                    sealed, mask = enc.encrypt_s(pt, seq, aad, hp, want[2])
                    ok = sealed == want[0] and mask == want[1]
                if not ok:
                    errors.append((t, i, kind, len(pt)))
        except Exception as e:  # noqa: BLE001 -- reported by the assertion below
            errors.append((t, repr(e)))
            barrier.abort()
        finally:
            enc.free()
            dec.free()
            hp.ks.free()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert errors == []


def test_free_right_after_launch_is_ordered(ref):
    # keyset_free does not wait on the host: it orders the clearing of the key material after the keyset's launches on
    # every stream. A batch launched on a side stream and freed at once still seals correctly, and keysets made right
    # after (reusing the device's entry pool) are correct too.
    rng = np.random.default_rng(77)
    n = 20000
    b = RecordBatch.build(np.full(n, 4096), 13, seqs=np.arange(n, dtype=np.uint64))
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    dev = torch.device("cuda:0")
    d_recs, d_pt, d_aad = (torch.from_numpy(x.view(np.uint8).copy()).to(dev) for x in (b.seal, pt, aad))
    side = torch.cuda.Stream(dev)
    outs = []
    for r in range(3):
        key, iv = rng.bytes(16), rng.bytes(12)
        ks = pa.Keyset(key, iv, 16)
        d_out = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device=dev)
        side.wait_stream(torch.cuda.current_stream())  # the inputs and the zeroed output are ready
        pa.seal_batch(ks, d_recs.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), side.cuda_stream)
        ks.free()  # immediately, with the batch most likely still running
        outs.append((key, iv, d_out))
        # a per-record context created now may take a freshly freed entry only after its clearing completed
        ctx = pa.aead_new_direct(pa.aes128gcm, True, rng.bytes(16), rng.bytes(12))
        ctx.encrypt(b"x" * 100, 1, b"")
        ctx.free()
    side.synchronize()
    for key, iv, d_out in outs:
        want = np.zeros(b.sealed_bytes, np.uint8)
        ref.run_batch(True, np.frombuffer(key, np.uint8), np.frombuffer(iv, np.uint8), 16, b.seal, pt, aad, want, nthreads=8)
        assert np.array_equal(d_out.cpu().numpy(), want)


def test_context_churn_reuses_entries_correctly(ref):
    # thousands of one-key contexts created and freed in a row (entries come back to the pool after clearing): every
    # context seals with its own key
    rng = np.random.default_rng(78)
    for i in range(3000):
        key, iv = rng.bytes(16), rng.bytes(12)
        ctx = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
        if i % 100 == 0:
            pt = rng.bytes(int(rng.integers(0, 200)))
            assert ctx.encrypt(pt, i, b"h") == ref.seal(key, iv, i, b"h", pt), i
        ctx.free()


def test_deferred_setup_on_every_kind_of_first_use(ref):
    # a one-key keyset's setup runs on its first use's stream: whatever that first use is (a batch on a side stream, an
    # IV change, a rekey, a per-record call, an ECB mask), the result equals fusion with the key and IV in force
    rng = np.random.default_rng(79)
    key, iv, iv2, key3, iv3 = rng.bytes(16), rng.bytes(12), rng.bytes(12), rng.bytes(16), rng.bytes(12)
    lens = rng.integers(0, 3000, 40)
    b = RecordBatch.build(lens, 13, seqs=np.arange(40, dtype=np.uint64))
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(b.aad_bytes), np.uint8)
    side = torch.cuda.Stream()

    def batch(ks, stream):
        d_recs, d_pt, d_aad = (torch.from_numpy(x.view(np.uint8).copy()).cuda() for x in (b.seal, pt, aad))
        d_out = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        pa.seal_batch(ks, d_recs.data_ptr(), b.n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        return d_out.cpu().numpy()

    def want(k, v):
        out = np.zeros(b.sealed_bytes, np.uint8)
        ref.run_batch(True, np.frombuffer(k, np.uint8), np.frombuffer(v, np.uint8), 16, b.seal, pt, aad, out)
        return out

    ks = pa.Keyset(key, iv, 16)  # first use: a batch on a side stream
    assert np.array_equal(batch(ks, side), want(key, iv))
    ks.free()
    ks = pa.Keyset(key, iv, 16)  # first use: set_iv (on the maintenance stream), then a batch
    ks.set_iv(iv2)
    assert np.array_equal(batch(ks, side), want(key, iv2))
    ks.free()
    ks = pa.Keyset(key, iv, 16)  # first use: a rekey
    ks.update([0], key3, iv3)
    assert np.array_equal(batch(ks, torch.cuda.current_stream()), want(key3, iv3))
    ks.free()
    ctx = pa.aead_new_direct(pa.aes128gcm, True, key, iv)  # first use: a per-record seal
    assert ctx.encrypt(b"x" * 100, 5, b"a") == ref.seal(key, iv, 5, b"a", b"x" * 100)
    ctx.free()
    hp = pa.CtrCipher(key)  # first use: an ECB block (header-protection mask)
    assert hp.mask(bytes(range(16))) == ref.aesecb(key, bytes(range(16)))
    hp.ks.free()


@pytest.mark.parametrize("aadlen", [65535, 65536, 70 << 10, (1 << 20) + 5])
def test_large_aad_batch_via_flags(ref, aadlen):
    # the AAD length's bits 16..31 travel in flags (PTLS_MI355X_RECORD_AAD_LEN); batch seal and open against fusion
    rng = np.random.default_rng(aadlen)
    lens = np.array([0, 1, 1500, 16384, 100000])
    n = len(lens)
    b = RecordBatch.build(lens, 0, seqs=rng.integers(0, 2**40, n, dtype=np.uint64))
    recs = b.seal.copy()
    recs["aad_off"] = np.arange(n) * ((aadlen + 15) // 16 * 16)
    recs["aad_len"] = aadlen & 0xFFFF
    recs["flags"] = aadlen >> 16
    key, iv = rng.bytes(32), rng.bytes(12)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(n * ((aadlen + 15) // 16 * 16)), np.uint8)
    ks = pa.Keyset(key, iv, 32)
    from gpu_util import gpu_open, gpu_seal

    sealed = gpu_seal(ks, recs, pt, aad, b.sealed_bytes)
    for i, r in enumerate(recs):
        a0 = int(r["aad_off"])
        want = ref.seal(key, iv, int(r["seq"]), aad[a0:a0 + aadlen].tobytes(),
                        pt[int(r["in_off"]):int(r["in_off"]) + int(r["len"])].tobytes())
        assert sealed[int(r["out_off"]):int(r["out_off"]) + int(r["len"]) + 16].tobytes() == want, i
    orecs = recs.copy()
    orecs["in_off"], orecs["out_off"] = b.open["in_off"], b.open["out_off"]
    back, ok = gpu_open(ks, orecs, sealed, aad, b.pt_bytes)
    assert ok.all()
    for r in orecs:
        assert np.array_equal(back[int(r["out_off"]):int(r["out_off"]) + int(r["len"])],
                              pt[int(r["out_off"]):int(r["out_off"]) + int(r["len"])])
    ks.free()


def test_per_record_large_aad_and_record(ref):
    rng = np.random.default_rng(79)
    for key_size, ln, al in [(16, 3000, 70 << 10), (32, 17 << 20, 13), (16, 5, 200000)]:
        key, iv = rng.bytes(key_size), rng.bytes(12)
        alg = pa.aes128gcm if key_size == 16 else pa.aes256gcm
        ctx = pa.aead_new_direct(alg, True, key, iv)
        pt, aad = rng.bytes(ln), rng.bytes(al)
        want = ref.seal(key, iv, 9, aad, pt)
        assert ctx.encrypt(pt, 9, aad) == want
        assert ctx.decrypt(want, 9, aad) == pt
        ctx.free()


def test_encrypt_v_and_fused_header_protection(ref):
    rng = np.random.default_rng(80)
    key, iv, hpkey = rng.bytes(16), rng.bytes(12), rng.bytes(16)
    ctx = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
    hp = pa.CtrCipher(hpkey)
    for parts in ([0], [5, 0, 7], [1] * 40, [16384, 1], [3, 1200, 0, 9]):
        vecs = [rng.bytes(p) for p in parts]
        aad = rng.bytes(5)
        assert ctx.encrypt_v(vecs, 42, aad) == ref.seal(key, iv, 42, aad, b"".join(vecs))
    for ln in (1, 4, 20, 1200):
        pt, aad = rng.bytes(ln), rng.bytes(13)
        sample_off = min(2, ln)  # the sample may reach into the tag
        sealed, mask = ctx.encrypt_s(pt, 7, aad, hp, sample_off)
        want, want_mask = ref.seal_with_hp(key, iv, 7, aad, pt, hpkey, sample_off)
        assert sealed == want and mask == want_mask, ln
    ctx.free()


def test_many_key_random_order_on_pinned_host_arenas(ref):
    # many-key keyset, records in random key order (device grouping reads the host-resident descriptors), every arena,
    # the descriptors and the ok bytes in pinned host memory
    rng = np.random.default_rng(81)
    n, nkeys = 4000, 333
    lens = rng.integers(0, 6000, n)
    key_idx = rng.integers(0, nkeys, n)
    b = RecordBatch.build(lens, rng.integers(0, 30, n), seqs=rng.integers(0, 2**48, n, dtype=np.uint64), key_idx=key_idx)
    keys, ivs = np.frombuffer(rng.bytes(nkeys * 16), np.uint8), np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    h_seal, h_open, h_pt, h_aad = pinned(b.seal), pinned(b.open), pinned(pt), pinned(aad)
    h_sealed = torch.zeros(b.sealed_bytes, dtype=torch.uint8).pin_memory()
    ks = pa.Keyset(keys, ivs, 16)
    s = torch.cuda.current_stream().cuda_stream
    pa.seal_batch(ks, h_seal.data_ptr(), n, h_pt.data_ptr(), h_aad.data_ptr(), h_sealed.data_ptr(), s)
    torch.cuda.synchronize()
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 16, b.seal, pt, aad, want, nthreads=8)
    assert np.array_equal(h_sealed.numpy(), want)
    h_back = torch.zeros(b.pt_bytes, dtype=torch.uint8).pin_memory()
    h_ok = torch.full((n,), 0xAA, dtype=torch.uint8).pin_memory()
    h_sealed[int(b.seal[17]["out_off"])] ^= 1
    pa.open_batch(ks, h_open.data_ptr(), n, h_sealed.data_ptr(), h_aad.data_ptr(), h_back.data_ptr(), h_ok.data_ptr(), s)
    torch.cuda.synchronize()
    want_ok = np.ones(n, np.uint8)
    want_ok[17] = 0
    assert np.array_equal(h_ok.numpy(), want_ok)
    ks.free()


def test_tls_records_on_pinned_host_arenas(ref):
    # TLS 1.3 framing + the unpad kernel with wire records, plaintext, ok bytes and results in pinned host memory
    rng = np.random.default_rng(82)
    n = 500
    lens = rng.integers(0, 16385, n)
    b = RecordBatch.build(lens, 0, seqs=np.arange(n, dtype=np.uint64))
    seal = b.seal.copy()
    seal["flags"] = 23
    wire_slot = (lens + 22 + 15) // 16 * 16
    wire_off = np.concatenate([[0], np.cumsum(wire_slot)[:-1]]).astype(np.uint64)
    seal["out_off"] = wire_off
    key, iv = rng.bytes(16), rng.bytes(12)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    h_seal, h_pt = pinned(seal), pinned(pt)
    h_wire = torch.zeros(int(wire_slot.sum()), dtype=torch.uint8).pin_memory()
    ks = pa.Keyset(key, iv, 16)
    s = torch.cuda.current_stream().cuda_stream
    pa.seal_tls_records(ks, h_seal.data_ptr(), n, h_pt.data_ptr(), h_wire.data_ptr(), s)
    torch.cuda.synchronize()
    wire = h_wire.numpy()
    for i in range(0, n, 37):
        ln, o = int(lens[i]), int(wire_off[i])
        inner = pt[int(b.seal[i]["in_off"]):int(b.seal[i]["in_off"]) + ln].tobytes() + b"\x17"
        hdr = bytes([23, 3, 3, (ln + 17) >> 8, (ln + 17) & 0xFF])
        assert wire[o:o + 5].tobytes() == hdr
        assert wire[o + 5:o + 22 + ln].tobytes() == ref.seal(key, iv, i, hdr, inner), i
    # the opened plaintext of record i is len + 1 bytes (the inner type follows the content): slots of their own
    back_b = RecordBatch.build(lens + 1, 0)
    opn = seal.copy()
    opn["in_off"], opn["out_off"], opn["len"] = wire_off, back_b.seal["in_off"], lens + 1
    h_open = pinned(opn)
    h_back = torch.zeros(back_b.pt_bytes, dtype=torch.uint8).pin_memory()
    h_ok = torch.zeros(n, dtype=torch.uint8).pin_memory()
    h_res = torch.zeros(n * 8, dtype=torch.uint8).pin_memory()
    pa.open_tls_records(ks, h_open.data_ptr(), n, h_wire.data_ptr(), h_back.data_ptr(), h_ok.data_ptr(), h_res.data_ptr(), s)
    torch.cuda.synchronize()
    assert h_ok.numpy().all()
    res = h_res.numpy().view(pa.TLS_RESULT_DTYPE)
    assert np.array_equal(res["plain_len"], lens) and (res["content_type"] == 23).all() and (res["status"] == 0).all()
    back = h_back.numpy()
    for i in range(0, n, 41):
        o, p0, ln = int(back_b.seal[i]["in_off"]), int(b.seal[i]["in_off"]), int(lens[i])
        assert np.array_equal(back[o:o + ln], pt[p0:p0 + ln])
    ks.free()


@pytest.mark.parametrize("key_size", [16, 32])
def test_long_records_over_many_workgroups_vs_fusion(ref, key_size):
    # a lone record from 256 KiB on runs over many workgroups (launch_span: spans of 2^e 16-step units, their partials
    # combined by a tree with H^(128 * 2^e)); lengths around the threshold and the span sizes, AADs of 0, 13 and 70,000
    # bytes, through the per-record calls: sealed bytes equal fusion's, open recovers them, a flipped bit anywhere fails
    rng = np.random.default_rng(4242 + key_size)
    alg = pa.aes128gcm if key_size == 16 else pa.aes256gcm
    key, iv = rng.bytes(key_size), rng.bytes(12)
    enc, dec = pa.aead_new_direct(alg, True, key, iv), pa.aead_new_direct(alg, False, key, iv)
    cases = [(262143, 13), (262144, 0), (262161, 13), (524288 + 5, 70000), ((1 << 20) + 17, 13), (3 * (1 << 20) + 1, 0),
             ((1 << 22) + 2047, 13)]
    for ln, al in cases:
        pt, aad, seq = rng.bytes(ln), rng.bytes(al), int(rng.integers(0, 2**62))
        want = ref.seal(key, iv, seq, aad, pt)
        assert enc.encrypt(pt, seq, aad) == want, (ln, al)
        assert dec.decrypt(want, seq, aad) == pt, (ln, al)
        bad = bytearray(want)
        bad[int(rng.integers(0, len(bad)))] ^= 0x08
        assert dec.decrypt(bytes(bad), seq, aad) is None, (ln, al)
    # with the header-protection mask of a sample after the long seal (a launch after the span launches)
    hpkey = rng.bytes(key_size)
    hp = pa.CtrCipher(hpkey)
    pt, aad = rng.bytes(300000), rng.bytes(13)
    sealed, mask = enc.encrypt_s(pt, 9, aad, hp, 299990)  # the sample reaches into the tag
    assert (sealed, mask) == ref.seal_with_hp(key, iv, 9, aad, pt, hpkey, 299990)
    hp.ks.free()
    enc.free()
    dec.free()


@pytest.mark.parametrize("key_size,ct,case", [(16, False, "10x1MiB"), (32, False, "mixed"), (16, True, "mixed"),
                                              (16, False, "threshold"), (32, True, "two_huge"), (16, False, "manykey"),
                                              (32, True, "manykey")])
def test_small_batch_long_records_spread_vs_fusion(ref, key_size, ct, case):
    # a batch of fewer records than CUs whose long records (>= 512 KiB) are shared by the spare workgroups
    # (spread_pieces): every sealed record equals fusion's, opens verify, and a tampered long record is rejected while
    # its neighbours still open. "manykey": records of 5 connections in random key order (the batch is grouped by key
    # on the device, and the pieces of one workgroup may change keys)
    rng = np.random.default_rng({"10x1MiB": 1, "mixed": 2, "threshold": 3, "two_huge": 4, "manykey": 5}[case] + key_size)
    if case == "10x1MiB":
        lens = np.full(10, 1 << 20)
    elif case == "mixed":
        lens = np.concatenate([rng.integers(0, 3000, 40), rng.integers(256 << 10, 3 << 20, 6)])
        rng.shuffle(lens)
    elif case == "threshold":
        lens = np.array([(512 << 10) - 1, 512 << 10, (512 << 10) + 1, 16, 0, (512 << 10) + 15, 100000, 300000])
    elif case == "manykey":
        lens = np.concatenate([rng.integers(0, 5000, 16), rng.integers(512 << 10, 2 << 20, 8)])
        rng.shuffle(lens)
    else:
        lens = np.array([5 << 20, 77, (9 << 20) + 3])
    n = len(lens)
    nkeys = 5 if case == "manykey" else 1
    key_idx = rng.integers(0, nkeys, n) if nkeys > 1 else None
    b = RecordBatch.build(lens, rng.integers(0, 40, n), seqs=rng.integers(0, 2**62, n, dtype=np.uint64), key_idx=key_idx)
    key, iv = rng.bytes(key_size * nkeys), rng.bytes(12 * nkeys)
    ks = pa.Keyset(key, iv, key_size)
    ks.set_constant_time(ct)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    dev = torch.device("cuda:0")
    d_seal, d_open = (torch.from_numpy(x.view(np.uint8).copy()).to(dev) for x in (b.seal, b.open))
    d_pt, d_aad = torch.from_numpy(pt.copy()).to(dev), torch.from_numpy(aad.copy()).to(dev)
    d_out = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):  # the second launch reuses the scratch (its counters back at zero)
        pa.seal_batch(ks, d_seal.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(), d_out.data_ptr(), s)
    torch.cuda.synchronize()
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, np.frombuffer(key, np.uint8), np.frombuffer(iv, np.uint8), key_size, b.seal, pt, aad, want, nthreads=8)
    got = d_out.cpu().numpy()
    for i in range(n):  # per record, so that a failure names it
        o, ln = int(b.seal["out_off"][i]), int(lens[i])
        assert np.array_equal(got[o:o + ln + 16], want[o:o + ln + 16]), (i, ln)
    long_idx = int(np.argmax(lens))
    bad = d_out.clone()
    o = int(b.seal["out_off"][long_idx]) + int(lens[long_idx]) // 2
    bad[o] ^= 1
    d_back = torch.zeros(b.pt_bytes, dtype=torch.uint8, device=dev)
    d_ok = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    pa.open_batch(ks, d_open.data_ptr(), n, bad.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    torch.cuda.synchronize()
    ok = d_ok.cpu().numpy()
    assert ok[long_idx] == 0 and all(ok[i] == 1 for i in range(n) if i != long_idx), ok
    back = d_back.cpu().numpy()
    for i in range(n):
        if i != long_idx:
            io, ln = int(b.seal["in_off"][i]), int(lens[i])
            assert np.array_equal(back[io:io + ln], pt[io:io + ln]), i
    ks.free()
