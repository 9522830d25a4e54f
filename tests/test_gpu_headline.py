"""The headline kernel at BASELINE.json configs[1]'s exact shape: 16 KiB TLS records,
unframed batch calls, the 5-byte TLS 1.3 record header {23, 3, 3, BE16(16384 + 16)} as AAD (lib/picotls.c:719-726,
the AAD aead_encrypt gives ptls_aead_encrypt_v), one AES-128 key, seq = record index -- picotls_amd.workloads' tls16k
workload, i.e. what bench.py times, scaled to 131,072 records: at 256 CUs that is 256-record chunks dealt out two per
workgroup (the full-size bench deals 512-record chunks, eight per workgroup), every chunk one whole run, so the batch
runs in the W8 pair's EXT 3 kernel (butterfly segment end) and its EXT 4 kernel only scans. Every sealed record and tag
against lib/fusion.c, every opened record and ok byte against fusion opening the same bytes, then tampered records
(ciphertext, tag and AAD bits) against fusion; the engine's counters show that EXT 3 processed the runs."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef  # noqa: E402
from picotls_amd.workloads import WORKLOADS, payload_torch  # noqa: E402
from gpu_util import dev  # noqa: E402

pytestmark = pytest.mark.gpu

HAVE_REF = os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                                       "libfusion_ref.so"))


def test_headline_tls16k_shape_seal_open_tamper_vs_fusion():
    assert torch.cuda.is_available(), "no GPU visible"
    if not HAVE_REF:
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    ref = FusionRef()
    n = 131072
    wl = WORKLOADS["tls16k"].scaled(n)
    b = wl.descriptors(0, n)
    assert (b.seal["len"] == 16384).all() and (b.seal["aad_len"] == 5).all()
    assert np.array_equal(b.seal["seq"], np.arange(n, dtype=np.uint64))
    keys, ivs = wl.keys()
    aad = wl.aad_arena(b, 0)
    assert bytes(aad[int(b.seal[7]["aad_off"]):int(b.seal[7]["aad_off"]) + 5]) == bytes([23, 3, 3, 0x40, 0x10])
    d_pt = payload_torch(wl.seed, b.pt_bytes, "cuda:0")
    pt = d_pt.cpu().numpy()
    ks = pa.Keyset(keys, ivs, 16)
    assert ks.constant_time  # the default every keyset has
    d_seal, d_open, d_aad = dev(b.seal), dev(b.open), dev(aad)
    d_sealed = torch.zeros(b.sealed_bytes, dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    pa.debug_counters(reset=True)
    pa.seal_batch(ks, d_seal.data_ptr(), n, d_pt.data_ptr(), d_aad.data_ptr(), d_sealed.data_ptr(), s)
    c = pa.debug_counters(reset=True)
    assert c["launches"]["w8_serial"] == 1 and c["launches"]["w8_tree"] == 1, c
    assert c["runs"]["w8_tree"] >= 256 and c["runs"]["w8_serial"] == 0, c  # every run in EXT 3
    sealed = d_sealed.cpu().numpy()
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, 16, b.seal, pt, aad, want, nthreads=8)
    if not np.array_equal(sealed, want):
        bad = [i for i in range(n) if not np.array_equal(sealed[int(b.seal[i]["out_off"]):int(b.seal[i]["out_off"]) + 16400],
                                                            want[int(b.seal[i]["out_off"]):int(b.seal[i]["out_off"]) + 16400])]
        pytest.fail(f"{len(bad)} sealed records differ from fusion, first {bad[:8]}")
    # open the sealed batch: plaintext and ok bytes against fusion opening the same records
    d_back = torch.full((b.pt_bytes,), 0x5A, dtype=torch.uint8, device="cuda:0")
    d_ok = torch.full((n,), 0xAA, dtype=torch.uint8, device="cuda:0")
    pa.open_batch(ks, d_open.data_ptr(), n, d_sealed.data_ptr(), d_aad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    c = pa.debug_counters(reset=True)
    assert c["launches"]["w8_tree"] == 1 and c["runs"]["w8_tree"] >= 256 and c["runs"]["w8_serial"] == 0, c
    ref_back, ref_ok = np.full(b.pt_bytes, 0x5A, np.uint8), np.zeros(n, np.uint8)
    _, fails = ref.run_batch(False, keys, ivs, 16, b.open, want, aad, ref_back, ok=ref_ok, nthreads=8)
    assert fails == 0 and ref_ok.all()
    assert (d_ok.cpu().numpy() == 1).all()
    assert np.array_equal(d_back.cpu().numpy(), ref_back)
    assert np.array_equal(ref_back, pt)
    # tampered records: ciphertext, tag and AAD bits of 24 records; ok bytes and the plaintext written anyway, as fusion
    rng = np.random.default_rng(1601)
    bad, badaad = want.copy(), aad.copy()
    victims = rng.choice(n, 24, replace=False)
    for t, v in enumerate(victims):
        o = int(b.open[v]["in_off"])
        if t % 3 == 0:
            bad[o + int(rng.integers(0, 16384))] ^= 1 << int(rng.integers(0, 8))
        elif t % 3 == 1:
            bad[o + 16384 + int(rng.integers(0, 16))] ^= 0x40
        else:
            badaad[int(b.open[v]["aad_off"]) + int(rng.integers(0, 5))] ^= 1
    d_bad, d_badaad = dev(bad), dev(badaad)
    d_ok.fill_(0xAA)
    pa.open_batch(ks, d_open.data_ptr(), n, d_bad.data_ptr(), d_badaad.data_ptr(), d_back.data_ptr(), d_ok.data_ptr(), s)
    c = pa.debug_counters(reset=True)
    assert c["runs"]["w8_tree"] >= 256, c
    ref_ok[:] = 0
    _, fails = ref.run_batch(False, keys, ivs, 16, b.open, bad, badaad, ref_back, ok=ref_ok, nthreads=8)
    expect = np.ones(n, np.uint8)
    expect[victims] = 0
    assert fails == 24 and np.array_equal(ref_ok, expect)
    assert np.array_equal(d_ok.cpu().numpy(), expect)
    assert np.array_equal(d_back.cpu().numpy(), ref_back)
    ks.free()
