"""Randomised batches against lib/fusion.c: every shape knob at once (key count and order, key size, record and AAD
lengths from a heavy-tailed mix, odd slot gaps, schedule), seal bit-exact and open with one tampered record.

Each case draws its knobs from a seeded generator, so a failure names a reproducible seed. GPU only."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef  # noqa: E402
from picotls_amd.records import RecordBatch  # noqa: E402

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
HAVE_REF = os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libfusion_ref.so"))

import sys  # noqa: E402

sys.path.insert(0, HERE)
from gpu_util import gpu_open, gpu_seal  # noqa: E402


@pytest.fixture(scope="module")
def ref():
    assert torch.cuda.is_available(), "no GPU visible"
    pa.load_library()
    if not HAVE_REF:
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    return FusionRef()


def _lengths(rng, n):
    # mostly short (QUIC-like), some TLS-sized, a few long: exercises whole, unit and steady-state paths together
    kind = rng.random(n)
    return np.where(kind < 0.5, rng.integers(0, 1500, n),
                    np.where(kind < 0.9, rng.integers(1500, 16641, n), rng.integers(16641, 70000, n)))


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_batches_vs_fusion(ref, seed):
    rng = np.random.default_rng(9000 + seed)
    n = int(rng.integers(1, 2500))
    nkeys = int(rng.choice([1, 2, 7, 300]))
    key_size = int(rng.choice([16, 32]))
    key_idx = rng.integers(0, nkeys, n)
    if rng.random() < 0.5:
        key_idx = np.sort(key_idx)
    lens = _lengths(rng, n)
    aads = rng.integers(0, 100, n)
    b = RecordBatch.build(lens, aads, seqs=rng.integers(0, 2**62, n, dtype=np.uint64), key_idx=key_idx,
                          pt_gap=int(rng.integers(0, 3)) * 16, sealed_gap=int(rng.integers(0, 3)) * 16)
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, key_size)
    ks.set_schedule(str(rng.choice(["auto", "lockstep", "chunked"])), allow_variable_time=True)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, key_size, b.seal, pt, aad, expect, nthreads=8)
    assert np.array_equal(sealed, expect), f"seed {seed}: n={n} nkeys={nkeys} key_size={key_size}"
    victim = int(rng.integers(0, n))
    bad = expect.copy()
    bad[int(b.seal[victim]["out_off"]) + int(rng.integers(0, int(lens[victim]) + 16))] ^= 0x80
    plain, ok = gpu_open(ks, b.open, bad, aad, b.pt_bytes)
    want_ok = np.ones(n, np.uint8)
    want_ok[victim] = 0
    assert np.array_equal(ok, want_ok), f"seed {seed}"
    for i in range(n):
        if i == victim:
            continue
        o, ln = int(b.open[i]["out_off"]), int(lens[i])
        assert np.array_equal(plain[o:o + ln], pt[o:o + ln]), f"seed {seed} record {i}"
    ks.free()


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_w8_batches_odd_offsets_vs_fusion(ref, seed):
    """Batches large enough for the W8 kernels (2048 records and more; W8_MIN_RECS is 256 since round 5) with records at odd byte offsets (slot gaps of 1-47
    bytes): the paired half-line and line stores of round 5 (4-lane groups, cut units) decide their pairs from the
    output addresses, which then straddle lines by any amount. Seal bit-exact against fusion, open with tampering."""
    rng = np.random.default_rng(9100 + seed)
    n = int(rng.integers(2048, 12000))
    nkeys = int(rng.choice([1, 3, 40, 500]))
    key_size = int(rng.choice([16, 32]))
    key_idx = np.sort(rng.integers(0, nkeys, n))
    lens = _lengths(rng, n) if seed % 2 else rng.integers(900, 1400, n)  # (odd seeds: the mixed shapes; even: short)
    aads = rng.integers(0, 40, n)
    b = RecordBatch.build(lens, aads, seqs=rng.integers(0, 2**62, n, dtype=np.uint64), key_idx=key_idx,
                          pt_gap=int(rng.integers(1, 48)), sealed_gap=int(rng.integers(1, 48)), aad_gap=int(rng.integers(0, 5)))
    assert (b.seal["out_off"] % 16 != 0).any()
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, key_size)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    expect = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, key_size, b.seal, pt, aad, expect, nthreads=8)
    assert np.array_equal(sealed, expect), f"seed {seed}: n={n} nkeys={nkeys} key_size={key_size}"
    victims = rng.choice(n, 5, replace=False)
    bad = expect.copy()
    for v in victims:
        bad[int(b.seal[v]["out_off"]) + int(rng.integers(0, int(lens[v]) + 16))] ^= 0x04
    plain, ok = gpu_open(ks, b.open, bad, aad, b.pt_bytes)
    want_ok = np.ones(n, np.uint8)
    want_ok[victims] = 0
    assert np.array_equal(ok, want_ok), f"seed {seed}"
    keep = np.ones(b.pt_bytes, bool)
    for v in victims:
        o = int(b.open[v]["out_off"])
        keep[o:o + int(lens[v])] = False
    mask = np.zeros(b.pt_bytes, bool)
    for i in range(n):
        o = int(b.open[i]["out_off"])
        mask[o:o + int(lens[i])] = True
    sel = mask & keep
    assert np.array_equal(plain[sel], pt[sel]), f"seed {seed}"
    ks.free()
