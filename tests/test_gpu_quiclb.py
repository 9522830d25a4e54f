"""QUIC-LB connection-ID cipher on the GPU (ptls_mi355x_quiclb_batch / ptls_mi355x_quiclb) against the reference's
known answer (t/quiclb.c:27-46), vectors written by ptls_fusion_quiclb (tests/golden/quiclb_vectors.json), the CPU
oracle (oracle/gcm_ref.c, a restatement of lib/quiclb-impl.h) and, where shipped, lib/fusion.c itself. Bit-exact.
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef, GcmOracle  # noqa: E402
from picotls_amd.records import CID_DTYPE  # noqa: E402
from vectors import splitmix_bytes  # noqa: E402

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
HAVE_REF = os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libfusion_ref.so"))

from gpu_util import dev, empty  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def engine():
    assert torch.cuda.is_available(), "no GPU visible"
    pa.load_library()
    assert pa.is_supported(), "engine reports no gfx950 device"


def _run(ks, cids, arena, out_size=None):
    """Runs one quiclb batch; returns the output arena (initialised to 0xa5 so skipped entries are visible)."""
    d_c = dev(cids.view(np.uint8))
    d_in = dev(arena)
    d_out = torch.full((out_size or len(arena),), 0xA5, dtype=torch.uint8, device="cuda")
    pa.quiclb_batch(ks, d_c.data_ptr(), len(cids), d_in.data_ptr(), d_out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_out.cpu().numpy()


def _pack(items, nkeys=1, spacing=32):
    """items: list of (data, key_idx, encrypt); returns (cids, arena) with each CID in its own 32-byte slot."""
    cids = np.zeros(len(items), CID_DTYPE)
    arena = np.zeros(max(1, len(items)) * spacing, np.uint8)
    for i, (data, ki, enc) in enumerate(items):
        off = i * spacing + (i % 5)  # odd offsets too
        arena[off:off + len(data)] = np.frombuffer(data, np.uint8)
        cids[i] = (off, off, ki, len(data), 1 if enc else 0, 0)
    return cids, arena


def test_quiclb_kat(kat):
    # t/quiclb.c:27-46 through the batch entry point: the draft vector at len 7, round trips for 7..19
    v = kat["quiclb"]
    key, pt19 = bytes.fromhex(v["key"]), bytes.fromhex(v["pt19"])
    ks = pa.Keyset(key, bytes(12), 16)
    cids, arena = _pack([(pt19[:ln], 0, True) for ln in range(7, 20)])
    out = _run(ks, cids, arena)
    assert out[0:7].tobytes().hex() == v["ct7"]
    cts = [out[c["out_off"]:c["out_off"] + c["len"]].tobytes() for c in cids]
    cids2, arena2 = _pack([(ct, 0, False) for ct in cts])
    back = _run(ks, cids2, arena2)
    for c, ln in zip(cids2, range(7, 20)):
        assert back[c["out_off"]:c["out_off"] + ln].tobytes() == pt19[:ln]
    ks.free()


def test_quiclb_fusion_vectors_multikey_both_directions():
    # every fixture vector (6 keys x lengths 7..19) in one launch, encrypt and decrypt entries interleaved
    with open(os.path.join(HERE, "golden", "quiclb_vectors.json")) as f:
        vecs = json.load(f)["vectors"]
    keys, items = [], []
    for i, v in enumerate(vecs):
        blob = splitmix_bytes(v["seed"], 16 + v["len"])
        keys.append(blob[:16])
        items.append((blob[16:], i, True))
        items.append((bytes.fromhex(v["ct"]), i, False))
    ks = pa.Keyset(b"".join(keys), bytes(12 * len(keys)), 16)
    cids, arena = _pack(items)
    out = _run(ks, cids, arena)
    for (data, ki, enc), c in zip(items, cids):
        v = vecs[ki]
        got = out[c["out_off"]:c["out_off"] + c["len"]].tobytes()
        want = bytes.fromhex(v["ct"]) if enc else splitmix_bytes(v["seed"], 16 + v["len"])[16:]
        assert got == want, (v["seed"], enc)
    ks.free()


def test_quiclb_in_place_invalid_entries_and_args():
    key = bytes(range(16))
    ks = pa.Keyset(key, bytes(12), 16)
    o = GcmOracle()
    items = [(bytes(range(ln)), 0, True) for ln in (7, 12, 19)] + [(bytes(6), 0, True), (bytes(20), 0, True),
                                                                   (bytes(9), 5, True)]
    cids, arena = _pack(items)
    cids["len"][4] = 20
    # in place: out arena == in arena
    d_c, d_a = dev(cids.view(np.uint8)), dev(arena)
    pa.quiclb_batch(ks, d_c.data_ptr(), len(cids), d_a.data_ptr(), d_a.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_a.cpu().numpy()
    for (data, _, _), c in list(zip(items, cids))[:3]:
        assert got[c["in_off"]:c["in_off"] + len(data)].tobytes() == o.quiclb(key, data, True)
    for c in cids[3:]:  # bad length / key index: untouched
        assert np.array_equal(got[c["in_off"]:c["in_off"] + 20], arena[c["in_off"]:c["in_off"] + 20])
    # empty batch is a no-op; an AES-256 keyset is refused (PTLS_QUICLB_KEY_SIZE is 16)
    pa.quiclb_batch(ks, 0, 0, 0, 0)
    ks256 = pa.Keyset(bytes(32), bytes(12), 32)
    with pytest.raises(pa.EngineError):
        pa.quiclb_batch(ks256, d_c.data_ptr(), 1, d_a.data_ptr(), d_a.data_ptr())
    ks256.free()
    ks.free()


@pytest.mark.parametrize("nkeys", [1, 37])
def test_quiclb_random_batch_vs_oracle_and_fusion(nkeys):
    rng = np.random.default_rng(nkeys)
    keys = [rng.bytes(16) for _ in range(nkeys)]
    n = 20000
    lens = rng.integers(7, 20, n)
    kidx = rng.integers(0, nkeys, n)
    enc = rng.integers(0, 2, n).astype(bool)
    items = [(rng.bytes(int(ln)), int(k), bool(e)) for ln, k, e in zip(lens, kidx, enc)]
    ks = pa.Keyset(b"".join(keys), bytes(12 * nkeys), 16)
    cids, arena = _pack(items)
    out = _run(ks, cids, arena)
    o = GcmOracle()
    ref = FusionRef() if HAVE_REF else None
    sample = rng.choice(n, 600, replace=False)
    for i in sample:
        data, k, e = items[i]
        c = cids[i]
        got = out[c["out_off"]:c["out_off"] + c["len"]].tobytes()
        assert got == o.quiclb(keys[k], data, e), i
        if ref is not None:
            assert got == ref.quiclb(keys[k], data, e), i
    ks.free()


def test_quiclb_cipher_object_round_trip(kat):
    # the picotls-shaped mirror (ptls_cipher_new(&ptls_mi355x_quiclb, is_enc, key) + ptls_cipher_encrypt)
    v = kat["quiclb"]
    key, pt19 = bytes.fromhex(v["key"]), bytes.fromhex(v["pt19"])
    enc, dec = pa.QuicLbCipher(True, key), pa.QuicLbCipher(False, key)
    for ln in range(7, 20):
        ct = enc.encrypt(pt19[:ln])
        if ln == 7:
            assert ct.hex() == v["ct7"]
        assert dec.encrypt(ct) == pt19[:ln]
    with pytest.raises(ValueError):
        enc.encrypt(bytes(6))
