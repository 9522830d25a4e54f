"""The constant-time GHASH variant (ptls_mi355x_keyset_set_constant_time / PTLS_MI355X_CONSTANT_TIME=1), bit-exact vs
lib/fusion.c on the paths it changes: the last multiply of every lane (whole records with aligned streams, 2 KiB units
of long records, units of a one-record launch) and the unit combine. The counter evidence that its LDS conflicts do not
depend on keys or data is tools/ct_probe.py under rocprofv3."""
import os
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef  # noqa: E402
from picotls_amd.records import RecordBatch  # noqa: E402
from gpu_util import gpu_open, gpu_seal  # noqa: E402

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
HAVE_REF = os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libfusion_ref.so"))


@pytest.fixture(scope="module")
def ref():
    assert torch.cuda.is_available()
    pa.load_library()
    if not HAVE_REF:
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    return FusionRef()


@pytest.mark.parametrize("key_size,nkeys,lens", [(16, 1, "uniform1200"), (32, 1, "uniform16k"), (16, 9, "mixed"),
                                                 (32, 300, "mixed")])
def test_ct_batches_vs_fusion(ref, key_size, nkeys, lens):
    rng = np.random.default_rng(900 + nkeys + key_size)
    n = {"uniform1200": 6000, "uniform16k": 600, "mixed": 3000}[lens]
    ln = {"uniform1200": np.full(n, 1200), "uniform16k": np.full(n, 16384),
          "mixed": rng.integers(0, 40000, n)}[lens]
    key_idx = np.sort(rng.integers(0, nkeys, n)) if nkeys > 1 else None
    b = RecordBatch.build(ln, rng.integers(0, 40, n), seqs=rng.integers(0, 2**48, n, dtype=np.uint64), key_idx=key_idx)
    keys = np.frombuffer(rng.bytes(nkeys * key_size), np.uint8)
    ivs = np.frombuffer(rng.bytes(nkeys * 12), np.uint8)
    pt = np.frombuffer(rng.bytes(b.pt_bytes), np.uint8)
    aad = np.frombuffer(rng.bytes(max(b.aad_bytes, 1)), np.uint8)
    ks = pa.Keyset(keys, ivs, key_size)
    ks.set_constant_time(True)
    sealed = gpu_seal(ks, b.seal, pt, aad, b.sealed_bytes)
    want = np.zeros(b.sealed_bytes, np.uint8)
    ref.run_batch(True, keys, ivs, key_size, b.seal, pt, aad, want, nthreads=8)
    assert np.array_equal(sealed, want)
    bad = want.copy()
    victim = n // 3
    bad[int(b.seal[victim]["out_off"]) + int(ln[victim]) + 3] ^= 0x40  # a tag byte
    back, ok = gpu_open(ks, b.open, bad, aad, b.pt_bytes)
    assert [i for i in range(n) if not ok[i]] == [victim]
    for r in b.open[::97]:
        o, L = int(r["out_off"]), int(r["len"])
        assert np.array_equal(back[o:o + L], pt[o:o + L])
    ks.free()


def test_ct_per_record_path_vs_fusion(ref):
    # one-record launches cut the record into 1..16-step units (combined with the uniform-table multiply in CT mode)
    rng = np.random.default_rng(950)
    key, iv = rng.bytes(16), rng.bytes(12)
    enc = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
    enc.ks.set_constant_time(True)
    for ln in [0, 1, 15, 16, 17, 100, 1199, 1200, 3000, 16384, 70000, 300000]:
        pt, aad = rng.bytes(ln), rng.bytes(int(rng.integers(0, 30)))
        want = ref.seal(key, iv, ln * 7, aad, pt)
        assert enc.encrypt(pt, ln * 7, aad) == want, ln
        assert enc.decrypt(want, ln * 7, aad) == pt, ln
    enc.free()


def test_ct_picotls_vtable_pairs():
    # the whole vtable suite against fusion with every keyset in constant-time mode (PTLS_MI355X_CONSTANT_TIME=1)
    exe = os.path.join(HERE, "c", "_bin", "test_vtable")
    if not os.path.exists(exe):
        pytest.skip("tests/c/_bin/test_vtable not built (needs picotls headers at build time)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, PTLS_MI355X_CONSTANT_TIME="1"))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "not ok" not in r.stdout
