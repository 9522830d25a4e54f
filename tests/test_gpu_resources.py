"""Resource bounds and the round-2 advisor's edge cases, through the engine's C ABI:

  * the staging pool is bounded (fusion's context owns and frees its memory,
    lib/fusion.c:1043-1049): a call on a 256 MiB record does not leave its pinned buffer behind;
  * the picotls AEAD contexts are constant-time by default (item 3; fusion's AES-NI / PCLMUL code is constant-time,
    lib/fusion.c:157-186, :323-335), and a lone long record still runs over many workgroups in that mode;
  * encrypt_s rejects a sample offset past the record, including one that would wrap (ADVICE);
  * keyset teardown that cannot be ordered on the device waits on the host instead of clearing under a launch, and
    combined per-record calls never mix entries of different slabs (ADVICE; fresh processes, gpu_engine_worker.py).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import picotls_amd as pa  # noqa: E402
from oracle import FusionRef  # noqa: E402

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
HAVE_REF = os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libfusion_ref.so"))


@pytest.fixture(scope="module", autouse=True)
def engine():
    assert torch.cuda.is_available(), "no GPU visible"
    pa.load_library()
    assert pa.is_supported()


@pytest.fixture(scope="module")
def ref():
    if not HAVE_REF:
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    return FusionRef()


def test_staging_pool_bounded_after_a_256_mib_record(ref):
    rng = np.random.default_rng(31)
    key, iv = rng.bytes(16), rng.bytes(12)
    ctx = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
    pt = np.frombuffer(rng.bytes(1 << 20), np.uint8)
    pt = np.tile(pt, 256).tobytes()  # 256 MiB
    sealed = ctx.encrypt(pt, 7, b"hdr")
    held = pa.staging_bytes()
    assert held <= 64 << 20, held  # the 512 MiB staging buffer of that call is gone
    # the record itself: tag and a sample of the ciphertext against fusion
    want = np.zeros(len(pt) + 16, np.uint8)
    recs = np.zeros(1, dtype=pa.RECORD_DTYPE)
    recs["len"], recs["seq"], recs["aad_len"] = len(pt), 7, 3
    ref.run_batch(True, np.frombuffer(key, np.uint8), np.frombuffer(iv, np.uint8), 16, recs,
                  np.frombuffer(pt + bytes(16), np.uint8), np.frombuffer(b"hdr", np.uint8), want, nthreads=8)
    got = np.frombuffer(sealed, np.uint8)
    assert np.array_equal(got, want)
    assert ctx.decrypt(sealed, 7, b"hdr") == pt
    ctx.free()
    # small calls keep their buffers pooled for the next call, and release frees the idle ones
    c2 = pa.aead_new_direct(pa.aes128gcm, True, key, iv)
    c2.encrypt(b"x" * 1200, 1, b"")
    assert 0 < pa.staging_bytes() <= 64 << 20
    c2.free()
    pa.release_staging()
    assert pa.staging_bytes() == 0


def test_picotls_contexts_are_constant_time_by_default(ref):
    rng = np.random.default_rng(32)
    key, iv = rng.bytes(32), rng.bytes(12)
    ctx = pa.aead_new_direct(pa.aes256gcm, True, key, iv)
    assert ctx.ks.constant_time
    # batch keysets too (round 4): constant-time unless PTLS_MI355X_CONSTANT_TIME=0, one-key and many-key alike
    ks = pa.Keyset(key, iv, 32)
    assert ks.constant_time == (os.environ.get("PTLS_MI355X_CONSTANT_TIME") != "0")
    ks.free()
    many = pa.Keyset(rng.bytes(16 * 300), rng.bytes(12 * 300), 16)
    assert many.constant_time == (os.environ.get("PTLS_MI355X_CONSTANT_TIME") != "0")
    many.set_constant_time(False)  # the opt-out per keyset
    assert not many.constant_time
    many.free()
    # lengths around the per-record unit rules and the many-workgroup span path (from 256 KiB), all in CT mode
    for ln in (0, 1, 16, 200, 1200, 16384, 100000, (256 << 10) - 1, 256 << 10, (1 << 20) + 33):
        pt, aad, seq = rng.bytes(ln), rng.bytes(int(rng.integers(0, 30))), int(rng.integers(0, 2**62))
        want = ref.seal(key, iv, seq, aad, pt)
        assert ctx.encrypt(pt, seq, aad) == want, ln
        assert ctx.decrypt(want, seq, aad) == pt, ln
        bad = bytearray(want)
        bad[len(bad) // 2] ^= 1
        assert ctx.decrypt(bytes(bad), seq, aad) is None, ln
    ctx.free()


def test_lockstep_schedule_never_silently_drops_constant_time():
    """asking a constant-time keyset for the lockstep schedule raises (the keyset stays constant-time),
    unless the caller says it accepts variable-time LDS access; then the schedule is set first and the setting turned
    off after. The C call itself records the schedule and a constant-time keyset keeps the chunked kernels."""
    rng = np.random.default_rng(33)
    ks = pa.Keyset(rng.bytes(16), rng.bytes(12), 16)
    ks.set_constant_time(True)
    with pytest.raises(pa.EngineError):
        ks.set_schedule("lockstep")
    assert ks.constant_time
    ks.set_schedule("chunked")
    assert ks.constant_time
    ks.set_schedule("lockstep", allow_variable_time=True)
    assert not ks.constant_time
    ks.set_schedule("lockstep")  # (no longer constant-time: nothing to protect)
    ks.free()


def test_encrypt_s_rejects_sample_past_the_record():
    rng = np.random.default_rng(33)
    ctx = pa.aead_new_direct(pa.aes128gcm, True, rng.bytes(16), rng.bytes(12))
    hp = pa.CtrCipher(rng.bytes(16))
    pt = rng.bytes(100)
    ctx.encrypt_s(pt, 1, b"", hp, 100)  # the sample may end at the tag's end
    for off in (101, 2**64 - 1, 2**64 - 8, 2**63):
        with pytest.raises(pa.EngineError):
            ctx.encrypt_s(pt, 1, b"", hp, off)
    ctx.free()
    hp.ks.free()


@pytest.mark.parametrize("mode,env", [("free_unordered", {"PTLS_MI355X_FAULT_ORDER": "1"}),
                                      ("combine_slabs", {"PTLS_MI355X_COMBINE": "4"})])
def test_engine_worker(mode, env):
    if not HAVE_REF:
        pytest.skip("oracle/_ref/libfusion_ref.so not shipped")
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_engine_worker.py"), mode], capture_output=True, text=True,
                       timeout=240, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["errors"] == []
