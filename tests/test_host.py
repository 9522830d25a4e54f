"""Host-side logic: batch layout, algorithmic byte counts, shard planning, workload definitions. CPU only."""
import numpy as np
import pytest

from picotls_amd.records import RecordBatch, algorithmic_bytes, shard_ranges
from picotls_amd import workloads


def test_batch_layout_is_aligned_and_disjoint():
    rng = np.random.default_rng(0)
    lens = rng.integers(0, 5000, 500)
    aads = rng.integers(0, 70, 500)
    b = RecordBatch.build(lens, aads)
    assert (b.seal["in_off"] % 16 == 0).all() and (b.seal["out_off"] % 16 == 0).all()
    assert (b.seal["aad_off"] % 16 == 0).all()
    ends = b.seal["in_off"] + b.seal["len"]
    assert (ends[:-1] <= b.seal["in_off"][1:]).all() and ends[-1] <= b.pt_bytes
    sealed_ends = b.seal["out_off"] + b.seal["len"] + 16
    assert (sealed_ends[:-1] <= b.seal["out_off"][1:]).all() and sealed_ends[-1] <= b.sealed_bytes
    assert (b.open["in_off"] == b.seal["out_off"]).all() and (b.open["out_off"] == b.seal["in_off"]).all()
    assert b.payload_bytes == int(lens.sum())


def test_empty_batch():
    b = RecordBatch.build([], [])
    assert b.n == 0 and b.pt_bytes == 0


def test_algorithmic_bytes():
    # per record seal+open = 4L + 2A + 32 (+ 2 descriptors, + ok byte)
    lens, aads = np.array([16384]), np.array([5])
    s = algorithmic_bytes(lens, aads, True)
    o = algorithmic_bytes(lens, aads, False)
    assert s == 2 * 16384 + 5 + 40 + 16
    assert o == 2 * 16384 + 5 + 40 + 17
    assert s + o == 4 * 16384 + 2 * 5 + 32 + 80 + 1


@pytest.mark.parametrize("nshards", [1, 2, 3, 4, 8])
def test_shard_ranges_cover_and_balance(nshards):
    rng = np.random.default_rng(nshards)
    w = rng.integers(64, 16385, 10000)
    r = shard_ranges(w, nshards)
    assert r[0][0] == 0 and r[-1][1] == len(w)
    for (a, b), (c, d) in zip(r, r[1:]):
        assert b == c and a <= b
    loads = [w[a:b].sum() for a, b in r]
    assert max(loads) - min(loads) <= 2 * w.max()


def test_shard_ranges_degenerate():
    assert shard_ranges([], 4) == [(0, 0)] * 4
    assert shard_ranges([5], 3)[-1][1] == 1
    with pytest.raises(ValueError):
        shard_ranges([1], 0)


def test_workload_definitions_match_baseline():
    import json
    import os

    base = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "BASELINE.json")))
    assert "16KiB" in base["metric"] and "1200B" in base["metric"]
    w = workloads.WORKLOADS
    assert w["tls16k"].nrecs == 1 << 20 and w["tls16k"].rec_len == 16384 and w["tls16k"].key_size == 16
    assert w["quic1200"].nrecs == 4 << 20 and w["quic1200"].rec_len == 1200 and w["quic1200"].aad_len == 13
    assert w["mixed"].nkeys == 65536 and w["mixed"].key_size == 32
    assert w["shard1200"].nrecs == 32 << 20


def test_workload_shard_is_a_slice_of_the_global_batch():
    wl = workloads.WORKLOADS["quic1200"].scaled(1000)
    full = wl.descriptors(0, wl.nrecs)
    half = wl.descriptors(500, 1000)
    assert (half.seal["seq"] == full.seal["seq"][500:]).all()
    assert (half.seal["len"] == full.seal["len"][500:]).all()


def test_tls_aad_bytes():
    # TLS 1.3 record header used as AAD (lib/picotls.c:719-726): {23, 3, 3, len_hi, len_lo}, len includes the tag
    aad = workloads.tls_aad(16384)
    assert aad == bytes([23, 3, 3, (16384 + 16) >> 8, (16384 + 16) & 0xFF])


def test_payload_generator_is_seekable():
    a = workloads.payload_np(0x5EED, 0, 4096)
    b = workloads.payload_np(0x5EED, 1024, 2048)
    assert a[1024:3072].tobytes() == b.tobytes()


def test_many_key_workload_orders():
    # "mixed": records grouped by connection; "mixedrand": SURVEY 8(d) config 4 as written (key = splitmix(i) mod
    # nkeys). Either way seq counts each connection's records 0, 1, 2, ... in batch order, and a shard is a slice
    for name in ("mixed", "mixedrand"):
        wl = workloads.WORKLOADS[name].scaled(20000)
        key, seq = wl.key_and_seq(0, wl.nrecs)
        assert key.max() < wl.nkeys
        for k in np.unique(key)[:50]:
            assert (seq[key == k] == np.arange((key == k).sum())).all()
        k2, s2 = wl.key_and_seq(7000, 9000)
        assert (k2 == key[7000:9000]).all() and (s2 == seq[7000:9000]).all()
    grouped = workloads.WORKLOADS["mixed"].scaled(20000).key_and_seq(0, 20000)[0]
    rand = workloads.WORKLOADS["mixedrand"].scaled(20000).key_and_seq(0, 20000)[0]
    assert (np.diff(grouped.astype(np.int64)) >= 0).all()
    assert (np.diff(rand.astype(np.int64)) != 0).mean() > 0.9  # runs of one record: the device regroups these


def test_mixed_analysis_workloads():
    # (round 5) mixedpois: mixedrand's key counts grouped in batch order; mixedshuf: mixed's keys (equal
    # counts) in random order; mixedscatter: mixed's records at random places in the arenas, descriptors in batch order
    n = 20000
    w = workloads.WORKLOADS
    rand = w["mixedrand"].scaled(n).key_and_seq(0, n)[0]
    pois = w["mixedpois"].scaled(n).key_and_seq(0, n)[0]
    assert (pois == np.sort(rand)).all()
    mixed = w["mixed"].scaled(n).key_and_seq(0, n)[0]
    shuf, sseq = w["mixedshuf"].scaled(n).key_and_seq(0, n)
    assert (np.sort(shuf) == mixed).all() and (np.diff(shuf.astype(np.int64)) != 0).mean() > 0.9
    for k in np.unique(shuf)[:50]:
        assert (sseq[shuf == k] == np.arange((shuf == k).sum())).all()
    m = w["mixed"].scaled(n).descriptors(0, n)
    sc = w["mixedscatter"].scaled(n).descriptors(0, n)
    for f in ("len", "key_idx", "seq", "aad_len"):
        assert (sc.seal[f] == m.seal[f]).all()
    assert sc.pt_bytes == m.pt_bytes and sc.sealed_bytes == m.sealed_bytes
    order = np.argsort(sc.seal["in_off"])
    assert (np.diff(order) != 1).mean() > 0.9  # arena order is not batch order
    ends = sc.seal["in_off"][order] + sc.seal["len"][order]
    assert (ends[:-1] <= sc.seal["in_off"][order][1:]).all()  # still disjoint
    assert (sc.open["in_off"] == sc.seal["out_off"]).all() and (sc.open["out_off"] == sc.seal["in_off"]).all()


def test_lds_model_ceiling():
    import bench

    res = {"stream_blocks": 10**9, "seal_ms": 10.0}
    m = bench.lds_model(res, 16, 100)
    # a batch below W8_MIN_RECS (256): 133 x 4 B at 75 TB/s + 32 x 16 B (4-bit GHASH windows) at 150 TB/s per block
    assert abs(m["peak_at_2.4GHz"] - 1 / (532 / 75e12 + 512 / 150e12)) < 1e6
    assert abs(m["frac"] - 1e11 / m["peak_at_2.4GHz"]) < 1e-3
    assert bench.lds_model(res, 32, 100)["peak_at_2.4GHz"] < m["peak_at_2.4GHz"]
    # the W8 kernels (W8_MIN_RECS records and more): 16 x 16 B per block for the 8-bit Horner table
    w8 = bench.lds_model(res, 16, 1 << 20)
    assert abs(w8["peak_at_2.4GHz"] - 1 / (532 / 75e12 + 256 / 150e12)) < 1e6
    assert "16 ds_read_b128" in w8["per_block"]
