"""CPU models of the W8 machinery (picotls_amd/csrc/engine/ghash.h, lds_tables.h): the segment end's
serial lane Horner (w8_lane_end) equals sum_r v_r H^(8 - r) for any rank permutation, the 8-bit H^8 table's build order
is a bijection whose 16-lane phases read and write 16 distinct bank groups, and the 8-bit lookups return the product
(a GF(2^128) model in GCM's bit order, SP 800-38D Algorithm 1). The GPU suite checks the kernels end to end against
lib/fusion.c (tests/test_gpu_w8.py)."""
import numpy as np

R = 0xE1 << 120


def gmul(x, y):  # GCM's GF(2^128) product, bit 127 of the integer = x^0 (SP 800-38D Algorithm 1)
    z, v = 0, y
    for i in range(127, -1, -1):
        if (x >> i) & 1:
            z ^= v
        v = (v >> 1) ^ R if v & 1 else v >> 1
    return z


def gpow(h, e):
    r = 1 << 127  # the unit element x^0
    for _ in range(e):
        r = gmul(r, h)
    return r


def test_serial_lane_horner_equals_the_powers_for_any_rotation():
    rng = np.random.default_rng(5)
    for _ in range(20):
        h = int.from_bytes(rng.bytes(16), "big")
        v = [int.from_bytes(rng.bytes(16), "big") for _ in range(8)]
        rot = int(rng.integers(0, 8))
        rank = [(j - rot) % 8 for j in range(8)]  # lane j's rank (gcm_segment: rank = 8 - e_last)
        want = 0
        for j in range(8):
            want ^= gmul(v[j], gpow(h, 8 - rank[j]))
        # w8_lane_end: g = (the rank-0 lane's value); g = g*H ^ (rank-r lane's value), r = 1..7; then g*H
        g = 0
        for j in range(8):
            g ^= v[j] if rank[j] == 0 else 0
        for r in range(1, 8):
            g = gmul(g, h)
            for j in range(8):
                g ^= v[j] if rank[j] == r else 0
        assert gmul(g, h) == want


def test_h8_byte_table_build_order_is_a_conflict_free_bijection():
    seen = set()
    for i0 in range(0, 4096, 16):  # one 16-lane phase of build_h8_byte_table
        reads0, reads1, writes = set(), set(), set()
        for i in range(i0, i0 + 16):
            w, n = i & 15, (i >> 4) ^ ((i & 15) << 4) ^ (i & 15)
            seen.add((w, n))
            reads0.add(n >> 4)  # scratch (2w)*256 + (n >> 4)*16: bank group n >> 4
            reads1.add(n & 15)  # scratch (2w + 1)*256 + (n & 15)*16
            writes.add(w)       # n*256 + w*16
        assert len(reads0) == len(reads1) == len(writes) == 16
    assert len(seen) == 4096


def test_8bit_lookup_is_the_product():
    # entry (w, n) = e4(2w, n >> 4) ^ e4(2w + 1, n & 15), e4(p, m) = (m's 4 bits at x^(4p)..x^(4p+3)) * H^8: the XOR of
    # the 16 byte entries of an operand is its product with H^8 (byte w = bits x^(8w)..x^(8w+7), MSB first)
    rng = np.random.default_rng(9)
    h = int.from_bytes(rng.bytes(16), "big")
    h8 = gpow(h, 8)

    def e4(p, m):  # window p's entry for nibble m: sum over set bits (MSB = x^(4p))
        acc = 0
        for q in range(4):
            if (m >> (3 - q)) & 1:
                acc ^= gmul(1 << (127 - (4 * p + q)), h8)
        return acc

    for _ in range(5):
        a = int.from_bytes(rng.bytes(16), "big")
        byts = a.to_bytes(16, "big")  # byte w holds x^(8w)..x^(8w+7)
        acc = 0
        for w in range(16):
            n = byts[w]
            acc ^= e4(2 * w, n >> 4) ^ e4(2 * w + 1, n & 15)
        assert acc == gmul(a, h8)
