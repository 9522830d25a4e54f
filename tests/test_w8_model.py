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


# ---- lane-level models of the scattered chains (ghash.h group_scatter / group_gather / group_ws, round 5)

def _dpp(vals, src_of):  # update_dpp within each 8-lane group: lane y reads lane src_of(y)
    return [vals[src_of(y)] for y in range(8)]


def _scatter(t):  # t[y] = the 4 dwords of lane y
    b = [(y & 4) != 0 for y in range(8)]
    c = [(y & 2) != 0 for y in range(8)]
    k0 = [t[y][2] if b[y] else t[y][0] for y in range(8)]
    k1 = [t[y][3] if b[y] else t[y][1] for y in range(8)]
    s0 = [t[y][0] if b[y] else t[y][2] for y in range(8)]
    s1 = [t[y][1] if b[y] else t[y][3] for y in range(8)]
    mirror = lambda y: 7 - y  # row_half_mirror inside 8 lanes
    m0 = [k ^ s for k, s in zip(k0, _dpp(s0, mirror))]
    m1 = [k ^ s for k, s in zip(k1, _dpp(s1, mirror))]
    kk = [m1[y] if c[y] else m0[y] for y in range(8)]
    ss = [m0[y] if c[y] else m1[y] for y in range(8)]
    m = [k ^ s for k, s in zip(kk, _dpp(ss, lambda y: y ^ 2))]  # quad_perm [2,3,0,1]
    return [a ^ s for a, s in zip(m, _dpp(m, lambda y: y ^ 1))]  # quad_perm [1,0,3,2]


def _gather(g):
    a = _dpp(g, lambda y: y & 4)  # quad_perm [0,0,0,0]
    b = _dpp(g, lambda y: (y & 4) | 2)  # quad_perm [2,2,2,2]
    am, bm = _dpp(a, lambda y: 7 - y), _dpp(b, lambda y: 7 - y)
    return [[am[y], bm[y], a[y], b[y]] if y & 4 else [a[y], b[y], am[y], bm[y]] for y in range(8)]


def test_group_scatter_gives_each_lane_its_dword_of_the_sum():
    rng = np.random.default_rng(11)
    for _ in range(200):
        t = [[int(x) for x in rng.integers(0, 2**32, 4, dtype=np.uint64)] for _ in range(8)]
        total = [0, 0, 0, 0]
        for y in range(8):
            for c in range(4):
                total[c] ^= t[y][c]
        g = _scatter(t)
        assert all(g[y] == total[y >> 1] for y in range(8))
        assert all(row == total for row in _gather(g))


def test_group_ws_nibble_offsets_equal_gmul_group_w():
    # gmul_group_w: shift sh ^ 4 (i ^ 1), sh = 4 f + 16 (y & 1); group_ws: 16 (y & 1) + (4 f ^ 4 (i ^ 1)); the same
    # nibble of the lane's dword y >> 1, i.e. window 4 y + (i ^ f) of its halfword (ghash.h, window-major comment)
    for lane in range(64):
        y, f = lane & 7, (lane >> 2) & 3
        for i in range(4):
            old = (4 * f + 16 * (y & 1)) ^ (4 * (i ^ 1))
            new = 16 * (lane & 1) + ((4 * f) ^ (4 * (i ^ 1)))
            assert old == new
            u = i ^ f  # window 4y + u sits at bit 4 (u ^ 1) of the halfword
            assert new == 16 * (y & 1) + 4 * (u ^ 1)


def test_scattered_serial_chain_equals_the_powers():
    # the chain run on scattered values is the plain chain: a link's terms XOR-reduced once over the group equal the
    # all-reduced product (linearity), so sum_r v_r H^(8 - r) comes out for any rank rotation
    rng = np.random.default_rng(12)
    h = int.from_bytes(rng.bytes(16), "big")
    for _ in range(10):
        v = [int.from_bytes(rng.bytes(16), "big") for _ in range(8)]
        rot = int(rng.integers(0, 8))
        rank = [(j - rot) % 8 for j in range(8)]
        want = 0
        for j in range(8):
            want ^= gmul(v[j], gpow(h, 8 - rank[j]))
        # scattered: each link's product split into 8 lane terms (any split whose XOR is the product), plus the value
        # of the lane of rank r on that lane; the reduce-scatter gives each lane its dword of the sum
        to_w = lambda x: [(x >> (96 - 32 * c)) & 0xFFFFFFFF for c in range(4)]
        from_w = lambda w: (w[0] << 96) | (w[1] << 64) | (w[2] << 32) | w[3]
        cur = 0
        for r in range(8):
            prod = gmul(cur, h) if r else 0
            parts = [int.from_bytes(rng.bytes(16), "big") for _ in range(7)]
            last = prod
            for p in parts:
                last ^= p
            terms = parts + [last]
            t = [to_w(terms[y] ^ (v[y] if rank[y] == r else 0)) for y in range(8)]
            g = _scatter(t)
            cur = from_w([g[2 * q] for q in range(4)])
            assert all(g[y] == to_w(cur)[y >> 1] for y in range(8))
        assert gmul(cur, h) == want


# ---- 4-lane groups (ghash.h group4_*, round 5: the W8 serial kernel's whole runs)

def _scatter4(t):  # t[y] = the 4 dwords of lane y of a quad
    b = [(y & 2) != 0 for y in range(4)]
    c = [(y & 1) != 0 for y in range(4)]
    k0 = [t[y][2] if b[y] else t[y][0] for y in range(4)]
    k1 = [t[y][3] if b[y] else t[y][1] for y in range(4)]
    s0 = [t[y][0] if b[y] else t[y][2] for y in range(4)]
    s1 = [t[y][1] if b[y] else t[y][3] for y in range(4)]
    m0 = [k0[y] ^ s0[y ^ 2] for y in range(4)]  # quad_perm [2,3,0,1]
    m1 = [k1[y] ^ s1[y ^ 2] for y in range(4)]
    kk = [m1[y] if c[y] else m0[y] for y in range(4)]
    ss = [m0[y] if c[y] else m1[y] for y in range(4)]
    return [kk[y] ^ ss[y ^ 1] for y in range(4)]  # quad_perm [1,0,3,2]


def test_group4_scatter_gives_each_lane_its_dword_of_the_sum():
    rng = np.random.default_rng(21)
    for _ in range(200):
        t = [[int(x) for x in rng.integers(0, 2**32, 4, dtype=np.uint64)] for _ in range(4)]
        total = [t[0][c] ^ t[1][c] ^ t[2][c] ^ t[3][c] for c in range(4)]
        assert _scatter4(t) == total


def _g8_window(w):  # gmul_group_w: window w -> (dword, bit offset in it, bank group, table row offset)
    y, u = w >> 2, w & 3
    return (y >> 1, 16 * (y & 1) + 4 * (u ^ 1), w & 15, (w >> 4) * 4096 + (w & 15) * 16)


def test_group4_lookups_read_the_same_windows_as_gmul_group_w():
    # lane y of a quad, lookup i: window 8y + (i ^ f), f = (lane >> 1) & 7, from its dword y at bit sh[i] and address
    # Wi[i] - T (group4_ws); every window of the operand once per group, at gmul_group_w's bit and table entry
    for lane in range(64):
        y, f = lane & 3, (lane >> 1) & 7
        B = (y >> 1) * 4096 + (y & 1) * 128 + f * 16
        ws = set()
        for i in range(8):
            w = 8 * y + (i ^ f)
            ws.add(w)
            dword, bit, _, off = _g8_window(w)
            assert dword == y and bit == 4 * ((i ^ f) ^ 1) and off == B ^ (i << 4)
        assert ws == set(range(8 * y, 8 * y + 8))


def test_group4_lookups_are_conflict_free_per_phase():
    # the 16 lanes of a ds_read_b128 phase (4 quads) read 16 distinct bank groups at every lookup
    for p0 in range(0, 64, 16):
        for i in range(8):
            banks = {_g8_window(8 * (l & 3) + (i ^ ((l >> 1) & 7)))[2] for l in range(p0, p0 + 16)}
            assert len(banks) == 16


def test_group4_scattered_chain_equals_the_powers():
    rng = np.random.default_rng(22)
    h = int.from_bytes(rng.bytes(16), "big")
    to_w = lambda x: [(x >> (96 - 32 * c)) & 0xFFFFFFFF for c in range(4)]
    from_w = lambda w: (w[0] << 96) | (w[1] << 64) | (w[2] << 32) | w[3]
    for _ in range(10):
        v = [int.from_bytes(rng.bytes(16), "big") for _ in range(4)]
        rot = int(rng.integers(0, 4))
        rank = [(j - rot) % 4 for j in range(4)]
        want = 0
        for j in range(4):
            want ^= gmul(v[j], gpow(h, 4 - rank[j]))
        cur = 0
        for r in range(4):
            prod = gmul(cur, h) if r else 0
            parts = [int.from_bytes(rng.bytes(16), "big") for _ in range(3)]
            terms = parts + [prod ^ parts[0] ^ parts[1] ^ parts[2]]
            g = _scatter4([to_w(terms[y] ^ (v[y] if rank[y] == r else 0)) for y in range(4)])
            cur = from_w(g)
        assert gmul(cur, h) == want
