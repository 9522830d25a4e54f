"""The window-major GHASH layout's invariants (picotls_amd/csrc/engine/ghash.h), checked on the CPU with
a model of the kernel's lane arithmetic: the bank group of every lookup depends on the lane only (never on the table or
the operand), the 16 lanes of any ds_read_b128 phase meet 16 distinct bank groups, every 8-lane group covers each of the
32 windows once, the nibble a lane takes is the window's nibble of the operand, and the three DPP butterfly stages of
coop_last_powers transpose the group's halfwords. The GPU parity tests check the same code end to end against fusion."""
import itertools

import numpy as np

TABLE = 8192
WINDOW_MAJOR_BASES = [0x10000 + t * TABLE for t in (0, 1, 2, 3, 4, 5, 6, 8)]  # H^1..H^7, the unit combine power


def lane_base(T, lane):  # wtab_lane_base
    y, f = lane & 7, (lane >> 2) & 3
    return T + (y >> 2) * 4096 + (y & 3) * 64 + f * 16


def lookup_addr(T, lane, i, n):  # the i-th lookup of a lane, nibble value n: (n << 8) + (W ^ (i << 4))
    return (n << 8) + (lane_base(T, lane) ^ (i << 4))


def window_of(lane, i):  # window 4y + (i ^ f) of the operand
    return 4 * (lane & 7) + (i ^ ((lane >> 2) & 3))


def wtab_entry_addr(T, w, n):  # build_ghash_tables / build_elem_table with wmask: (w >> 4) * 4096 + n * 256 + (w & 15) * 16
    return T + (w >> 4) * 4096 + n * 256 + (w & 15) * 16


def test_lookup_reads_the_window_major_entry():
    for T in WINDOW_MAJOR_BASES + [146688 + TABLE]:  # + the spread fold's element table (CLDS_PART + 8192, 64-aligned)
        for lane, i, n in itertools.product(range(64), range(4), range(16)):
            assert lookup_addr(T, lane, i, n) == wtab_entry_addr(T, window_of(lane, i), n)


def test_bank_group_depends_on_lane_only_and_phases_are_conflict_free():
    rng = np.random.default_rng(7)
    # phases of 16 lanes: the plain grouping and the gfx950 ds_read_b128 one (lanes 0-3, 12-15, 20-27, ...), and any
    # set of 16 lanes with distinct lane & 15
    phases = [list(range(16 * k, 16 * k + 16)) for k in range(4)]
    phases.append([0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27])
    for _ in range(50):
        phases.append([int(16 * rng.integers(0, 4) + r) for r in range(16)])
    for phase in phases:
        assert len({lane & 15 for lane in phase}) == 16
        for i in range(4):
            for _ in range(20):  # random tables (each lane its own, as in the segment end) and random nibbles
                tabs = rng.choice(WINDOW_MAJOR_BASES, size=16)
                nibs = rng.integers(0, 16, size=16)
                groups = [(lookup_addr(int(T), lane, i, int(n)) >> 4) & 15 for T, lane, n in zip(tabs, phase, nibs)]
                assert len(set(groups)) == 16


def test_each_group_covers_every_window_once():
    for g in range(8):
        ws = sorted(window_of(lane, i) for lane in range(8 * g, 8 * g + 8) for i in range(4))
        assert ws == list(range(32))


def test_nibble_extraction_matches_the_window_definition():
    # gmul_tab's window 8q + 2k + h: dword q, byte k, high nibble (h = 0) first; coop_last_powers / gmul_group_w take
    # window 4y + u of halfword y at bit 4 (u ^ 1)
    rng = np.random.default_rng(3)
    for _ in range(200):
        a = [int(x) for x in rng.integers(0, 2**32, size=4, dtype=np.uint64)]
        for w in range(32):
            q, k, h = w >> 3, (w >> 1) & 3, w & 1
            ref = (a[q] >> (8 * k + (4 if h == 0 else 0))) & 15
            y, u = w >> 2, w & 3
            half = (a[y >> 1] >> (16 * (y & 1))) & 0xFFFF
            assert (half >> (4 * (u ^ 1))) & 15 == ref


def _dpp(v, ctrl):  # one DPP move over a 64-lane vector (quad_perm, row_half_mirror)
    out = [0] * 64
    for lane in range(64):
        if ctrl == 0x141:  # row_half_mirror: lane l <- 7 - l within 8
            src = (lane & ~7) | (7 - (lane & 7))
        else:  # quad_perm: 2 bits per lane of the quad
            src = (lane & ~3) | ((ctrl >> (2 * (lane & 3))) & 3)
        out[lane] = v[src]
    return out


def _perm(s0, s1, sel):  # v_perm_b32: bytes 0-3 of s1, 4-7 of s0
    b = list(s1.to_bytes(4, "little")) + list(s0.to_bytes(4, "little"))
    return int.from_bytes(bytes(b[(sel >> (8 * i)) & 0xFF] for i in range(4)), "little")


def test_coop_transpose_stages():
    rng = np.random.default_rng(11)
    d = [[int(x) for x in rng.integers(0, 2**32, size=64, dtype=np.uint64)] for _ in range(4)]
    orig = [list(c) for c in d]
    y = [lane & 7 for lane in range(64)]
    # slot bit 2 with lane ^ 4 (row_half_mirror, then quad_perm [3,2,1,0])
    b = [(v & 4) != 0 for v in y]
    x4 = lambda v: _dpp(_dpp(v, 0x141), 0x1B)  # noqa: E731
    r0 = x4([d[0][l] if b[l] else d[2][l] for l in range(64)])
    r1 = x4([d[1][l] if b[l] else d[3][l] for l in range(64)])
    d = [[r0[l] if b[l] else d[0][l] for l in range(64)], [r1[l] if b[l] else d[1][l] for l in range(64)],
         [d[2][l] if b[l] else r0[l] for l in range(64)], [d[3][l] if b[l] else r1[l] for l in range(64)]]
    # slot bit 1 with lane ^ 2 (quad_perm [2,3,0,1])
    b = [(v & 2) != 0 for v in y]
    r0 = _dpp([d[0][l] if b[l] else d[1][l] for l in range(64)], 0x4E)
    r1 = _dpp([d[2][l] if b[l] else d[3][l] for l in range(64)], 0x4E)
    d = [[r0[l] if b[l] else d[0][l] for l in range(64)], [d[1][l] if b[l] else r0[l] for l in range(64)],
         [r1[l] if b[l] else d[2][l] for l in range(64)], [d[3][l] if b[l] else r1[l] for l in range(64)]]
    # slot bit 0 with lane ^ 1 (quad_perm [1,0,3,2]), the sent halves packed two per dword
    b = [(v & 1) != 0 for v in y]
    ps = [0x05040100 if b[l] else 0x07060302 for l in range(64)]
    q0 = _dpp([_perm(d[1][l], d[0][l], ps[l]) for l in range(64)], 0xB1)
    q1 = _dpp([_perm(d[3][l], d[2][l], ps[l]) for l in range(64)], 0xB1)
    ua = [0x03020504 if b[l] else 0x05040100 for l in range(64)]
    ub = [0x03020706 if b[l] else 0x07060100 for l in range(64)]
    d = [[_perm(q0[l], d[0][l], ua[l]) for l in range(64)], [_perm(q0[l], d[1][l], ub[l]) for l in range(64)],
         [_perm(q1[l], d[2][l], ua[l]) for l in range(64)], [_perm(q1[l], d[3][l], ub[l]) for l in range(64)]]

    def half(dw, lane, s):  # halfword s of a lane's 128-bit value
        return (dw[s >> 1][lane] >> (16 * (s & 1))) & 0xFFFF

    for lane in range(64):
        g0 = lane & ~7
        for x in range(8):  # lane y's slot x = halfword y of lane x of the group
            assert half(d, lane, x) == half(orig, g0 + x, lane & 7)
