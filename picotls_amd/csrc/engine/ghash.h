// picotls_amd/csrc/engine/ghash.h -- GHASH multiplies from the LDS window tables (per lane and per 8-lane group).
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_GHASH_H
#define PTLS_MI355X_ENGINE_GHASH_H

// ------------------------------------------------------------------------------------------------ GHASH (tables)

// returns a * (table t's power), where tsel = 0x10000 + t * 8192: table base for the lane (t < 8: H^(t+1)).
// The 32 window lookups are independent and folded pairwise with 3-input XORs as they land, so one multiply costs a few
// overlapped LDS round trips rather than a chain of 32 (the compiler keeps ~10 reads in flight).
__device__ __forceinline__ u32x4 gmul_tab(const lds_u8 *, u32x4 a, u32 tsel)
{
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const u32 w = a[q];
        const u32 hi = w & 0xf0f0f0f0u, lo = (w << 4) & 0xf0f0f0f0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32 sel = 0x0c020100u | (4u + k);
            const u32x4 e0 = lds_load128(__builtin_amdgcn_perm(hi, tsel, sel) + (8 * q + 2 * k) * 256);
            const u32x4 e1 = lds_load128(__builtin_amdgcn_perm(lo, tsel, sel) + (8 * q + 2 * k + 1) * 256);
#pragma unroll
            for (int c = 0; c < 4; ++c)
                acc[c] = xor3(acc[c], e0[c], e1[c]);
        }
    }
    return acc;
}

// a * (table t's power) computed by the G = 8 lanes of a group together (every lane holds a; every lane gets the
// product): lane j does the four window lookups of nibbles 4j..4j+3 and the group XOR-reduces them.
__device__ __forceinline__ u32x4 gmul_group(const lds_u8 *, u32x4 a, u32 tsel, u32 j)
{
    static_assert(ENGINE_G == 8, "one word half per lane");
    const u32 q = j >> 1, k0 = 2 * (j & 1);
    const u32 w = q == 0 ? a[0] : q == 1 ? a[1] : q == 2 ? a[2] : a[3];
    const u32 hi = w & 0xf0f0f0f0u, lo = (w << 4) & 0xf0f0f0f0u;
    const u32 base = (8 * q + 2 * k0) * 256;
    const u32x4 e0 = lds_load128(__builtin_amdgcn_perm(hi, tsel, 0x0c020100u | (4u + k0)) + base);
    const u32x4 e1 = lds_load128(__builtin_amdgcn_perm(lo, tsel, 0x0c020100u | (4u + k0)) + base + 256);
    const u32x4 e2 = lds_load128(__builtin_amdgcn_perm(hi, tsel, 0x0c020100u | (5u + k0)) + base + 512);
    const u32x4 e3 = lds_load128(__builtin_amdgcn_perm(lo, tsel, 0x0c020100u | (5u + k0)) + base + 768);
    u32x4 r;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        r[c] = xor3(e0[c], e1[c], e2[c]) ^ e3[c];
#pragma unroll
    for (int c = 0; c < 4; ++c)
        r[c] = dpp_xor8(r[c]);
    return r;
}

// ------------------------------------------------------------------------------------------------ GHASH (window-major)
//
// gmul_tab's tables are nibble-major: entry (window w, nibble n) at T + w * 256 + n * 16, so a ds_read_b128's 16-byte
// bank group is the nibble n. Lanes that read one table row at one window (the Horner step: every lane H^8, window by
// window) then never conflict: equal nibbles read the same address, different ones different bank groups. Lanes that
// read different rows in one instruction (each lane its own power, or its own windows of a shared product) conflict
// whenever two of them meet the same nibble: a count that follows the data (profiles/r2_ct_evidence.txt).
//
// Window-major tables (H^1..H^7 in slots 0..6 in both modes, the unit combine power in slot 8 in the default mode) put entry
// (w, n) at T + (w >> 4) * 4096 + n * 256 + (w & 15) * 16: the bank group is (w & 15), whatever the data. Lane `lane`
// of an 8-lane group (index y = lane & 7) handles the four windows 4y..4y+3 of the operand's halfword y, window
// 4y + (i ^ f) at its i-th lookup, f = (lane >> 2) & 3. At every lookup the 16 lanes of a ds_read_b128 phase (16
// distinct values of lane & 15) then read the 16 bank groups 4 (lane & 3) + (i ^ f) once each, for any tables and
// operands: conflict-free by construction, so these multiplies take the same LDS cycles for every key and payload.
// Within a halfword, window 4y + u sits at bit 4 (u ^ 1) (the high nibble of a byte is the earlier window).

// lane's base for its lookups in a window-major table at T: T + (y >> 2) * 4096 + (y & 3) * 64 + f * 16 (then ^ i * 16)
__device__ __forceinline__ u32 wtab_lane_base(u32 T, u32 lane)
{
    const u32 y = lane & 7, f = (lane >> 2) & 3;
    return T + (y >> 2) * 4096u + (y & 3) * 64u + f * 16u;
}

// a * (window-major table at tsel) by the G = 8 lanes of a group together (every lane holds a; every lane gets the
// product): gmul_group's work split, conflict-free (above). tsel is a multiple of 64.
__device__ __forceinline__ u32x4 gmul_group_w(const lds_u8 *, u32x4 a, u32 tsel, u32 lane)
{
    static_assert(ENGINE_G == 8, "one halfword per lane");
    const u32 y = lane & 7, f = (lane >> 2) & 3, q = y >> 1;
    const u32 w = q == 0 ? a[0] : q == 1 ? a[1] : q == 2 ? a[2] : a[3];
    const u32 W = wtab_lane_base(tsel, lane), sh = 4u * f + 16u * (y & 1);
    u32x4 e[4];
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
        const u32 n = (w >> (sh ^ (4u * (i ^ 1u)))) & 15u;
        e[i] = lds_load128((n << 8) + (W ^ (i << 4)));
    }
    u32x4 r;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        r[c] = dpp_xor8(xor3(e[0][c], e[1][c], e[2][c]) ^ e[3][c]);
    return r;
}

// ------------------------------------------------------------------------------------------------ GHASH (8-bit Horner)
//
// Whole-record runs of long records (W8 runs, gcm_chunked_kernel) keep H^8 as an 8-bit window-major table of 64 KiB at
// LDS_AES_BYTES: entry (operand byte w, value n) at LDS_AES_BYTES + n * 256 + w * 16, the bank group being the byte
// index. Lane l = lane & 15 takes the operand's byte i ^ l at its i-th lookup (the operand permuted once per multiply:
// dwords by the bits 2-3 of l, bytes within a dword by v_perm with the lane's selector), so the 16 lanes of a
// ds_read_b128 phase read 16 distinct bank groups for any data: 16 conflict-free lookups per multiply instead of 32
// (tools/mb/ghash8.hip: +20.8 % on the engine's step). W8Lane holds the lane's address base B (l in the window bits of
// bytes 0 and 1, byte 2 of the table base) and byte selector; the lookups' address words B ^ (2k, 2k + 1 window bits)
// are formed at each multiply (B made opaque there: kept live through the loop, the eight words spilled the kernel).
//
// W8_SWAP (round 5): the table sits at LDS address 0, so an address is two bytes: byte 0 the window (operand byte
// (i ^ l), times 16), byte 1 the operand's byte value, bytes 2-3 zero (v_perm's constant selector). The window bytes of
// lookups 4c..4c+3 are one register, L_c = L_0 ^ 0x40404040 c (bits 6-7 of ((4c + t) ^ l) << 4 are c ^ (l >> 2)), so
// the 16 addresses cost 16 v_perm and 3 XORs per multiply instead of 16 v_perm and 8 XORs; and the operand's dword swap
// by bit 2 of l and byte permutation by bits 0-1 merge into one two-source v_perm per dword (4 selects and 4 v_perm
// instead of 8 and 4): 9 VALU operations fewer per Horner step.
struct W8Lane {
    u32 base;  // W8_SWAP: L_0, the window bytes of lookups 0..3; else B
    u32 psel;  // byte c <- byte c ^ (l & 3) (W8_SWAP: from the pair's other dword when bit 2 of l is set)
};
__device__ __forceinline__ W8Lane w8_lane(u32 lane)
{
    const u32 l = lane & 15, lb = l & 3;
    // (x * 0x01010101 for a byte x as a v_perm broadcast of byte 0: v_mul_lo_u32 issues at a quarter of the rate)
    auto bcast = [](u32 x) { return __builtin_amdgcn_perm(0u, x, 0u); };
    if constexpr (W8_SWAP)  // byte t of L_0: (t ^ l) << 4 (l < 16: no carries between bytes)
        return W8Lane{(bcast(l) ^ 0x03020100u) << 4, (bcast(lb) ^ 0x03020100u) | bcast(l & 4)};
    return W8Lane{(l << 4) | (l << 12) | ((u32)(LDS_AES_BYTES >> 16) << 16), lb * 0x01010101u ^ 0x03020100u};
}
__device__ __forceinline__ u32x4 gmul8(const lds_u8 *, u32x4 t, u32 lane, W8Lane w)
{
    asm volatile("" : "+v"(w.base));
    if constexpr (W8_SWAP) {
        static_assert(!W8_SWAP || W8_H8_BASE == 0, "the table's address bytes 2-3 are zero");
        u32 L[4];
#pragma unroll
        for (u32 c = 0; c < 4; ++c)
            L[c] = w.base ^ (c * 0x40404040u);
        // p[k] byte c = t byte ((4k + c) ^ l): the dword pair by bit 3 of l (selects), then dword k ^ (bit 2 of l) and
        // the bytes by bits 0-1 in one v_perm of the pair (psel picks from the other dword when bit 2 is set)
        u32 a0, a1, a2, a3;
#if GMUL8_CONST_MASK  // (the W8_SWAP form: the other one reads the lane index)
        // (round 5) the selects by bit 3 of the lane take a constant lane mask (lanes 8-15 of every 16:
        // 0xff00ff00ff00ff00) in VCC instead of a compare of the lane index, which the loop re-derived every step
        // (v_mbcnt x2, v_and, v_cmp: the kernel is short of SGPRs to keep the mask)
        (void)lane;
        asm("s_mov_b32 vcc_lo, 0xff00ff00\n\t"
            "s_mov_b32 vcc_hi, 0xff00ff00\n\t"
            "v_cndmask_b32 %0, %4, %6, vcc\n\t"
            "v_cndmask_b32 %1, %5, %7, vcc\n\t"
            "v_cndmask_b32 %2, %6, %4, vcc\n\t"
            "v_cndmask_b32 %3, %7, %5, vcc"
            : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3)
            : "v"(t[0]), "v"(t[1]), "v"(t[2]), "v"(t[3])
            : "vcc");
#else
        const bool s2 = (lane & 8) != 0;
        a0 = s2 ? t[2] : t[0], a1 = s2 ? t[3] : t[1], a2 = s2 ? t[0] : t[2], a3 = s2 ? t[1] : t[3];
#endif
        u32 p[4] = {__builtin_amdgcn_perm(a1, a0, w.psel), __builtin_amdgcn_perm(a0, a1, w.psel),
                    __builtin_amdgcn_perm(a3, a2, w.psel), __builtin_amdgcn_perm(a2, a3, w.psel)};
        if (CT_PROBE_CONST)
            p[0] = p[1] = p[2] = p[3] = 0;
        u32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (u32 i = 0; i < 16; i += 2) {
            const u32 c = i >> 2, b = i & 3;
            const u32x4 e0 = lds_load128(__builtin_amdgcn_perm(p[c], L[c], 0x0c0c0000u | ((4u + b) << 8) | b));
            const u32x4 e1 = lds_load128(__builtin_amdgcn_perm(p[c], L[c], 0x0c0c0000u | ((5u + b) << 8) | (b + 1)));
#pragma unroll
            for (int k = 0; k < 4; ++k)
                acc[k] = xor3(acc[k], e0[k], e1[k]);
        }
        return acc;
    }
    u32 wreg[8];
#pragma unroll
    for (u32 k = 0; k < 8; ++k)
        wreg[k] = w.base ^ (((2 * k) << 4) | ((2 * k + 1) << 12));
    static_assert(LDS_AES_BYTES == 0x10000, "the table base is byte 2 of the address");
    const u32 l = lane & 15;
    const bool s2 = (l & 8) != 0, s1 = (l & 4) != 0;
    const u32 a0 = s2 ? t[2] : t[0], a1 = s2 ? t[3] : t[1], a2 = s2 ? t[0] : t[2], a3 = s2 ? t[1] : t[3];
    const u32 b[4] = {s1 ? a1 : a0, s1 ? a0 : a1, s1 ? a3 : a2, s1 ? a2 : a3};
    u32 p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        p[k] = __builtin_amdgcn_perm(b[k], b[k], w.psel);  // byte c <- byte c ^ (l & 3)
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (u32 i = 0; i < 16; i += 2) {
        const u32x4 e0 = lds_load128(__builtin_amdgcn_perm(p[i >> 2], wreg[i >> 1], 0x0c020000u | ((4u + (i & 3)) << 8)));
        const u32x4 e1 =
            lds_load128(__builtin_amdgcn_perm(p[i >> 2], wreg[i >> 1], 0x0c020001u | ((4u + ((i + 1) & 3)) << 8)));
#pragma unroll
        for (int c = 0; c < 4; ++c)
            acc[c] = xor3(acc[c], e0[c], e1[c]);
    }
    return acc;
}

// ------------------------------------------------------------------------------------------------ GHASH (multi-key runs)
//
// (round 6) Multi-key whole runs (MK runs, gcm_chunked_kernel EXT 4): the short records of up to MK_SLOTS connections
// share one run, each connection's tables in a 16 KiB slot of the W8 map's [0, 64K): H^4 (the 4-lane Horner power) and H
// (the segment end, w8_lane_end4), both 4-bit window-major (entry (w, n) at T + (w >> 4) * 4096 + n * 256 + (w & 15) *
// 16, T = slot << 14). gmul4w is gmul8's scheme on that 4-bit table: lane l = lane & 15 takes window i ^ l at its i-th
// lookup (i < 32), so the 16 lanes of a ds_read_b128 phase read 16 distinct bank groups (w & 15) for any data and any
// slots (the slot is address bits 14-15): 32 conflict-free lookups per multiply instead of 16, in exchange for a table a
// quarter of the 8-bit one's size. The operand is spread once per multiply into eight "nibble bytes" registers R[c]
// (byte b of R[c] = nibble of window (4c + b) ^ l, with the slot's address bits above it), so a lookup's address is one
// v_perm of R[c] and the window bytes L (gmul8's W8_SWAP form), as in gmul8.
struct MK4Lane {
    u32 s0, s1;  // v_perm selectors of R[2k], R[2k + 1] from (hi_k, lo_k) for this lane's bits 0-2
};
__device__ __forceinline__ MK4Lane mk4_lane(u32 lane)
{
    // byte b of R[2k + r] = (e even ? hi : lo) byte 2 (r ^ l2) + (e >> 1), e = b ^ (l & 3); perm(hi, lo, sel): hi is
    // bytes 4-7, lo bytes 0-3
    const u32 lb = lane & 3, l2 = (lane >> 2) & 1;
    u32 s[2];
#pragma unroll
    for (u32 r = 0; r < 2; ++r) {
        u32 sel = 0;
#pragma unroll
        for (u32 b = 0; b < 4; ++b) {
            const u32 e = b ^ lb, byte = 2u * (r ^ l2) + (e >> 1);
            sel |= ((e & 1u) ? byte : 4u + byte) << (8 * b);
        }
        s[r] = sel;
    }
    return MK4Lane{s[0], s[1]};
}
// t * (the 4-bit window-major table of slot `slot`) for this lane (W8Lane w: the window bytes L_0, W8_SWAP)
__device__ __forceinline__ u32x4 gmul4w(const lds_u8 *, u32x4 t, W8Lane w, MK4Lane m, u32 kslot)
{
    static_assert(W8_SWAP, "the window bytes of gmul8's W8_SWAP form");
    asm volatile("" : "+v"(w.base), "+v"(m.s0), "+v"(m.s1));
    u32 L[4];
#pragma unroll
    for (u32 c = 0; c < 4; ++c)
        L[c] = w.base ^ (c * 0x40404040u);
    // dwords k <- k ^ (bit 3 of the lane), by the constant lane mask of lanes 8-15 of every 16 (gmul8)
    u32 a0, a1, a2, a3;
    asm("s_mov_b32 vcc_lo, 0xff00ff00\n\t"
        "s_mov_b32 vcc_hi, 0xff00ff00\n\t"
        "v_cndmask_b32 %0, %4, %5, vcc\n\t"
        "v_cndmask_b32 %1, %5, %4, vcc\n\t"
        "v_cndmask_b32 %2, %6, %7, vcc\n\t"
        "v_cndmask_b32 %3, %7, %6, vcc"
        : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3)
        : "v"(t[0]), "v"(t[1]), "v"(t[2]), "v"(t[3])
        : "vcc");
    const u32 a[4] = {a0, a1, a2, a3};
    u32 R[8];
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 lo = (a[k] & 0x0f0f0f0fu) | kslot, hi = ((a[k] >> 4) & 0x0f0f0f0fu) | kslot;
        R[2 * k] = __builtin_amdgcn_perm(hi, lo, m.s0);
        R[2 * k + 1] = __builtin_amdgcn_perm(hi, lo, m.s1);
    }
    if (CT_PROBE_CONST)
#pragma unroll
        for (u32 c = 0; c < 8; ++c)
            R[c] = kslot * 0x01010101u;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (u32 i = 0; i < 32; i += 2) {
        const u32 c = i >> 2, b = i & 3, off = c >= 4 ? 4096u : 0u;
        const u32x4 e0 = lds_load128(__builtin_amdgcn_perm(R[c], L[c & 3], 0x0c0c0000u | ((4u + b) << 8) | b) + off);
        const u32x4 e1 = lds_load128(__builtin_amdgcn_perm(R[c], L[c & 3], 0x0c0c0000u | ((5u + b) << 8) | (b + 1)) + off);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            acc[k] = xor3(acc[k], e0[k], e1[k]);
    }
    return acc;
}

// A group's product by the unit combine power (table 8) or another combine element: with SEG_COOP gmul_group_w
// (window-major, conflict-free by construction) in both modes; without it, the constant-time mode gmul_tab (every lane
// the whole product from the same rows of a nibble-major table) and the default mode gmul_group
template <bool CT>
__device__ __forceinline__ u32x4 gmul_combine(const lds_u8 *lds, u32x4 a, u32 tsel, u32 lane)
{
    if constexpr (SEG_COOP)
        return gmul_group_w(lds, a, tsel, lane);
    else if constexpr (CT)
        return gmul_tab(lds, a, tsel);
    else
        return gmul_group(lds, a, tsel, lane % ENGINE_G);
}

// The segment end (gcm_segment, both modes): lane j of a group holds a_j, its partial with its last stream position
// unmultiplied, and owes it the power H^(e_j), e_j = 8 - rank_j (the ranks are the lanes rotated by rot, uniform over the
// group). Returns this lane's share of sum_j a_j H^(e_j - 1) (the caller XOR-reduces the group and multiplies the sum by
// H): the value of rank r moves to lane r (ds_bpermute, only when some group of the wave has rot != 0), an 8 x 8
// transpose of halfwords over the group (three DPP butterfly stages: lane y then holds halfword y of every rank, rank x
// in halfword slot x), and lane y looks up its four windows of ranks 0..6 in the window-major tables H^7..H^1 (slots
// 6..0; rank 7 owes H^0). With the group's product by H (gmul_group_w, 4 lookups) that is 32 conflict-free lookups per
// lane, what the per-lane last multiply read from each lane's own table with data-dependent conflicts, and no lane
// needs the Horner multiply in the segment's last step (gcm_segment skips it).
__device__ __forceinline__ u32 dpp_xor4(u32 v)  // lane ^ 4 within 8 lanes: row_half_mirror (7 - l), then quad_perm [3,2,1,0]
{
    return (u32)__builtin_amdgcn_update_dpp(0, __builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false), 0x1B,
                                            0xF, 0xF, false);
}
__device__ __forceinline__ u32x4 coop_last_powers(const lds_u8 *lds, u32x4 v, u32 lane, u32 rot)
{
    static_assert(ENGINE_G == 8, "halfword transpose over 8 lanes");
    const u32 y = lane & 7;
    if (__any(rot != 0)) {
        const int src = (int)(((lane & ~7u) | ((y + rot) & 7u)) * 4u);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            v[c] = (u32)__builtin_amdgcn_ds_bpermute(src, (int)v[c]);
    }
    u32x4 sum = y == 7 ? v : u32x4{0, 0, 0, 0};  // rank 7: H^0
    u32 d0 = v[0], d1 = v[1], d2 = v[2], d3 = v[3];
    {  // slot bit 2 (dword pairs) with lane ^ 4
        const bool b = (y & 4) != 0;
        const u32 r0 = dpp_xor4(b ? d0 : d2), r1 = dpp_xor4(b ? d1 : d3);
        d0 = b ? r0 : d0, d1 = b ? r1 : d1, d2 = b ? d2 : r0, d3 = b ? d3 : r1;
    }
    {  // slot bit 1 (dword within a pair) with lane ^ 2
        const bool b = (y & 2) != 0;
        const u32 r0 = (u32)__builtin_amdgcn_update_dpp(0, (int)(b ? d0 : d1), 0x4E, 0xF, 0xF, false);
        const u32 r1 = (u32)__builtin_amdgcn_update_dpp(0, (int)(b ? d2 : d3), 0x4E, 0xF, 0xF, false);
        d0 = b ? r0 : d0, d1 = b ? d1 : r0, d2 = b ? r1 : d2, d3 = b ? d3 : r1;
    }
    {  // slot bit 0 (halfword within a dword) with lane ^ 1: the sent halves packed two per dword
        const bool b = (y & 1) != 0;
        const u32 ps = b ? 0x05040100u : 0x07060302u;  // b: send the low halves, else the high ones
        const u32 q0 = (u32)__builtin_amdgcn_update_dpp(0, (int)__builtin_amdgcn_perm(d1, d0, ps), 0xB1, 0xF, 0xF, false);
        const u32 q1 = (u32)__builtin_amdgcn_update_dpp(0, (int)__builtin_amdgcn_perm(d3, d2, ps), 0xB1, 0xF, 0xF, false);
        const u32 ua = b ? 0x03020504u : 0x05040100u, ub = b ? 0x03020706u : 0x07060100u;
        d0 = __builtin_amdgcn_perm(q0, d0, ua), d1 = __builtin_amdgcn_perm(q0, d1, ub);
        d2 = __builtin_amdgcn_perm(q1, d2, ua), d3 = __builtin_amdgcn_perm(q1, d3, ub);
    }
    // per lookup i: the nibble's shift, less 8 so that the nibble lands at bits 8..11 (even slots from the dword moved up
    // by 8 bits: their nibbles sit at bits 0..15), and the lane's window base; opaque to the compiler, which otherwise
    // re-derives them at every lookup (3-4 VALU operations per lookup instead of 2)
    const u32 W = wtab_lane_base(LDS_AES_BYTES, lane), f4 = 4u * ((lane >> 2) & 3);
    u32 Wi[4], she[4], sho[4];
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
        Wi[i] = W ^ (i << 4);
        she[i] = f4 ^ (4u * (i ^ 1u));  // (even slot, dword << 8): shift - 8 + 8
        sho[i] = she[i] + 8u;           // (odd slot): 16 + shift - 8
        asm volatile("" : "+v"(Wi[i]), "+v"(she[i]), "+v"(sho[i]));
    }
    const u32 dw[4] = {d0, d1, d2, d3};
    const u32 dwe[4] = {d0 << 8, d1 << 8, d2 << 8, d3 << 8};
#pragma unroll
    for (u32 x = 0; x < 7; ++x) {
        u32x4 e[4];
#pragma unroll
        for (u32 i = 0; i < 4; ++i) {
            const u32 n8 = ((x & 1) ? dw[x >> 1] >> sho[i] : dwe[x >> 1] >> she[i]) & 0xf00u;
            e[i] = lds_load128((n8 | Wi[i]) + (6u - x) * GHASH_TABLE_BYTES);  // H^(7 - x)
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
            sum[c] = xor3(xor3(sum[c], e[0][c], e[1][c]), e[2][c], e[3][c]);
    }
    return sum;
}

// a * (window-major table at tsel) + sum over the group of x (x: this lane's term, zero in all lanes but one): gmul_group_w
// with x folded into the lane's share before the group's reduction, at no extra instruction
__device__ __forceinline__ u32x4 gmul_group_w_add(const lds_u8 *, u32x4 a, u32 tsel, u32 lane, u32x4 x)
{
    const u32 y = lane & 7, f = (lane >> 2) & 3, q = y >> 1;
    const u32 w = q == 0 ? a[0] : q == 1 ? a[1] : q == 2 ? a[2] : a[3];
    const u32 W = wtab_lane_base(tsel, lane), sh = 4u * f + 16u * (y & 1);
    u32x4 e[4];
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
        const u32 n = (w >> (sh ^ (4u * (i ^ 1u)))) & 15u;
        e[i] = lds_load128((n << 8) + (W ^ (i << 4)));
    }
    u32x4 r;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        r[c] = dpp_xor8(xor3(xor3(e[0][c], e[1][c], e[2][c]), e[3][c], x[c]));
    return r;
}

// ------------------------------------------------------------------------------------------------ GHASH (scattered chains)
//
// A chain of group products (a Horner over the group's ranks, a record's unit combine) needs, for each link, lane y's
// halfword y of the previous product, not the whole product in every lane. gmul_group_w all-reduces each product over
// the 8 lanes (dpp_xor8 of 4 dwords: 12 DPP operations) and each lane then picks its dword (3 selects). Here a link
// reduce-scatters instead (group_scatter: 10 operations; lane y keeps dword y >> 1 of the sum, complete) and extracts
// its nibbles with a bit-field extract and a shift-add onto the opaque per-lane window bases (2 operations a lookup
// instead of 4): ~30 VALU operations a link instead of ~46 (the EXT 4 kernel's segment end: 413 VALU instructions in the code
// object before, round 5). The lookups and tables are gmul_group_w's: conflict-free by construction.
struct GroupWs {
    u32 Wi[4];  // the lane's window base for lookup i (wtab_lane_base ^ i << 4)
    u32 sh[4];  // the bit offset of the lane's nibble for lookup i in its dword: 16 (y & 1) + (4 f ^ 4 (i ^ 1))
};
__device__ __forceinline__ GroupWs group_ws(u32 tsel, u32 lane)
{
    GroupWs k;
    const u32 W = wtab_lane_base(tsel, lane), h16 = 16u * (lane & 1), f4 = 4u * ((lane >> 2) & 3);
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
        k.Wi[i] = W ^ (i << 4);
        k.sh[i] = h16 + (f4 ^ (4u * (i ^ 1u)));
        asm volatile("" : "+v"(k.Wi[i]), "+v"(k.sh[i]));  // (computed once, not re-derived at every lookup)
    }
    return k;
}

// Reduce-scatter of t over the 8 lanes of a group: returns dword (y >> 1) of the XOR of the group's t, complete (both
// halves), in lane y = lane & 7. Three butterfly stages: lane 7 - y (row_half_mirror) exchanges the dword pair the
// other needs, lane y ^ 2 (quad_perm [2,3,0,1]) the dword, lane y ^ 1 (quad_perm [1,0,3,2]) the sum of the last two.
__device__ __forceinline__ u32 group_scatter(u32x4 t, u32 lane)
{
    const bool b = (lane & 4) != 0, c = (lane & 2) != 0;
    const u32 k0 = b ? t[2] : t[0], k1 = b ? t[3] : t[1], s0 = b ? t[0] : t[2], s1 = b ? t[1] : t[3];
    const u32 m0 = k0 ^ (u32)__builtin_amdgcn_update_dpp(0, (int)s0, 0x141, 0xF, 0xF, false);
    const u32 m1 = k1 ^ (u32)__builtin_amdgcn_update_dpp(0, (int)s1, 0x141, 0xF, 0xF, false);
    const u32 kk = c ? m1 : m0, ss = c ? m0 : m1;
    const u32 m = kk ^ (u32)__builtin_amdgcn_update_dpp(0, (int)ss, 0x4E, 0xF, 0xF, false);
    return m ^ (u32)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xF, 0xF, false);
}

// The whole value in every lane of the group from its scattered form (lanes 2q, 2q + 1 hold dword q): each quad's
// lanes 0 and 2 broadcast (quad_perm [0,0,0,0], [2,2,2,2]), the other quad's copies come over row_half_mirror
__device__ __forceinline__ u32x4 group_gather(u32 g, u32 lane)
{
    const u32 a = (u32)__builtin_amdgcn_update_dpp(0, (int)g, 0x00, 0xF, 0xF, false);
    const u32 b = (u32)__builtin_amdgcn_update_dpp(0, (int)g, 0xAA, 0xF, 0xF, false);
    const u32 am = (u32)__builtin_amdgcn_update_dpp(0, (int)a, 0x141, 0xF, 0xF, false);
    const u32 bm = (u32)__builtin_amdgcn_update_dpp(0, (int)b, 0x141, 0xF, 0xF, false);
    const bool hi = (lane & 4) != 0;
    return u32x4{hi ? am : a, hi ? bm : b, hi ? a : am, hi ? b : bm};
}

// the lane's dword (y >> 1) of a value every lane of the group holds
__device__ __forceinline__ u32 group_dword(u32x4 v, u32 lane)
{
    const u32 q = (lane & 7) >> 1;
    return q == 0 ? v[0] : q == 1 ? v[1] : q == 2 ? v[2] : v[3];
}

// the 4 table entries of the lane's windows of a (ga: the lane's dword of a), folded with x (this lane's share of a
// term added to the product: zero in all lanes but one)
__device__ __forceinline__ u32x4 group_ws_terms(u32 ga, const GroupWs &k, u32x4 x)
{
    u32x4 e[4];
#pragma unroll
    for (u32 i = 0; i < 4; ++i)  // (v_bfe_u32 + v_lshl_add_u32: a table base need only be a multiple of 256)
        e[i] = lds_load128((CT_PROBE_CONST ? 0u : __builtin_amdgcn_ubfe(ga, k.sh[i], 4u) << 8) + k.Wi[i]);
    u32x4 t;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        t[c] = xor3(xor3(e[0][c], e[1][c], e[2][c]), e[3][c], x[c]);
    return t;
}

// a link of a scattered chain: the lane's dword of a * T + x
__device__ __forceinline__ u32 gmul_group_ws(const lds_u8 *, u32 ga, const GroupWs &k, u32x4 x, u32 lane)
{
    return group_scatter(group_ws_terms(ga, k, x), lane);
}

// the last link: a * T whole in every lane (all-reduce)
__device__ __forceinline__ u32x4 gmul_group_ws_full(const lds_u8 *, u32 ga, const GroupWs &k)
{
    u32x4 t = group_ws_terms(ga, k, u32x4{0, 0, 0, 0});
#pragma unroll
    for (int c = 0; c < 4; ++c)
        t[c] = dpp_xor8(t[c]);
    return t;
}

#ifndef W8_END_SCATTER
#define W8_END_SCATTER 1  // round 5: the segment end's chain as a scattered chain (gmul_group_ws)
#endif

// The W8 segment end (gcm_segment, W8 runs): lane j of a group holds a_j, its partial with its last stream position
// unmultiplied, owing H^(8 - rank_j). Returns sum_j a_j H^(8 - rank_j) in every lane of the group, as the Horner
// ((v_0 H + v_1) H + ... + v_7) H over the ranks (v_r: the value of the lane of rank r) by eight group multiplies with
// the window-major H table at W8_TAB_H; the lane of rank r folds its value into its share of the r-th product, so the
// values never move between lanes. The W8 map has room for that one table only (the 8-bit H^8 table takes slots
// 0..7), where coop_last_powers needs seven: the lookups are the same 32 per lane, conflict-free, the price is a
// chain of eight dependent products, run scattered (above) since round 5.
__device__ __forceinline__ u32x4 w8_lane_end(const lds_u8 *lds, u32x4 v, u32 lane, u32 rank)
{
    static_assert(ENGINE_G == 8, "a chain over 8 lanes");
    const u32x4 z = {0, 0, 0, 0};
#if W8_END_SCATTER
    const GroupWs k = group_ws(W8_TAB_H, lane);
    u32 g = group_scatter(rank == 0 ? v : z, lane);
#pragma unroll
    for (u32 r = 1; r < 8; ++r)
        g = gmul_group_ws(lds, g, k, rank == r ? v : z, lane);
    return gmul_group_ws_full(lds, g, k);
#else
    u32x4 g;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        g[c] = dpp_xor8(rank == 0 ? v[c] : 0u);
#pragma unroll
    for (u32 r = 1; r < 8; ++r)
        g = gmul_group_w_add(lds, g, W8_TAB_H, lane, rank == r ? v : z);
    return gmul_group_w(lds, g, W8_TAB_H, lane);
#endif
}

// ------------------------------------------------------------------------------------------------ GHASH (4-lane groups)
//
// (round 5) Whole runs of short records in the W8 serial kernel (EXT 4) give each record a group of 4 lanes
// (gcm_segment<..., 4>): a wave then carries 16 records instead of 8, so every per-record instruction (the descriptor and
// segment setup, the first and last steps, the segment end) serves twice as many records, and the segment end is a chain
// of 4 group products instead of 8. The Horner step multiplies by H^4 (the 8-bit table built from H^4). Lane y = lane & 3
// of a group holds dword y of a scattered value and looks up the 8 windows 8y..8y+7 of the window-major table (layout
// above: window w at bit 16 ((w >> 2) & 1) + 4 ((w & 3) ^ 1) of dword w >> 3, i.e. window 8y + t at bit 4 (t ^ 1) of
// dword y), window 8y + (i ^ f) at its i-th lookup with f = (lane >> 1) & 7. The 16 lanes of a ds_read_b128 phase, 4 (g)
// groups x 4 (y) lanes, have distinct (y & 1, f = 2g + (y >> 1)), so they read the bank groups 8 (y & 1) + (i ^ f)
// once each: conflict-free for any data, as gmul_group_w.
struct Group4Ws {
    u32 Wi[8];  // the lane's address base for lookup i (the window's column and bank group)
    u32 sh[8];  // the bit offset of the lane's nibble for lookup i in its dword: 4 ((i ^ f) ^ 1)
};
__device__ __forceinline__ Group4Ws group4_ws(u32 tsel, u32 lane)
{
    Group4Ws k;
    const u32 y = lane & 3, f = (lane >> 1) & 7;
    const u32 B = tsel + (y >> 1) * 4096u + (y & 1) * 128u + f * 16u;  // (tsel a multiple of 256: bits 4-6 are f)
#pragma unroll
    for (u32 i = 0; i < 8; ++i) {
        k.Wi[i] = B ^ (i << 4);
        k.sh[i] = 4u * ((i ^ f) ^ 1u);
        asm volatile("" : "+v"(k.Wi[i]), "+v"(k.sh[i]));  // (computed once per segment end)
    }
    return k;
}
// the 8 table entries of the lane's windows of a (ga: the lane's dword of a), folded with x
__device__ __forceinline__ u32x4 group4_ws_terms(u32 ga, const Group4Ws &k, u32x4 x)
{
    u32x4 t = x;
#pragma unroll
    for (u32 i = 0; i < 8; i += 2) {
        const u32x4 e0 = lds_load128((__builtin_amdgcn_ubfe(ga, k.sh[i], 4u) << 8) + k.Wi[i]);
        const u32x4 e1 = lds_load128((__builtin_amdgcn_ubfe(ga, k.sh[i + 1], 4u) << 8) + k.Wi[i + 1]);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            t[c] = xor3(t[c], e0[c], e1[c]);
    }
    return t;
}
// Reduce-scatter of t over the 4 lanes of a group (a quad): dword y of the XOR in lane y. Lane y ^ 2 (quad_perm
// [2,3,0,1]) takes the dword pair this lane does not keep, then lane y ^ 1 (quad_perm [1,0,3,2]) the other dword.
__device__ __forceinline__ u32 group4_scatter(u32x4 t, u32 lane)
{
    const bool b = (lane & 2) != 0, c = (lane & 1) != 0;
    const u32 k0 = b ? t[2] : t[0], k1 = b ? t[3] : t[1], s0 = b ? t[0] : t[2], s1 = b ? t[1] : t[3];
    const u32 m0 = k0 ^ (u32)__builtin_amdgcn_update_dpp(0, (int)s0, 0x4E, 0xF, 0xF, false);
    const u32 m1 = k1 ^ (u32)__builtin_amdgcn_update_dpp(0, (int)s1, 0x4E, 0xF, 0xF, false);
    const u32 kk = c ? m1 : m0, ss = c ? m0 : m1;
    return kk ^ (u32)__builtin_amdgcn_update_dpp(0, (int)ss, 0xB1, 0xF, 0xF, false);
}
// XOR over the 4 lanes of a group, the whole value in every lane
__device__ __forceinline__ u32x4 group4_allreduce(u32x4 t)
{
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        t[c] ^= (u32)__builtin_amdgcn_update_dpp(0, (int)t[c], 0x4E, 0xF, 0xF, false);
        t[c] ^= (u32)__builtin_amdgcn_update_dpp(0, (int)t[c], 0xB1, 0xF, 0xF, false);
    }
    return t;
}
// The W8 segment end of a 4-lane group: sum_j a_j H^(4 - rank_j) = ((v_0 H + v_1) H + v_2) H + v_3) H over the ranks, a
// scattered chain of four group products with the window-major H table (32 lookups per product, 8 per lane)
__device__ __forceinline__ u32x4 w8_lane_end4(const lds_u8 *, u32x4 v, u32 lane, u32 rank, u32 htab = W8_TAB_H)
{
    const u32x4 z = {0, 0, 0, 0};
    const Group4Ws k = group4_ws(htab, lane);
    u32 g = group4_scatter(rank == 0 ? v : z, lane);
#pragma unroll
    for (u32 r = 1; r < 4; ++r)
        g = group4_scatter(group4_ws_terms(g, k, rank == r ? v : z), lane);
    return group4_allreduce(group4_ws_terms(g, k, z));
}

// The W8 segment end of a long whole record (at least W8_MIN_STEPS steps, the EXT 3 kernel): the same sum by a butterfly over the
// ranks, every lane multiplying by the same nibble-major table (H at W8_TAB_H, H^2 at W8_TAB_COMB, H^4 as two of it):
// level k pairs rank t (bit k clear) with rank t + k as v_t H^k + v_(t+k), each lane taking its partner's product or
// value through the crossbar; then one more xH. 160 lookups per lane (gmul_tab, conflict-free for any data) against the
// serial chain's 32, but three short levels of independent products instead of eight dependent ones: on a record this
// long the chain's latency cost more (-0.7 % on 16 KiB records) than the lookups
__device__ __forceinline__ u32x4 w8_tree_end(const lds_u8 *lds, u32x4 v, u32 lane, u32 rank)
{
    const u32 rot = ((lane & 7u) - rank) & 7u;
#pragma unroll 1
    for (u32 lv = 0; lv < 3; ++lv) {
        const u32 k = 1u << lv;
        u32x4 y = gmul_tab(lds, v, lv == 0 ? (u32)W8_TAB_H : (u32)W8_TAB_COMB);
        if (lv == 2)
            y = gmul_tab(lds, y, W8_TAB_COMB);
        const bool hi = (rank & k) != 0;
        const u32x4 send = hi ? v : y;
        const int src = (int)(((lane & ~7u) | (((rank ^ k) + rot) & 7u)) * 4u);
        u32x4 recv;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            recv[c] = (u32)__builtin_amdgcn_ds_bpermute(src, (int)send[c]);
        v = hi ? (recv ^ v) : (y ^ recv);
    }
    return gmul_tab(lds, v, W8_TAB_H);  // * H
}

#endif  // PTLS_MI355X_ENGINE_GHASH_H
