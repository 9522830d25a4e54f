// picotls_amd/csrc/engine/aes_tt.h -- T-table AES rounds from LDS and the counter-mode round cache.
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_AES_TT_H
#define PTLS_MI355X_ENGINE_AES_TT_H

// ------------------------------------------------------------------------------------------------ AES (T-table)

// LDS byte address of Te0[byte r of w] in this lane's bank: byte0 = bank*4 (from laneoff), byte1 = byte r of w, byte2 =
// laneoff's byte 2: the table's 64 KiB slot (0 in most kernels; 1 in the W8 kernels, whose 8-bit GHASH table takes
// [0, 64K), W8_SWAP), at no cost -- the same single v_perm
#if CT_PROBE_CONST  // (diagnosis build only, tools/gpu_r5.sh ct6: every lookup of entry 0; outputs are garbage)
#define TE_ADDR(w, r, laneoff) __builtin_amdgcn_perm(0u, (laneoff), 0x0c020000u | ((4u + (r)) << 8))
#else
#define TE_ADDR(w, r, laneoff) __builtin_amdgcn_perm((w), (laneoff), 0x0c020000u | ((4u + (r)) << 8))
#endif

// LDS is addressed absolutely: the kernels declare no static __shared__ data, so their dynamic region starts at LDS
// address 0 (checked at kernel entry by check_lds_base) and a v_perm result is directly a ds_read address; going
// through the extern array's symbol would cost one v_add per lookup.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wint-to-pointer-cast"
__device__ __forceinline__ u32 lds_load32(u32 addr) { return *(const lds_u32 *)addr; }
__device__ __forceinline__ u32x4 lds_load128(u32 addr) { return *(const lds_u32x4 *)addr; }
#pragma clang diagnostic pop

__device__ __forceinline__ void check_lds_base(const void *smem)
{
    if ((u32)(size_t)(const lds_u8 *)smem != 0)
        __builtin_trap();
}

__device__ __forceinline__ u32 te0(const lds_u8 *, u32 w, int r, u32 laneoff) { return lds_load32(TE_ADDR(w, r, laneoff)); }
__device__ __forceinline__ u32 te2(const lds_u8 *, u32 w, int r, u32 laneoff) { return lds_load32(TE_ADDR(w, r, laneoff) + 128); }

// rounds FIRST .. NR of AES (T-table rounds, then the final SubBytes/ShiftRows/AddRoundKey) on NB independent
// LE-column states; the NB blocks advance in lockstep so each round has 16*NB independent LDS lookups in flight.
template <int NR, int FIRST, int NB>
__device__ __forceinline__ void aes_rounds_n(const lds_u8 *lds, u32 laneoff, const u32 (*rk)[4], u32 (&s)[NB][4])
{
#pragma unroll
    for (int r = FIRST; r < NR; ++r) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const u32 s0 = s[i][0], s1 = s[i][1], s2 = s[i][2], s3 = s[i][3];
            // the round key is stored rotated right by 8 (KeyEntry), so it joins the rotated half: three VALU ops a
            // column (two 3-input XORs and a rotate) instead of four
            s[i][0] = xor3(te0(lds, s0, 0, laneoff), te2(lds, s2, 2, laneoff),
                           rotl8(xor3(te0(lds, s1, 1, laneoff), te2(lds, s3, 3, laneoff), rk[r][0])));
            s[i][1] = xor3(te0(lds, s1, 0, laneoff), te2(lds, s3, 2, laneoff),
                           rotl8(xor3(te0(lds, s2, 1, laneoff), te2(lds, s0, 3, laneoff), rk[r][1])));
            s[i][2] = xor3(te0(lds, s2, 0, laneoff), te2(lds, s0, 2, laneoff),
                           rotl8(xor3(te0(lds, s3, 1, laneoff), te2(lds, s1, 3, laneoff), rk[r][2])));
            s[i][3] = xor3(te0(lds, s3, 0, laneoff), te2(lds, s1, 2, laneoff),
                           rotl8(xor3(te0(lds, s0, 1, laneoff), te2(lds, s2, 3, laneoff), rk[r][3])));
        }
    }
    // last round: SubBytes + ShiftRows + AddRoundKey; S(x) is byte 1/2 of Te0[x] and byte 0/3 of Te2[x]
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        u32 o[4];
#pragma unroll
        for (int col = 0; col < 4; ++col) {
            const u32 a = te2(lds, s[i][col], 0, laneoff);
            const u32 b = te0(lds, s[i][(col + 1) & 3], 1, laneoff);
            const u32 c = te0(lds, s[i][(col + 2) & 3], 2, laneoff);
            const u32 d = te2(lds, s[i][(col + 3) & 3], 3, laneoff);
            const u32 x = __builtin_amdgcn_perm(b, a, 0x0c0c0500u);
            const u32 y = __builtin_amdgcn_perm(d, c, 0x07020c0cu);
            o[col] = __builtin_amdgcn_bitop3_b32(x, y, rk[NR][col], 0x56);  // (x | y) ^ rk
        }
#pragma unroll
        for (int col = 0; col < 4; ++col)
            s[i][col] = o[col];
    }
}

template <int NR>
__device__ __forceinline__ void aes_encrypt_tt(const lds_u8 *lds, u32 laneoff, const u32 (*rk)[4], u32 &s0, u32 &s1, u32 &s2,
                                               u32 &s3)
{
    u32 st[1][4] = {{s0, s1, s2, s3}};
    aes_rounds_n<NR, 1, 1>(lds, laneoff, rk, st);
    s0 = st[0][0], s1 = st[0][1], s2 = st[0][2], s3 = st[0][3];
}

// Counter-mode round caching. Within a window of 256 consecutive counters only the counter's low byte (block byte 15)
// changes, so round 1 has ONE varying lookup (its column 0) and round 2 has four (one per column, all indexed by that
// column); the other 27 lookups of rounds 1-2 fold into five per-window constants: 133 instead of 160 lookups per
// AES-128 block. The cache is keyed per lane by the counter's upper 24 bits and rebuilt when they change (once per 256
// counters; a 1200-byte record never does), so every counter value is covered. Against a two-byte cache (fixed per
// record, 138 lookups, records below 1 MiB only): +2.9 % on 1200-byte records, neutral on 16 KiB and mixed batches.
struct CtrCache1 {
    u32 a0, b0, b1, b2, b3;
};

// n0..n2: nonce words XORed with round key 0; s3: bswap32(ctr) ^ rk[0][3] for any counter of the window (its byte 3,
// the counter's low byte, is not used)
template <int NR>
__device__ __forceinline__ CtrCache1 ctr_cache1_init(const lds_u8 *lds, u32 laneoff, const u32 (*rk)[4], u32 n0, u32 n1, u32 n2,
                                                     u32 s3)
{
    CtrCache1 c;
    // rk[1], rk[2] are stored rotated right by 8 (KeyEntry): they join the rotated half of each column
    c.a0 = xor3(te0(lds, n0, 0, laneoff), te2(lds, n2, 2, laneoff), rotl8(te0(lds, n1, 1, laneoff) ^ rk[1][0]));
    const u32 u1 = xor3(te0(lds, n1, 0, laneoff), te2(lds, s3, 2, laneoff),
                        rotl8(xor3(te0(lds, n2, 1, laneoff), te2(lds, n0, 3, laneoff), rk[1][1])));
    const u32 t2 = xor3(te0(lds, n2, 0, laneoff), te2(lds, n0, 2, laneoff),
                        rotl8(xor3(te0(lds, s3, 1, laneoff), te2(lds, n1, 3, laneoff), rk[1][2])));
    const u32 t3 = xor3(te0(lds, s3, 0, laneoff), te2(lds, n1, 2, laneoff),
                        rotl8(xor3(te0(lds, n0, 1, laneoff), te2(lds, n2, 3, laneoff), rk[1][3])));
    c.b0 = te2(lds, t2, 2, laneoff) ^ rotl8(xor3(te0(lds, u1, 1, laneoff), te2(lds, t3, 3, laneoff), rk[2][0]));
    c.b1 = xor3(te0(lds, u1, 0, laneoff), te2(lds, t3, 2, laneoff), rotl8(te0(lds, t2, 1, laneoff) ^ rk[2][1]));
    c.b2 = te0(lds, t2, 0, laneoff) ^ rotl8(xor3(te0(lds, t3, 1, laneoff), te2(lds, u1, 3, laneoff), rk[2][2]));
    c.b3 = xor3(te0(lds, t3, 0, laneoff), te2(lds, u1, 2, laneoff), rotl8(te2(lds, t2, 3, laneoff) ^ rk[2][3]));
    return c;
}

// AES of one counter block of the cache's window; s[3] holds bswap32(ctr) ^ rk[0][3] on entry (words 0..2 are
// ignored) and s the keystream block on return
template <int NR>
__device__ __forceinline__ void aes_ctr_cached1(const lds_u8 *lds, u32 laneoff, const u32 (*rk)[4], const CtrCache1 &c, u32 (&s)[1][4])
{
    const u32 u0 = c.a0 ^ rotl8(te2(lds, s[0][3], 3, laneoff));
    s[0][0] = c.b0 ^ te0(lds, u0, 0, laneoff);
    s[0][1] = c.b1 ^ rotl8(te2(lds, u0, 3, laneoff));
    s[0][2] = c.b2 ^ te2(lds, u0, 2, laneoff);
    s[0][3] = c.b3 ^ rotl8(te0(lds, u0, 1, laneoff));
    aes_rounds_n<NR, 3, 1>(lds, laneoff, rk, s);
}

#endif  // PTLS_MI355X_ENGINE_AES_TT_H
