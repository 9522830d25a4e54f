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

#endif  // PTLS_MI355X_ENGINE_GHASH_H
