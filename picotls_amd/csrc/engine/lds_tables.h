// picotls_amd/csrc/engine/lds_tables.h -- LDS table builders: the replicated AES T-tables and the GHASH 4-bit-window tables.
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_LDS_TABLES_H
#define PTLS_MI355X_ENGINE_LDS_TABLES_H

// ------------------------------------------------------------------------------------------------ LDS tables

#ifndef AES_TTAB_COPY
#define AES_TTAB_COPY 1
#endif
#ifndef AES_TTAB_BATCH
#define AES_TTAB_BATCH 4
#endif

// AES T-table: Te0 replicated into banks 0..31 (bytes 0..127 of row n), Te2 = rotl16(Te0) into bytes 128..255
constexpr u32 aes_ttab_word(const SboxTable &sb, u32 idx)
{
    const u32 s = sb.v[(idx >> 6) & 255];
    const u32 s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
    const u32 te0 = s2 | s << 8 | s << 16 | (s2 ^ s) << 24;
    return (idx & 63) < 32 ? te0 : ((te0 << 16) | (te0 >> 16));
}

// The whole 64 KiB LDS image of the table, derived at compile time into the code object: a launch copies it with
// 16-byte loads (L2 hits after the first workgroup of an XCD) instead of deriving it
struct alignas(16) AesTtabImage {
    u32 v[256 * 64];
};
constexpr AesTtabImage make_aes_ttab()
{
    const SboxTable sb = make_sbox();
    AesTtabImage t = {};
    for (u32 idx = 0; idx < 256 * 64; ++idx)
        t.v[idx] = aes_ttab_word(sb, idx);
    return t;
}
__device__ const AesTtabImage g_aes_ttab = make_aes_ttab();

// Threads [skip, end) build it (end 0: blockDim.x; both multiples of 64; the chunked kernel's other waves scan the first
// run and build the GHASH tables meanwhile), at LDS offset base (0, or 64 KiB in the W8 kernels: W8_SWAP)
__device__ void build_aes_tables(lds_u8 *lds, u32 skip = 0, u32 end = 0, u32 base = 0)
{
    const u32 tid = threadIdx.x - skip, nthr = (end != 0 ? end : blockDim.x) - skip;
#if AES_TTAB_COPY
    const u32x4 *src = (const u32x4 *)g_aes_ttab.v;
    lds_u32x4 *dst = (lds_u32x4 *)(lds + base);
    // every thread's loads are in flight before its first LDS write (AES_TTAB_BATCH of them: one round trip for 512
    // threads or more)
    for (u32 base = 0; base < 256 * 64 / 4; base += AES_TTAB_BATCH * nthr) {
        u32x4 v[AES_TTAB_BATCH];
#pragma unroll
        for (int k = 0; k < AES_TTAB_BATCH; ++k) {
            const u32 idx = base + tid + k * nthr;
            v[k] = idx < 256 * 64 / 4 ? src[idx] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < AES_TTAB_BATCH; ++k) {
            const u32 idx = base + tid + k * nthr;
            if (idx < 256 * 64 / 4)
                dst[idx] = v[k];
        }
    }
#else
    lds_u32 *t = (lds_u32 *)(lds + base);
    // entry n = idx >> 6 is wave-uniform (blockDim.x is a multiple of 64): scalar S-box loads, 16 in flight per batch,
    // so a launch pays one memory latency here instead of one per loop trip (the per-record path is a launch of one)
    for (u32 base = 0; base < 256 * 64; base += 16 * nthr) {
        u32 sv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            sv[k] = c_sbox.v[__builtin_amdgcn_readfirstlane((base + tid + k * nthr) >> 6) & 255u];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const u32 idx = base + tid + k * nthr, slot = idx & 63;
            const u32 s = sv[k];
            const u32 s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
            const u32 te0 = s2 | s << 8 | s << 16 | (s2 ^ s) << 24;
            if (idx < 256 * 64)
                t[idx] = slot < 32 ? te0 : ((te0 << 16) | (te0 >> 16));
        }
    }
#endif
}

// The 16 entries of one window (v: x^(4p)..x^(4p+3) times the element; ec: entry c), entry n at row + n * stride
// (nibble-major 16, window-major 256), written in the order n ^ c
template <bool WL>
__device__ __forceinline__ void store_window(lds_u8 *row, const u32x4 (&v)[4], u32x4 ec, u32 c)
{
    constexpr u32 stride = WL ? 256 : 16;
#pragma unroll
    for (u32 n = 0; n < 16; ++n) {
        u32x4 e = ec;
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if ((n >> (3 - m)) & 1u)
                e ^= v[m];
        *(lds_u32x4 *)(row + (n ^ c) * stride) = e;
    }
}

// GHASH window tables of one key: table t (element key->h[t]), window p (x^(4p)..x^(4p+3)), entry n (4-bit value,
// MSB = coefficient of x^(4p)) = sum over set bits of n of x^(4p+q) * h[t]. Thread (t, p) derives V_0 = x^(4p) h[t]
// with at most three 32-bit steps and one step of 4 (p mod 8) bits, V_1..V_3 by single steps, and writes the window's
// 16 entries. Entries are GF(2)-linear in n, so the XOR combinations are formed after the byte swap back to memory
// order, and entry n ^ c = e(n) ^ e(c): at store n a lane writes slot n ^ (p mod 16), spreading a wave's 16-byte stores
// over the bank groups. A few hundred VALU operations per thread: the build is a small part of a launch of one record.
// Threads [tid0, tid0 + nthr) take part (nthr 0: the whole workgroup).
// ct (the chunked kernel's constant-time mode, CT_COMBINE_TREE): tables 4, 5, 6 hold M^2, M^4, M^8 for the combine
// power M = key->h[src8] (the elements after it in the chain H^8, H^16, ..., H^1024: [7], [9..15]; src8 8 is H^128 = [12])
__device__ __forceinline__ u32 ct_chain_elem(u32 src8, u32 k)
{
    const u32 pos = src8 == 7 ? 0u : src8 == 8 ? 4u : src8 - 8u;
    return 8u + pos + k;
}

// wmask: bit t set = table t window-major (GHASH_WMASK; ghash.h: entry (p, n) at (p >> 4) * 4096 + n * 256 + (p & 15) * 16
// instead of p * 256 + n * 16).
template <typename KeyPtr>  // a KeyEntry in global memory, or its copy staged in LDS (the chunked kernel)
__device__ void build_ghash_tables(lds_u8 *lds, KeyPtr key, u32 ntables = ENGINE_G, u32 src8 = 8, u32 first = 0, u32 tid0 = 0,
                                   u32 nthr = 0, bool ct = false, u32 wmask = 0)
{
    const u32 stride = nthr != 0 ? nthr : blockDim.x;
    for (u32 idx = first * 32 + threadIdx.x - tid0; idx < ntables * 32; idx += stride) {
        const u32 t = idx >> 5, p = idx & 31;
        // table 8: the unit combine power (chunked kernel)
        const u32 el = t == 8 ? src8 : ct && t >= 4 && t <= 6 ? ct_chain_elem(src8, t - 3) : t;
        const auto *h = key->h[el];
        u32 b0 = bswap32(h[0]), b1 = bswap32(h[1]), b2 = bswap32(h[2]), b3 = bswap32(h[3]);
        for (u32 k = 0; k < (p >> 3); ++k)
            gf_mulxs_be(b0, b1, b2, b3, 32);
        if (p & 7)
            gf_mulxs_be(b0, b1, b2, b3, 4 * (p & 7));
        u32x4 v[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            v[m] = u32x4{bswap32(b0), bswap32(b1), bswap32(b2), bswap32(b3)};
            if (m < 3)
                gf_mulxs_be(b0, b1, b2, b3, 1);
        }
        const u32 c = p & 15;
        u32x4 ec = {0, 0, 0, 0};
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if ((c >> (3 - m)) & 1u)
                ec ^= v[m];
        const u32 T = LDS_AES_BYTES + t * GHASH_TABLE_BYTES;
        if ((wmask >> t) & 1u)
            store_window<true>(lds + T + (p >> 4) * 4096 + (p & 15) * 16, v, ec, c);
        else
            store_window<false>(lds + T + p * 256, v, ec, c);
    }
}

// W8 runs (ghash.h): the 8-bit window-major H^8 table at W8_H8_BASE from H^8's 4-bit nibble-major table at `scratch`
// (entry (w, n) = e4(2w, n >> 4) ^ e4(2w + 1, n & 15): byte w of the operand is 4-bit windows 2w and 2w + 1)
// Lane w of a 16-lane phase takes value n = k ^ (w << 4) ^ w (k = i >> 4): its two reads land in bank groups
// (n >> 4) and (n & 15), both distinct across w, and its store in group w (round 4: the plain order n = k read one bank
// group from 16 rows at once, 1.44M conflict cycles per tls16k dispatch).
__device__ __forceinline__ void build_h8_byte_table(lds_u8 *lds, u32 scratch)
{
    for (u32 i = threadIdx.x; i < 4096; i += blockDim.x) {
        const u32 w = i & 15, n = (i >> 4) ^ (w << 4) ^ w;
        const u32x4 e = u32x4(*(const lds_u32x4 *)(lds + scratch + (2 * w) * 256 + (n >> 4) * 16)) ^
                        u32x4(*(const lds_u32x4 *)(lds + scratch + (2 * w + 1) * 256 + (n & 15) * 16));
        *(lds_u32x4 *)(lds + W8_H8_BASE + n * 256 + w * 16) = e;
    }
}

// The 4-bit window table of one GHASH element at LDS offset `base` (a multiple of 256; window-major with wl: a multiple
// of 64), by threads [tid0, tid0 + 32): the same construction as build_ghash_tables for an element given by value.
__device__ __forceinline__ void build_elem_table(lds_u8 *lds, u32 base, u32x4 h, u32 tid0 = 0, bool wl = false)
{
    const u32 p = threadIdx.x - tid0;
    if (p >= 32)
        return;
    u32 b0 = bswap32(h[0]), b1 = bswap32(h[1]), b2 = bswap32(h[2]), b3 = bswap32(h[3]);
    for (u32 k = 0; k < (p >> 3); ++k)
        gf_mulxs_be(b0, b1, b2, b3, 32);
    if (p & 7)
        gf_mulxs_be(b0, b1, b2, b3, 4 * (p & 7));
    u32x4 v[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        v[m] = u32x4{bswap32(b0), bswap32(b1), bswap32(b2), bswap32(b3)};
        if (m < 3)
            gf_mulxs_be(b0, b1, b2, b3, 1);
    }
    const u32 c = p & 15;
    u32x4 ec = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 4; ++m)
        if ((c >> (3 - m)) & 1u)
            ec ^= v[m];
    if (wl)
        store_window<true>(lds + base + (p >> 4) * 4096 + (p & 15) * 16, v, ec, c);
    else
        store_window<false>(lds + base + p * 256, v, ec, c);
}

// (round 6, MK runs) the same window-major table by 128 threads [tid0, tid0 + 128): four per window, each deriving the
// window's elements and storing 4 of its 16 entries (entries n with n >> 2 == the thread's quarter), so that the eight
// tables of a multi-key run take the whole workgroup at once
__device__ __forceinline__ void build_elem_table_w4(lds_u8 *lds, u32 base, u32x4 h, u32 tid0)
{
    // (window p = i mod 32, quarter i / 32: the 16 lanes of a store phase write 16 windows, i.e. 16 distinct bank groups)
    const u32 i = threadIdx.x - tid0, p = i & 31, qt = i >> 5;
    if (i >= 128)
        return;
    u32 b0 = bswap32(h[0]), b1 = bswap32(h[1]), b2 = bswap32(h[2]), b3 = bswap32(h[3]);
    for (u32 k = 0; k < (p >> 3); ++k)
        gf_mulxs_be(b0, b1, b2, b3, 32);
    if (p & 7)
        gf_mulxs_be(b0, b1, b2, b3, 4 * (p & 7));
    u32x4 v[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        v[m] = u32x4{bswap32(b0), bswap32(b1), bswap32(b2), bswap32(b3)};
        if (m < 3)
            gf_mulxs_be(b0, b1, b2, b3, 1);
    }
    lds_u8 *row = lds + base + (p >> 4) * 4096 + (p & 15) * 16;
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 n = 4 * qt + k;
        u32x4 e = {0, 0, 0, 0};
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if ((n >> (3 - m)) & 1u)
                e ^= v[m];
        *(lds_u32x4 *)(row + n * 256) = e;
    }
}

#endif  // PTLS_MI355X_ENGINE_LDS_TABLES_H
