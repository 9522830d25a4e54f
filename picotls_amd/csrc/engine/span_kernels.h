// picotls_amd/csrc/engine/span_kernels.h -- One long record over many workgroups (the per-record path's records of
// SPAN_MIN_BYTES and more): gcm_span_kernel + span_combine_kernel.
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
//
// The chunked kernel gives a record to one workgroup, so a lone 4 MiB record ran on one CU (1.7-1.9 ms through
// ptls_aead_encrypt, slower than one x86 core). Here the record's units (16 steps = 128 GHASH stream blocks each,
// counted from the stream's end exactly as in the chunked kernel, so unit k's partial P_k carries H^(128 k) in the
// record's GHASH = sum_k P_k H^(128 k), and P_0 carries E(K, J0)) are dealt in spans of Us = 2^e units to S
// workgroups: span s = units [s Us, (s + 1) Us). Workgroup s seals or opens its units, one per 8-lane group, and
// folds their partials into Q_s = sum_u P_(s Us + u) H^(128 u) (Horner with the H^128 table, as the chunked kernel
// combines a record's units). One more workgroup then evaluates GHASH = sum_s Q_s M^s, M = H^(128 Us), as a binary
// tree: level l pairs neighbours with M^(2^l), whose window table it builds from the element (M itself is e
// squarings of H^128), and writes the tag (seal) or checks it (open).
#ifndef PTLS_MI355X_ENGINE_SPAN_KERNELS_H
#define PTLS_MI355X_ENGINE_SPAN_KERNELS_H

// SPAN_MAX_UNITS (units per span, the LDS partials): common.h
#define SPAN_LDS (LDS_BYTES + GHASH_TABLE_BYTES + 16 * SPAN_MAX_UNITS)  // AES + H^1..H^8 + H^128 tables + partials

// Workgroup s: the units [s * span, min(units, (s + 1) * span)) of the record args.one (key 0 of args.keys), Q_s to
// part[s]. 16-step units; the record's stream is front-padded to whole steps (gcm_segment, not aligned). CT: the
// constant-time variant (gcm_segment's uniform-table last multiply; the span's Horner with gmul_tab, every lane the same
// table rows, instead of the group-cooperative gmul_group whose lanes read different window rows).
template <int NR, bool OPEN, bool CT>
__global__ __launch_bounds__(ENGINE_WG) __attribute__((amdgpu_waves_per_eu(ENGINE_WAVES_PER_SIMD, ENGINE_WAVES_PER_SIMD))) void gcm_span_kernel(BatchArgs args, u32 span, u32 units, u32x4 *part)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    constexpr int G = ENGINE_G;
    lds_u32x4 *s_part = (lds_u32x4 *)(lds + LDS_BYTES + GHASH_TABLE_BYTES);
    const u32 wave = threadIdx.x >> 6;
    // AES tables on waves 0..10, H^1..H^8 and H^128 (slot 8) on waves 11..15
    if (wave >= EARLY_GHASH_WAVE)
        build_ghash_tables(lds, args.keys, 9, 8, 0, EARLY_GHASH_WAVE * 64, ENGINE_WG - EARLY_GHASH_WAVE * 64, false,
                           GHASH_WMASK(CT));
    else
        build_aes_tables(lds, 0, EARLY_GHASH_WAVE * 64);
    __syncthreads();
    const KeyEntry *key = args.keys;
    u32 rk[NR + 1][4];
#pragma unroll
    for (int r = 0; r <= NR; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            rk[r][c] = __builtin_amdgcn_readfirstlane(key->rk[r][c]);
    const u32 iv0 = __builtin_amdgcn_readfirstlane(key->iv[0]), iv1 = __builtin_amdgcn_readfirstlane(key->iv[1]),
              iv2 = __builtin_amdgcn_readfirstlane(key->iv[2]);
    const ptls_mi355x_record_t r = args.one;
    const u32 steps = gcm_steps<OPEN, 0>(r);
    const u32 k0 = blockIdx.x * span, n = min(units - k0, span);
    const u32 tsel_horner = 0x10000u + (u32)(G - 1) * GHASH_TABLE_BYTES, tsel_chunk = 0x10000u + 8u * GHASH_TABLE_BYTES;
    for (u32 uu0 = wave * 8; uu0 < n; uu0 += ENGINE_WG / G) {
        const u32 lane = lane_here(), j = lane % G, uu = uu0 + lane / G, laneoff = (lane & 31) * 4;
        const bool valid = uu < n;
        const u32 k = k0 + uu;
        u32 m_hi = 0, m_lo = 0;
        if (valid) {
            m_hi = steps - k * CHUNK_STEPS;
            m_lo = k + 1 == units ? 0u : m_hi - CHUNK_STEPS;
        }
        u32x4 acc;
        u32 okw;
        gcm_segment<NR, OPEN, 1, 0, CT>(args, lds, rk, iv0, iv1, iv2, r, valid, m_lo, m_hi, j, laneoff, tsel_horner, acc,
                                        false, okw, false, LDS_BYTES + GHASH_TABLE_BYTES + 16u * uu);
        if (valid && j == G - 1)  // (the record's last unit includes E(K, J0), gcm_segment)
            s_part[uu] = acc;
    }
    __syncthreads();
    if (wave == 0) {  // Q_s by Horner from the span's highest unit down (group 0; every lane of it holds the result)
        const u32 lane = lane_here(), j = lane % G;
        if (lane < G) {
            u32x4 g = s_part[n - 1];
            for (u32 i = n - 1; i-- > 0;)
                g = gmul_combine<CT>(lds, g, tsel_chunk, lane) ^ s_part[i];
            if (j == 0)
                part[blockIdx.x] = g;
        }
    }
}

// One workgroup: GHASH = sum_s part[s] M^s with M = (H^CHUNK_BLOCKS)^(2^e), the record's tag: written after the
// ciphertext (seal) or compared with the received one (open, ok[0]). Constant-time as it stands: every product is a
// gmul_tab in which all threads read the same window row of the same table.
static_assert((CHUNK_BLOCKS & (CHUNK_BLOCKS - 1)) == 0 && CHUNK_BLOCKS >= 8 && CHUNK_BLOCKS <= 1024,
              "span_combine_kernel starts M = H^(CHUNK_BLOCKS 2^e) from a power H^(2^m), m <= 10, of the keyset");
template <bool OPEN>
__global__ __launch_bounds__(256) void span_combine_kernel(BatchArgs args, u32 nspans, u32 e, const u32x4 *part)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    lds_u32x4 *s_val = (lds_u32x4 *)(lds + GHASH_TABLE_BYTES);  // the level's values (256)
    lds_u32x4 *s_pow = s_val + 256;                               // the level's multiplier
    const u32 t = threadIdx.x;
    s_val[t] = t < nspans ? part[t] : u32x4{0, 0, 0, 0};
    // M = H^(2^m0), m0 = log2(CHUNK_BLOCKS) + e: the keyset holds H^(2^m) up to m = 10 (H^1024), the rest are squarings
    constexpr u32 CL = __builtin_ctz(CHUNK_BLOCKS);
    const u32 m0 = CL + e, mb = m0 < 10u ? m0 : 10u;
    if (t == 0) {
        const u32 *h = args.keys->h[key_pow2_idx(mb)];
        *s_pow = u32x4{h[0], h[1], h[2], h[3]};
    }
    __syncthreads();
    for (u32 i = mb; i < m0; ++i) {  // the squarings left (a table of the element, then one product)
        build_elem_table(lds, 0, *s_pow);
        __syncthreads();
        const u32x4 sq = gmul_tab(lds, *s_pow, 0);
        __syncthreads();
        if (t == 0)
            *s_pow = sq;
        __syncthreads();
    }
    // tree: v[i] = v[2i] + v[2i+1] * M^(2^l)
    for (u32 cnt = nspans; cnt > 1; cnt = (cnt + 1) / 2) {
        build_elem_table(lds, 0, *s_pow);
        __syncthreads();
        u32x4 v = {0, 0, 0, 0};
        if (t < (cnt + 1) / 2) {
            const u32x4 hi = 2 * t + 1 < cnt ? s_val[2 * t + 1] : u32x4{0, 0, 0, 0};
            v = s_val[2 * t] ^ gmul_tab(lds, hi, 0);
        }
        const u32x4 sq = gmul_tab(lds, *s_pow, 0);  // the next level's multiplier
        __syncthreads();
        if (t < (cnt + 1) / 2)
            s_val[t] = v;
        if (t == 0)
            *s_pow = sq;
        __syncthreads();
    }
    if (t == 0) {
        const ptls_mi355x_record_t r = args.one;
        const u32x4 tag = s_val[0];
        if (OPEN) {
            const u32x4 rt = *(const u32x4_u *)(args.in + r.in_off + r.len);
            const u32x4 d = rt ^ tag;
            args.ok[0] = (d[0] | d[1] | d[2] | d[3]) == 0;
        } else {
            *(u32x4_u *)(args.out + r.out_off + r.len) = tag;
        }
    }
    publish_done(args.done_flag, args.done_token);
}

#endif  // PTLS_MI355X_ENGINE_SPAN_KERNELS_H
