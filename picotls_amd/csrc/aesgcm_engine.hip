// picotls_amd/csrc/aesgcm_engine.hip -- MI355X (gfx950 / CDNA4) AES-GCM record engine: HIP kernels + the C ABI
// declared in include/picotls/mi355x.h.
//
// What it replaces: picotls' fusion AES-GCM engine (lib/fusion.c:401-845 seal/open, :847-929 AES core and key
// schedule, :114-321 + :934-1011 GHASH and H-power tables), re-designed for a GPU: one launch seals or opens a
// whole batch of independent records.
//
// Design (DESIGN.md has the numbers):
//   * one persistent 1024-thread workgroup per CU; G = 8 lanes of a wavefront work on one record, so a wave holds 8
//     records and lane j of a record handles GHASH stream positions j, j+G, j+2G, ... (the stream is
//     [zero padding | AAD blocks | ciphertext blocks | length block], front-padded to a multiple of G, which leaves
//     GHASH unchanged). A record's ciphertext block b sits at one stream position, so the lane that runs AES-CTR
//     on counter 2+b is the lane that folds that block into its GHASH accumulator: no data exchange.
//   * AES: T-table rounds from LDS. Te0 and Te2 (= rotl16 Te0) are replicated into all 32 banks
//     (entry n at n*256 + bank*4, Te2 at +128): lane l always reads bank l%32, so every ds_read_b32 is
//     conflict-free; Te1/Te3 are one v_alignbit away. The byte -> LDS address step is a single v_perm_b32.
//   * GHASH: 4-bit-window tables in LDS. For each H power one table = 32 windows x 16 entries x 16 B (8 KiB);
//     the 16 entries of a window fill exactly one 256-byte LDS bank row, so a ds_read_b128 of 16 lanes never
//     conflicts (equal entries broadcast). A product X*H^k is the XOR of 32 table entries; the reduction is baked
//     into the tables. Horner with stride H^G on every step except the last, where lane j multiplies by H^(G-j)
//     instead; an XOR over the G lanes then gives GHASH. Tables for H^1..H^G (64 KiB) are built on chip from the
//     keyset's H powers at kernel start.
//   * Data path: 16-byte unaligned-capable global loads/stores (unaligned access mode is on for gfx950), G lanes
//     of a record touch G*16 contiguous bytes per step. Partial first/last blocks use byte accesses so nothing
//     outside [in_off, in_off+len) / [out_off, out_off+len+16) is touched.
//
// All word-level state is kept in "LE column" form: a 16-byte block is 4 little-endian u32 words, word c = bytes
// 4c..4c+3 = AES state column c. GHASH elements use the same byte order (byte 0 holds x^0..x^7, MSB first).

#include <hip/hip_runtime.h>
#include <type_traits>
#include <vector>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#include "picotls/mi355x.h"

typedef uint32_t u32;
typedef uint64_t u64;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4_u;
typedef u32 __attribute__((aligned(1))) u32_u;

static_assert(sizeof(ptls_mi355x_record_t) == PTLS_MI355X_RECORD_SIZE, "record descriptor must be 40 bytes");
static_assert(sizeof(ptls_mi355x_cid_t) == 24, "CID descriptor must be 24 bytes");

// ------------------------------------------------------------------------------------------------ constants

namespace {

struct SboxTable {
    uint8_t v[256];
};

constexpr uint8_t xtime_c(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

// FIPS-197 S-box derived at compile time: multiplicative inverse via exp/log tables of generator 3, then the
// affine transform.
constexpr SboxTable make_sbox()
{
    uint8_t exp_t[256] = {}, log_t[256] = {};
    uint8_t x = 1;
    for (int i = 0; i < 255; ++i) {
        exp_t[i] = x;
        log_t[x] = (uint8_t)i;
        x = (uint8_t)(x ^ xtime_c(x));  // x * 3
    }
    SboxTable t = {};
    for (int v = 0; v < 256; ++v) {
        uint8_t inv = v == 0 ? 0 : exp_t[(255 - log_t[v]) % 255];
        uint8_t s = inv;
        for (int k = 1; k <= 4; ++k)
            s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
        t.v[v] = (uint8_t)(s ^ 0x63);
    }
    return t;
}

}  // namespace

__constant__ SboxTable c_sbox = make_sbox();

// one keyset entry in HBM (512 bytes, 16-byte aligned)
struct KeyEntry {
    u32 rk[15][4];  // round keys, LE column words; rounds 1..NR-1 stored rotated right by 8 bits (see aes_rounds_n)
    u32 iv[4];      // static IV as LE words (word 3 = 0)
    u32 h[16][4];   // GHASH elements (LE words): [0..7] = H^1..H^8, [8] = H^CHUNK_BLOCKS, [9..11] = H^16, H^32, H^64
                    // (the combine powers of smaller units), [12..15] = 0
};
static_assert(sizeof(KeyEntry) == 512, "KeyEntry layout");

#ifndef ENGINE_FAST_STEP
#define ENGINE_FAST_STEP 1         // wave-uniform fast path for steps where every lane holds a full text block
#endif

#define ENGINE_G 8                 // lanes per record
#ifndef ENGINE_NB
#define ENGINE_NB 1                // AES-CTR blocks per lane per step (independent chains in flight)
#endif
#ifndef ENGINE_WG
#define ENGINE_WG 1024             // threads per workgroup (one workgroup per CU)
#endif
#define ENGINE_WAVES_PER_SIMD (ENGINE_WG / 256)
#define LDS_AES_BYTES 65536        // Te0/Te2, 32-bank replicated
#define GHASH_TABLE_BYTES 8192     // 32 windows x 16 entries x 16 B
#define LDS_BYTES (LDS_AES_BYTES + ENGINE_G * GHASH_TABLE_BYTES)
#define LDS_ALLOC (LDS_BYTES + 16)  // + scratch word for the key-run scan

// Chunked schedule (many-key batches): records are cut into units of at most CHUNK_BLOCKS GHASH-stream blocks, and
// the per-unit GHASH partials are recombined with H^CHUNK_BLOCKS (one more 8 KiB table, LDS table slot 8).
#ifndef CHUNK_BLOCKS
#define CHUNK_BLOCKS 128  // 2 KiB units: 64K-key mixed +3 %, one-key mixed +7 % over 1 KiB units (interleaved A/B); 256: +1 % / +10 %
#endif
#define CHUNK_STEPS (CHUNK_BLOCKS / ENGINE_G)
#define CHUNK_LOG2 (__builtin_ctz(CHUNK_STEPS))
#ifndef CHUNK_MAX_UNITS
#define CHUNK_MAX_UNITS CRUN_UNITS  // records longer than this many units (> ~2 MiB) use units of a multiple length
#endif
#define BKT_STRIDE (CHUNK_STEPS + 1)             // per-wave front-unit bucket counters in s_ctl (<= 32)
#define CRUN_RECS 256        // records per run (one key)
#ifndef CRUN_UNITS
#define CRUN_UNITS 1024      // units per run
#endif
#define WHOLE_RUN_RECS 4096  // records per run when a one-key run is uniform (every record one unit)
#define UNIFORM_SLACK 2      // a run is uniform when its records' step counts differ by at most this
#define WHOLE_MIN_RECS (ENGINE_WG / ENGINE_G)  // whole-record mode needs at least one record per 8-lane group
#define CLDS_CTL_WORDS ((32 + (CRUN_RECS / 64) * BKT_STRIDE + 127) / 128 * 128)
#define CLDS_CTL (LDS_BYTES + GHASH_TABLE_BYTES)                // CLDS_CTL_WORDS control words
#define CLDS_UBASE (CLDS_CTL + 4 * CLDS_CTL_WORDS)              // u32[CRUN_RECS + 1]: first unit of each record
#define CLDS_DONE (CLDS_UBASE + 4 * (CRUN_RECS + 16))           // u32[CRUN_RECS]: finished units per record
#define CLDS_EK0 (CLDS_DONE + 4 * CRUN_RECS)                    // 16 B per record: E(K, J0)
#define CLDS_PART (CLDS_EK0 + 16 * CRUN_RECS)                   // 16 B per unit: GHASH partial
#define CLDS_FRONT (CLDS_PART + 16 * CRUN_UNITS)                // u32[CRUN_RECS]: records by front-unit size
#define CLDS_ALLOC (CLDS_FRONT + 4 * CRUN_RECS)
static_assert(CLDS_ALLOC <= 160 * 1024, "chunked schedule LDS budget");
static_assert(CHUNK_BLOCKS % ENGINE_G == 0, "units are whole steps");
static_assert((CHUNK_STEPS & (CHUNK_STEPS - 1)) == 0 && CHUNK_STEPS <= 16, "unit lengths are powers of two up to 16 steps");


// ------------------------------------------------------------------------------------------------ small helpers

__device__ __forceinline__ u32 bswap32(u32 x) { return __builtin_bswap32(x); }
__device__ __forceinline__ u32 rotl8(u32 x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ u32 rotr8(u32 x) { return __builtin_amdgcn_alignbit(x, x, 8); }
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// Cross-lane steps on the VALU (DPP) instead of the LDS crossbar (__shfl lowers to ds_bpermute, which competes with the
// table lookups for the LDS): XOR over each aligned group of 8 lanes (quad_perm [1,0,3,2], [2,3,0,1], then
// row_half_mirror pairs the two quads), result in all 8 lanes.
__device__ __forceinline__ u32 dpp_xor8(u32 v)
{
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    return v;
}
// lane 7 of each aligned 8-lane group, to all 8 lanes (quad_perm [3,3,3,3], then row_half_mirror for lanes 0-3)
__device__ __forceinline__ u32 dpp_bcast7(u32 v, u32 lane)
{
    const u32 t = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xFF, 0xF, 0xF, false);
    const u32 u = (u32)__builtin_amdgcn_update_dpp(0, (int)t, 0x141, 0xF, 0xF, false);
    return (lane & 4) ? t : u;
}
// maximum over the wave of a value that is uniform within each 8-lane group
__device__ __forceinline__ u32 wave_max_per8(u32 v)
{
    u32 m = (u32)__builtin_amdgcn_readlane((int)v, 0);
#pragma unroll
    for (int g = 1; g < 8; ++g)
        m = max(m, (u32)__builtin_amdgcn_readlane((int)v, 8 * g));
    return m;
}
// signed maximum / minimum over the wave of a value that is uniform within each 8-lane group
__device__ __forceinline__ int wave_smax_per8(int v)
{
    int m = __builtin_amdgcn_readlane(v, 0);
#pragma unroll
    for (int g = 1; g < 8; ++g)
        m = max(m, __builtin_amdgcn_readlane(v, 8 * g));
    return m;
}
__device__ __forceinline__ int wave_smin_per8(int v)
{
    int m = __builtin_amdgcn_readlane(v, 0);
#pragma unroll
    for (int g = 1; g < 8; ++g)
        m = min(m, __builtin_amdgcn_readlane(v, 8 * g));
    return m;
}

// GF(2^128) * x on a GHASH element held as big-endian words (b0 most significant; bit 127 of the integer is x^0)
__device__ __forceinline__ void gf_mulx_be(u32 &b0, u32 &b1, u32 &b2, u32 &b3)
{
    u32 lsb = b3 & 1;
    b3 = (b3 >> 1) | (b2 << 31);
    b2 = (b2 >> 1) | (b1 << 31);
    b1 = (b1 >> 1) | (b0 << 31);
    b0 = (b0 >> 1) ^ (lsb ? 0xe1000000u : 0u);
}

// ------------------------------------------------------------------------------------------------ keyset setup

// x = x * y in GF(2^128), big-endian words (SP 800-38D Algorithm 1); setup only
__device__ void gf_mul_be(u32 (&x)[4], const u32 (&y)[4])
{
    u32 z0 = 0, z1 = 0, z2 = 0, z3 = 0, v0 = y[0], v1 = y[1], v2 = y[2], v3 = y[3];
    for (int b = 0; b < 128; ++b) {
        if ((x[b >> 5] >> (31 - (b & 31))) & 1)
            z0 ^= v0, z1 ^= v1, z2 ^= v2, z3 ^= v3;
        gf_mulx_be(v0, v1, v2, v3);
    }
    x[0] = z0, x[1] = z1, x[2] = z2, x[3] = z3;
}

__device__ __forceinline__ u32 sub_word(u32 w)
{
    return (u32)c_sbox.v[w & 0xff] | (u32)c_sbox.v[(w >> 8) & 0xff] << 8 | (u32)c_sbox.v[(w >> 16) & 0xff] << 16 |
           (u32)c_sbox.v[w >> 24] << 24;
}

__device__ __forceinline__ u32 xtime_w(u32 w) { return ((w & 0x7f7f7f7fu) << 1) ^ (((w >> 7) & 0x01010101u) * 0x1bu); }

// plain word-level AES (setup only: H = E_K(0^128))
__device__ void aes_plain(const u32 (*rk)[4], int nr, u32 s[4])
{
    for (int c = 0; c < 4; ++c)
        s[c] ^= rk[0][c];
    for (int r = 1; r <= nr; ++r) {
        u32 t[4];
        for (int c = 0; c < 4; ++c)
            t[c] = sub_word(s[c]);
        for (int c = 0; c < 4; ++c)
            s[c] = (t[c] & 0xff) | (t[(c + 1) & 3] & 0xff00) | (t[(c + 2) & 3] & 0xff0000) | (t[(c + 3) & 3] & 0xff000000);
        if (r != nr) {
            for (int c = 0; c < 4; ++c) {
                u32 w = s[c], r1 = (w >> 8) | (w << 24), r2 = (w >> 16) | (w << 16), r3 = (w >> 24) | (w << 8);
                s[c] = xtime_w(w ^ r1) ^ r1 ^ r2 ^ r3;
            }
        }
        for (int c = 0; c < 4; ++c)
            s[c] ^= rk[r][c];
    }
}

// one thread per key: FIPS-197 key expansion, H = E_K(0), H^1..H^16, static IV
// (slot: entry i goes to out[slot[i]] when slot != nullptr: a rekey of some connections of a keyset)
__global__ void keyset_setup_kernel(const uint8_t *__restrict__ keys, const uint8_t *__restrict__ ivs, KeyEntry *__restrict__ out,
                                    u32 nkeys, u32 key_size, const u32 *__restrict__ slot = nullptr)
{
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkeys)
        return;
    const int nk = (int)key_size / 4, nr = nk + 6;
    u32 w[60];
    const uint8_t *k = keys + (size_t)i * key_size;
    for (int j = 0; j < nk; ++j)
        w[j] = (u32)k[4 * j] | (u32)k[4 * j + 1] << 8 | (u32)k[4 * j + 2] << 16 | (u32)k[4 * j + 3] << 24;
    u32 rcon = 1;
    for (int j = nk; j < 4 * (nr + 1); ++j) {
        u32 t = w[j - 1];
        if (j % nk == 0) {
            t = sub_word((t >> 8) | (t << 24)) ^ rcon;
            rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0)) & 0xff;
        } else if (nk > 6 && j % nk == 4) {
            t = sub_word(t);
        }
        w[j] = w[j - nk] ^ t;
    }
    KeyEntry *e = out + (slot != nullptr ? slot[i] : i);
    u32 rk[15][4];
    for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 4; ++c)
            rk[r][c] = r <= nr ? w[4 * r + c] : 0;
    for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 4; ++c)
            e->rk[r][c] = r >= 1 && r < nr ? rotr8(rk[r][c]) : rk[r][c];
    const uint8_t *v = ivs + (size_t)i * 12;
    for (int c = 0; c < 3; ++c)
        e->iv[c] = (u32)v[4 * c] | (u32)v[4 * c + 1] << 8 | (u32)v[4 * c + 2] << 16 | (u32)v[4 * c + 3] << 24;
    e->iv[3] = 0;

    u32 s[4] = {0, 0, 0, 0};
    aes_plain(rk, nr, s);
    // H as big-endian words for the bitwise multiply (SP 800-38D Algorithm 1)
    const u32 h0 = bswap32(s[0]), h1 = bswap32(s[1]), h2 = bswap32(s[2]), h3 = bswap32(s[3]);
    const u32 hb[4] = {h0, h1, h2, h3};
    u32 p[4] = {h0, h1, h2, h3};  // current power, big-endian words
    for (int n = 1; n <= (CHUNK_BLOCKS > 64 ? CHUNK_BLOCKS : 64); ++n) {
        if (n <= 8)
            for (int c = 0; c < 4; ++c)
                e->h[n - 1][c] = bswap32(p[c]);
        if (n == CHUNK_BLOCKS || n == 16 || n == 32 || n == 64) {
            const int slot = n == CHUNK_BLOCKS ? 8 : n == 16 ? 9 : n == 32 ? 10 : 11;
            for (int c = 0; c < 4; ++c)
                e->h[slot][c] = bswap32(p[c]);
        }
        gf_mul_be(p, hb);
    }
    for (int n = 12; n < 16; ++n)
        for (int c = 0; c < 4; ++c)
            e->h[n][c] = 0;
}

// ------------------------------------------------------------------------------------------------ LDS tables

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) u32 lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

// AES T-table: Te0 replicated into banks 0..31 (bytes 0..127 of row n), Te2 = rotl16(Te0) into bytes 128..255
__device__ void build_aes_tables(lds_u8 *lds)
{
    lds_u32 *t = (lds_u32 *)lds;
    // entry n = idx >> 6 is wave-uniform (blockDim.x is a multiple of 64): scalar S-box loads, 16 in flight per batch,
    // so a launch pays one memory latency here instead of one per loop trip (the per-record path is a launch of one)
    for (u32 base = 0; base < 256 * 64; base += 16 * blockDim.x) {
        u32 sv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            sv[k] = c_sbox.v[__builtin_amdgcn_readfirstlane((base + threadIdx.x + k * blockDim.x) >> 6) & 255u];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const u32 idx = base + threadIdx.x + k * blockDim.x, slot = idx & 63;
            const u32 s = sv[k];
            const u32 s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
            const u32 te0 = s2 | s << 8 | s << 16 | (s2 ^ s) << 24;
            if (idx < 256 * 64)
                t[idx] = slot < 32 ? te0 : ((te0 << 16) | (te0 >> 16));
        }
    }
}

// (b0..b3) *= x^s in GF(2^128), big-endian words (GCM bit order: the MSB of b0 is x^0), 1 <= s <= 32, in closed form:
// bit i of the s bits shifted out of b3 is x^(127 - i) and comes back as x^(s - 1 - i) * (1 + x + x^2 + x^7), i.e. the
// shifted-out bits land at the top of b0 ("1") and again 1, 2 and 7 bits further down, the last spilling into b1
__device__ __forceinline__ void gf_mulxs_be(u32 &b0, u32 &b1, u32 &b2, u32 &b3, u32 s)
{
    const u32 top = s == 32 ? b3 : b3 << (32 - s);
    if (s == 32) {
        b3 = b2, b2 = b1, b1 = b0, b0 = 0;
    } else {
        b3 = __builtin_amdgcn_alignbit(b2, b3, s);
        b2 = __builtin_amdgcn_alignbit(b1, b2, s);
        b1 = __builtin_amdgcn_alignbit(b0, b1, s);
        b0 >>= s;
    }
    const u64 v = (u64)top << 32;
    const u64 r = v ^ (v >> 1) ^ (v >> 2) ^ (v >> 7);
    b0 ^= (u32)(r >> 32);
    b1 ^= (u32)r;
}

// GHASH window tables of one key: table t (element key->h[t]), window p (x^(4p)..x^(4p+3)), entry n (4-bit value,
// MSB = coefficient of x^(4p)) = sum over set bits of n of x^(4p+q) * h[t]. Thread (t, p) derives V_0 = x^(4p) h[t]
// with at most three 32-bit steps and one step of 4 (p mod 8) bits, V_1..V_3 by single steps, and writes the window's
// 16 entries. Entries are GF(2)-linear in n, so the XOR combinations are formed after the byte swap back to memory
// order, and entry n ^ c = e(n) ^ e(c): at store n a lane writes slot n ^ (p mod 16), spreading a wave's 16-byte stores
// over the bank groups. A few hundred VALU operations per thread: the build is a small part of a launch of one record.
__device__ void build_ghash_tables(lds_u8 *lds, const KeyEntry *__restrict__ key, u32 ntables = ENGINE_G, u32 src8 = 8)
{
    for (u32 idx = threadIdx.x; idx < ntables * 32; idx += blockDim.x) {
        const u32 t = idx >> 5, p = idx & 31;
        const u32 *h = key->h[t == 8 ? src8 : t];  // table 8: the unit combine power (chunked kernel)
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
        lds_u32x4 *row = (lds_u32x4 *)(lds + LDS_AES_BYTES + t * GHASH_TABLE_BYTES + p * 256);
#pragma unroll
        for (u32 n = 0; n < 16; ++n) {
            u32x4 e = ec;
#pragma unroll
            for (int m = 0; m < 4; ++m)
                if ((n >> (3 - m)) & 1u)
                    e ^= v[m];
            row[n ^ c] = e;
        }
    }
}

// ------------------------------------------------------------------------------------------------ AES (T-table)

// LDS byte address of Te0[byte r of w] in this lane's bank: byte0 = bank*4 (from laneoff), byte1 = byte r of w.
#define TE_ADDR(w, r, laneoff) __builtin_amdgcn_perm((w), (laneoff), 0x0c0c0000u | ((4u + (r)) << 8))

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

// ------------------------------------------------------------------------------------------------ byte-exact I/O

// zero bytes n..15
__device__ __forceinline__ u32x4 mask_tail(u32x4 v, u32 n)
{
    u32x4 r;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        int nb = (int)n - 4 * c;
        u32 m = nb >= 4 ? 0xffffffffu : nb <= 0 ? 0u : (0xffffffffu >> (32 - 8 * nb));
        r[c] = v[c] & m;
    }
    return r;
}

// loads n (< 16) bytes, zero padded. As fusion's loadn128 (lib/fusion.c:355-368): when the 16 bytes at p stay inside
// p's 4 KiB page (which holds valid data, so it is mapped) one unaligned 16-byte load plus a mask replaces n byte loads;
// only a tail within 15 bytes of a page end is read byte by byte. Bytes past n are never used. n = 0 reads nothing (p
// may then be one past the end of a buffer).
__device__ __forceinline__ u32x4 load_partial(const uint8_t *p, u32 n)
{
    if (n != 0 && ((uintptr_t)p & 4095u) <= 4096u - 16u)
        return mask_tail(*(const u32x4_u *)p, n);
    u32x4 v = {0, 0, 0, 0};
#pragma unroll
    for (u32 i = 0; i < 15; ++i)
        if (i < n)
            v[i >> 2] |= (u32)p[i] << (8 * (i & 3));
    return v;
}

__device__ __forceinline__ void store_partial(uint8_t *p, u32x4 v, u32 n)
{
    for (u32 i = 0; i < n; ++i)
        p[i] = (uint8_t)(v[i >> 2] >> (8 * (i & 3)));
}

// ------------------------------------------------------------------------------------------------ main kernel

struct BatchArgs {
    const KeyEntry *keys;
    const ptls_mi355x_record_t *recs;
    u64 nrecs;
    const uint8_t *in;
    const uint8_t *aad;
    uint8_t *out;
    uint8_t *ok;
    u32 multi_key;  // 0: every record uses key 0 (no key-run scan)
    u32 nkeys;      // records whose key_idx >= nkeys are skipped (open: ok = 0)
    u32 unit_log2;  // chunked kernel: units of 2^unit_log2 steps (<= CHUNK_STEPS; smaller for a launch of one record)
    // chunked kernel, ungrouped many-key batches (key_*_kernel): when *perm_on != 0 the kernel walks `grouped` (the
    // descriptors in key order) and perm[i] is the batch index of grouped[i] (for the ok bytes)
    const ptls_mi355x_record_t *grouped;
    const u32 *perm;
    const u32 *perm_on;
};

#define RUN_SCAN_CAP 256  // records examined per key-run scan (multi-key batches)

// TLS 1.3 record framing (FRAME = 1; lib/picotls.c:719-749, :770-817, :5952-5974). Seal: the GCM plaintext is the
// record's len payload bytes plus the inner content type (flags & 0xff); the wire record at out_off is the 5-byte
// header {23, 3, 3, BE16(len + 17)} (also the AAD), the ciphertext, the tag. Open: the wire record at in_off is header
// (the AAD, as received), len ciphertext bytes (inner type and padding included), tag; the plaintext goes to out_off.
//
// TLS 1.2 AES-GCM record framing (FRAME = 2; buffer_push_encrypted_records lib/picotls.c:779-799, handle_input_tls12
// :6019-6060, build_tls12_aad :753-762). The wire record is header {type, 3, 3, BE16(8 + len + 16)} || explicit nonce
// (8 bytes, big endian: the record IV, tls12.record_iv_size) || ciphertext || tag. GCM nonce = static IV ^ (0^32 ||
// explicit nonce), i.e. ptls_aead_encrypt(..., seq = record IV), and the 13-byte AAD is BE64(seq) || type || 3 || 3 ||
// BE16(len) with seq the record sequence number. Seal: in_off holds the explicit nonce followed by the len payload
// bytes; the type is flags & 0xff. Open: the wire record is at in_off; the AAD takes the header's type.
#define TLS_HEADER_SIZE 5
#define TLS12_RECORD_IV_SIZE 8
#define TLS12_AAD_SIZE 13
template <bool OPEN, int FRAME>
__device__ __forceinline__ u32 gcm_text_len(const ptls_mi355x_record_t &r)
{
    return FRAME == 1 && !OPEN ? r.len + 1 : r.len;
}
template <bool OPEN, int FRAME>
__device__ __forceinline__ u32 gcm_aad_len(const ptls_mi355x_record_t &r)
{
    return FRAME == 1 ? (u32)TLS_HEADER_SIZE : FRAME == 2 ? (u32)TLS12_AAD_SIZE : (u32)r.aad_len;
}
// bytes in front of the GCM text in the input / output record
template <bool OPEN, int FRAME>
__device__ __forceinline__ constexpr u32 frame_in_skip()
{
    return FRAME == 1 ? (OPEN ? TLS_HEADER_SIZE : 0) : FRAME == 2 ? (OPEN ? TLS_HEADER_SIZE : 0) + TLS12_RECORD_IV_SIZE : 0;
}
template <bool OPEN, int FRAME>
__device__ __forceinline__ constexpr u32 frame_out_skip()
{
    return FRAME && !OPEN ? TLS_HEADER_SIZE + (FRAME == 2 ? TLS12_RECORD_IV_SIZE : 0) : 0;
}
// G-lane steps of a record's GHASH stream [pad | AAD | text | length]
template <bool OPEN, int FRAME>
__device__ __forceinline__ u32 gcm_steps(const ptls_mi355x_record_t &r)
{
    return (((gcm_aad_len<OPEN, FRAME>(r) + 15u) >> 4) + ((gcm_text_len<OPEN, FRAME>(r) + 15u) >> 4) + 1 + ENGINE_G - 1) /
           ENGINE_G;
}

// GHASH/CTR work of one G-lane group on steps [m_lo, m_hi) of record r's stream (see file header): lane j owns stream
// positions j + G*m and runs them NB at a time. The NB AES-CTR blocks of a step are independent (NB x 16 LDS lookups
// per round in flight); their GHASH folds stay sequential (Horner with H^G, the segment's last step with H^(G-j)).
// On return every lane of the group holds the segment's GHASH partial sum(X_i * H^(end - i)) and the length lane
// (lane G-1, when the segment holds the length block) holds E(K, J0) in ek0. Invalid groups pass m_lo == m_hi.
template <int NR, bool OPEN, int NB, int FRAME = 0>
__device__ __forceinline__ void gcm_segment(const BatchArgs &args, const lds_u8 *lds, const u32 (&rk)[NR + 1][4], u32 iv0,
                                            u32 iv1, u32 iv2, const ptls_mi355x_record_t &r, bool valid, u32 m_lo,
                                            u32 m_hi, u32 j, u32 laneoff, u32 tsel_horner, u32 tsel_last, u32x4 &acc,
                                            u32x4 &ek0, bool finish, u64 rec)
{
    constexpr int G = ENGINE_G;
    constexpr bool SEAL_FRAME = FRAME == 1 && !OPEN, OPEN_FRAME = FRAME == 1 && OPEN, TLS12 = FRAME == 2;
    const u32 L = gcm_text_len<OPEN, FRAME>(r), A = gcm_aad_len<OPEN, FRAME>(r);
    // bytes of text readable at src (a framed seal reads len payload bytes; its last text byte is the content type)
    const u32 Lsrc = SEAL_FRAME ? L - 1 : L;
    const u32 na = (A + 15) >> 4, nb = (L + 15) >> 4;
    const u32 total = na + nb + 1;
    const u32 K = (total + G - 1) / G;
    const int P = (int)(K * G) - (int)total;

    const u32 Smax = wave_max_per8(m_hi - m_lo);  // m_lo, m_hi are uniform within a group

    // nonce = iv ^ (0^32 || BE64(seq)) (lib/picotls.c:6587-6601); TLS 1.2 takes the explicit nonce of the record in
    // place of seq, read as stored (big endian), so its two words need no swap
    u32 nw1 = bswap32((u32)(r.seq >> 32)), nw2 = bswap32((u32)r.seq);
    if (TLS12) {
        const uint8_t *e = args.in + r.in_off + (OPEN ? TLS_HEADER_SIZE : 0);
        nw1 = *(const u32_u *)e;
        nw2 = *(const u32_u *)(e + 4);
    }
    const u32 n0 = iv0 ^ rk[0][0];
    const u32 n1 = iv1 ^ nw1 ^ rk[0][1];
    const u32 n2 = iv2 ^ nw2 ^ rk[0][2];
    const uint8_t *src = args.in + r.in_off + frame_in_skip<OPEN, FRAME>();
    uint8_t *dst = args.out + r.out_off + frame_out_skip<OPEN, FRAME>();
    const uint8_t *aadp = OPEN_FRAME ? args.in + r.in_off : args.aad + r.aad_off;

    acc = u32x4{0, 0, 0, 0};
    ek0 = u32x4{0, 0, 0, 0};

    static_assert(NB == 1, "the counter cache runs one block per lane and step");
    CtrCache1 cc1 = {};
    u32 cc1_key = 0xffffffffu;  // counter >> 8 of the cached window (none yet)

    // data block of lane j at step m: b = j + G*m - P - na; a full 16-byte input block is loaded one step ahead, so
    // its HBM latency hides under the AES of the current step
    auto full_block = [&](u32 m, int &b) -> bool {
        b = (int)(j + G * m) - P - (int)na;
        return m < m_hi && b >= 0 && b < (int)nb && Lsrc - 16u * (u32)b >= 16;
    };
    u32x4 nxt[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        int b;
        nxt[i] = u32x4{0, 0, 0, 0};
        if (full_block(m_lo + i, b))
            nxt[i] = *(const u32x4_u *)(src + 16u * (u32)b);
    }

    // step m, part 1: the next step's input prefetch and this step's counter block (refreshing the counter cache when
    // the lane enters a new 256-counter window)
    u32x4 cur;
    auto setup_step = [&](u32 m0, u32 (&st)[1][4]) {
        cur = nxt[0];
        int bn;
        if (full_block(m0 + 1, bn))
            nxt[0] = *(const u32x4_u *)(src + 16u * (u32)bn);
        // AES-CTR input: data positions encrypt counter 2+b, all others J0 (kept by the length lane as E(K, J0))
        const int logical = (int)(j + G * m0) - P;
        const int b = logical - (int)na;
        const bool is_data = m0 < m_hi && logical >= (int)na && b < (int)nb;
        st[0][0] = n0, st[0][1] = n1, st[0][2] = n2;
        const u32 ctr = is_data ? (u32)(b + 2) : 1u;
        st[0][3] = bswap32(ctr) ^ rk[0][3];
        if ((ctr >> 8) != cc1_key) {  // entering a new 256-counter window (divergent; skipped when no lane does)
            cc1 = ctr_cache1_init<NR>(lds, laneoff, rk, n0, n1, n2, st[0][3]);
            cc1_key = ctr >> 8;
        }
    };
    // step m, part 2: with the keystream block ks, write the output and return the GHASH input block X of position
    // j + G*m
    auto finish_step = [&](u32 m, const u32x4 &ks) -> u32x4 {
        const bool act = m < m_hi;
        const int logical = (int)(j + G * m) - P;
        const int b = logical - (int)na;
        const bool is_data = act && logical >= (int)na && b < (int)nb;
        const bool is_aad = act && logical >= 0 && logical < (int)na;
        const bool is_len = act && logical == (int)(na + nb);
        u32x4 X = {0, 0, 0, 0};
#if ENGINE_FAST_STEP
        // steady state: every active lane of the wave holds a full 16-byte text block (one uniform branch, no
        // per-case dispatch)
        const bool full = is_data && Lsrc - 16u * (u32)b >= 16;
        if (__all(!act || full)) {
            const u32x4 o = cur ^ ks;
            if (act)
                *(u32x4_u *)(dst + 16u * (u32)b) = o;
            return OPEN ? cur : o;
        }
#endif
        if (is_data) {
            const u32 rem = L - 16u * (u32)b;
            uint8_t *op = dst + 16u * (u32)b;
            if (rem >= 16 && (!SEAL_FRAME || Lsrc - 16u * (u32)b >= 16)) {
                const u32x4 v = cur;
                const u32x4 o = v ^ ks;
                *(u32x4_u *)op = o;
                X = OPEN ? v : o;
            } else {
                const u32 srem = Lsrc - 16u * (u32)b;
                u32x4 v = load_partial(src + 16u * (u32)b, srem);
                if (SEAL_FRAME)  // the inner content type follows the payload
                    v[srem >> 2] |= (u32)(r.flags & 0xffu) << (8 * (srem & 3));
                const u32x4 o = rem >= 16 ? v ^ ks : mask_tail(v ^ ks, rem);
                if (rem >= 16)
                    *(u32x4_u *)op = o;
                else
                    store_partial(op, o, rem);
                X = OPEN ? v : o;
            }
        } else if (is_aad) {
            if (SEAL_FRAME) {  // the record header: built here, written to the wire, and authenticated
                const u32 wl = L + 16;
                X = u32x4{0x00030317u | ((wl >> 8) & 0xffu) << 24, wl & 0xffu, 0, 0};
                store_partial(args.out + r.out_off, X, TLS_HEADER_SIZE);
            } else if (TLS12) {  // AAD = BE64(seq) || type || 3 || 3 || BE16(len) (build_tls12_aad)
                const u32 type = OPEN ? (u32)args.in[r.in_off] : (r.flags & 0xffu);
                X = u32x4{bswap32((u32)(r.seq >> 32)), bswap32((u32)r.seq), type | 0x030300u | ((L >> 8) & 0xffu) << 24,
                          L & 0xffu};
                if (!OPEN) {  // the wire header and the explicit nonce
                    const u32 wl = TLS12_RECORD_IV_SIZE + L + 16;
                    const u32x4 h = {type | 0x030300u | ((wl >> 8) & 0xffu) << 24, (wl & 0xffu) | nw1 << 8,
                                     nw1 >> 24 | nw2 << 8, nw2 >> 24};
                    store_partial(args.out + r.out_off, h, TLS_HEADER_SIZE + TLS12_RECORD_IV_SIZE);
                }
            } else {
                const u32 rem = A - 16u * (u32)logical;
                const uint8_t *ap = aadp + 16u * (u32)logical;
                X = rem >= 16 ? *(const u32x4_u *)ap : load_partial(ap, rem);
            }
        } else if (is_len) {
            const u64 abits = (u64)A * 8, cbits = (u64)L * 8;
            X[0] = bswap32((u32)(abits >> 32));
            X[1] = bswap32((u32)abits);
            X[2] = bswap32((u32)(cbits >> 32));
            X[3] = bswap32((u32)cbits);
            ek0 = ks;
        }
        return X;
    };

    // Steady state: the steps [sa, sb) (relative to m_lo, wave-uniform) in which every lane of every group of the wave
    // holds a full text block, the next step's block is full too (the prefetch needs no check) and no group is at its
    // segment's last step (Horner with H^G throughout). They run without the per-lane position logic: the counter,
    // source and destination just advance by one step, about 30 VALU operations fewer per block.
    const int D0 = P + (int)na;         // stream position of text block 0
    const int nbf = (int)(Lsrc >> 4);   // full text blocks
    const int ms = (D0 + G - 1) / G;    // first step whose 8 positions are all >= D0
    const int me = nbf + D0 >= G ? (nbf + D0 - G) / G : -1;  // last step whose 8 positions are all full text
    int sa = max(ms, (int)m_lo) - (int)m_lo;
    int sb = min(me - 1, (int)m_hi - 2) + 1 - (int)m_lo;
    if (!valid || m_hi <= m_lo)
        sa = 1, sb = 0;
    sa = wave_smax_per8(sa);
    sb = wave_smin_per8(sb);

    for (u32 s0 = 0; s0 < Smax; ++s0) {
        if ((int)s0 == sa && sb > sa) {
            const int b0 = (int)(j + G * (m_lo + (u32)sa)) - D0;  // this lane's text block at step sa
            u32 off = 16u * (u32)b0;                               // its byte offset in the text
            u32 ctr = (u32)b0 + 2;
            for (int s = sa; s < sb; ++s) {
                cur = nxt[0];
                nxt[0] = *(const u32x4_u *)(src + off + 16 * G);
                u32 st[1][4] = {{n0, n1, n2, bswap32(ctr) ^ rk[0][3]}};
                if ((ctr >> 8) != cc1_key) {
                    cc1 = ctr_cache1_init<NR>(lds, laneoff, rk, n0, n1, n2, st[0][3]);
                    cc1_key = ctr >> 8;
                }
                aes_ctr_cached1<NR>(lds, laneoff, rk, cc1, st);
                __builtin_amdgcn_sched_barrier(0);
                const u32x4 o = cur ^ u32x4{st[0][0], st[0][1], st[0][2], st[0][3]};
                *(u32x4_u *)(dst + off) = o;
                __builtin_amdgcn_sched_barrier(0);
                acc = gmul_tab(lds, acc ^ (OPEN ? cur : o), tsel_horner);
                __builtin_amdgcn_sched_barrier(0);
                ctr += G;
                off += 16 * G;
            }
            s0 = (u32)sb;
        }
        const u32 m0 = m_lo + s0;
        u32 st[1][4];
        setup_step(m0, st);
        aes_ctr_cached1<NR>(lds, laneoff, rk, cc1, st);
        __builtin_amdgcn_sched_barrier(0);
        const u32x4 X = finish_step(m0, u32x4{st[0][0], st[0][1], st[0][2], st[0][3]});
        // scheduling fence: keeps the 32 table loads of this fold from being hoisted next to the other work (that
        // hoisting spills them to scratch)
        __builtin_amdgcn_sched_barrier(0);
        const u32x4 prod = gmul_tab(lds, acc ^ X, m0 + 1 == m_hi ? tsel_last : tsel_horner);
        if (m0 < m_hi)
            acc = prod;
        __builtin_amdgcn_sched_barrier(0);
    }

    // XOR over the G lanes of the group
    static_assert(G == 8, "dpp_xor8 reduces groups of 8 lanes");
#pragma unroll
    for (int c = 0; c < 4; ++c)
        acc[c] = dpp_xor8(acc[c]);
    // whole record (finish): tag = GHASH ^ E(K, J0), written after the ciphertext (seal) or compared with the
    // received one (open)
    if (finish && valid && j == G - 1) {
        const u32x4 tag = acc ^ ek0;
        if (OPEN) {
            const u32x4 rt = *(const u32x4_u *)(src + L);
            const u32x4 d = rt ^ tag;
            args.ok[rec] = (d[0] | d[1] | d[2] | d[3]) == 0;
        } else {
            *(u32x4_u *)(dst + L) = tag;
        }
    }
}

// Unit length multiplier of a record of `steps` steps: 1, or for a record that would need more than CHUNK_MAX_UNITS units
// of 2^log2 steps the least factor that fits it in CHUNK_MAX_UNITS (its partials are then combined with the unit power
// applied mul times). Records up to PTLS_MI355X_MAX_RECORD_LEN thus always spread over the workgroup.
__device__ __forceinline__ u32 unit_mul(u32 steps, u32 log2)
{
    const u32 nc = (steps + (1u << log2) - 1) >> log2;
    return nc > CHUNK_MAX_UNITS ? (nc + CHUNK_MAX_UNITS - 1) / CHUNK_MAX_UNITS : 1u;
}

// Descriptors whose len exceeds PTLS_MI355X_MAX_RECORD_LEN or whose key_idx is not below the keyset size are rejected
// as a whole: nothing is written for them and an open reports ok = 0, so a corrupt length cannot make the kernel address
// memory far past the record's offsets. (Multi-key batches also reject invalid keys per key run, before any table build.)
__device__ __forceinline__ bool record_ok(const BatchArgs &args, const ptls_mi355x_record_t &r)
{
    return r.len <= PTLS_MI355X_MAX_RECORD_LEN && r.key_idx < args.nkeys;
}

// Seals / opens one whole record per G-lane group.
template <int NR, bool OPEN, int NB>
__device__ __forceinline__ void process_group(const BatchArgs &args, const lds_u8 *lds, const u32 (&rk)[NR + 1][4], u32 iv0,
                                              u32 iv1, u32 iv2, u64 rec, bool valid, u32 j, u32 laneoff, u32 tsel_horner,
                                              u32 tsel_last)
{
    constexpr int G = ENGINE_G;
    ptls_mi355x_record_t r = {};
    if (valid)
        r = args.recs[rec];
    if (valid && !record_ok(args, r)) {
        if (OPEN && j == 0)
            args.ok[rec] = 0;
        valid = false;
    }
    const u32 K = valid ? gcm_steps<OPEN, 0>(r) : 0;
    u32x4 acc, ek0;
    gcm_segment<NR, OPEN, NB>(args, lds, rk, iv0, iv1, iv2, r, valid, 0, K, j, laneoff, tsel_horner, tsel_last, acc, ek0,
                              true, rec);
}

// Persistent kernel: workgroup w owns the contiguous record range [n*w/grid, n*(w+1)/grid) and walks it in key runs
// (maximal stretches of equal key_idx, at most RUN_SCAN_CAP records); the GHASH tables in LDS are rebuilt only when
// the key changes, so a single-key batch builds them once and a key-sorted many-connection batch once per key.
// ENGINE_WG threads and 128+ KiB of LDS per workgroup: exactly one workgroup (ENGINE_WG/256 waves per SIMD) per CU, so
// the register allocator may use the whole per-wave budget instead of chasing an occupancy the LDS budget rules out.
template <int NR, bool OPEN>
__global__ __launch_bounds__(ENGINE_WG) __attribute__((amdgpu_waves_per_eu(ENGINE_WAVES_PER_SIMD, ENGINE_WAVES_PER_SIMD))) void gcm_batch_kernel(BatchArgs args)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    lds_u32 *s_run = (lds_u32 *)(lds + LDS_BYTES);  // scratch word after the tables
    check_lds_base(smem);
    constexpr int G = ENGINE_G;
    constexpr int RPW = 64 / G;  // records per wave-iteration

    build_aes_tables(lds);

    const u32 lane = threadIdx.x & 63;
    const u32 j = lane % G;
    const u32 slot = lane / G;
    const u32 laneoff = (lane & 31) * 4;
    const u32 wave = threadIdx.x >> 6;
    const u32 waves_per_wg = blockDim.x >> 6;
    const u32 tsel_horner = 0x10000u + (u32)(G - 1) * GHASH_TABLE_BYTES;
    const u32 tsel_last = 0x10000u + (u32)(G - 1 - j) * GHASH_TABLE_BYTES;

    const u64 n = args.nrecs;
    const u64 beg = n * blockIdx.x / gridDim.x, end = n * (blockIdx.x + 1) / gridDim.x;
    u32 loaded_key = 0xffffffffu;

    for (u64 pos = beg; pos < end;) {
        const u32 key_idx = args.multi_key ? args.recs[pos].key_idx : 0u;
        u64 run_end = end;
        if (args.multi_key) {
            const u64 lim = min(end, pos + RUN_SCAN_CAP);
            if (threadIdx.x == 0)
                *s_run = (u32)(lim - pos);
            __syncthreads();
            for (u64 t = pos + threadIdx.x; t < lim; t += blockDim.x)
                if (args.recs[t].key_idx != key_idx)
                    atomicMin((u32 *)s_run, (u32)(t - pos));
            __syncthreads();
            run_end = pos + *s_run;
            __syncthreads();
        }
        if (key_idx >= args.nkeys) {  // invalid key: nothing is written except a failed ok byte
            if (OPEN)
                for (u64 t = pos + threadIdx.x; t < run_end; t += blockDim.x)
                    args.ok[t] = 0;
            pos = run_end;
            continue;
        }
        if (key_idx != loaded_key) {
            __syncthreads();  // no wave still reads the previous key's tables
            build_ghash_tables(lds, args.keys + key_idx);
            __syncthreads();
            loaded_key = key_idx;
        }
        const KeyEntry *key = args.keys + key_idx;
        // round keys and IV are workgroup-uniform: pin them in SGPRs
        u32 rk[NR + 1][4];
#pragma unroll
        for (int r = 0; r <= NR; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                rk[r][c] = __builtin_amdgcn_readfirstlane(key->rk[r][c]);
        const u32 iv0 = __builtin_amdgcn_readfirstlane(key->iv[0]), iv1 = __builtin_amdgcn_readfirstlane(key->iv[1]),
                  iv2 = __builtin_amdgcn_readfirstlane(key->iv[2]);

        const u64 ngroups = (run_end - pos + RPW - 1) / RPW;
        for (u64 grp = wave; grp < ngroups; grp += waves_per_wg) {
            const u64 rec = pos + grp * RPW + slot;
            process_group<NR, OPEN, ENGINE_NB>(args, lds, rk, iv0, iv1, iv2, rec, rec < run_end, j, laneoff, tsel_horner, tsel_last);
        }
        pos = run_end;
    }
}

// Diagnostic build only (-DENGINE_PROFILE=1): s_memtime stamps of the chunked kernel's phases, summed over runs and
// workgroups: [0] run setup, [1] GHASH table build, [2] unit loop, [3] kernel prologue (AES tables), [4] wave idle at the unit-loop barrier,
// [5] units, [6] runs, [7] table builds.
#ifndef ENGINE_PROFILE
#define ENGINE_PROFILE 0
#endif
#if ENGINE_PROFILE
__device__ unsigned long long g_prof[8];
__device__ __forceinline__ unsigned long long stamp()
{
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define PROF_STAMP(v) const unsigned long long v = stamp()
#define PROF_ADD(i, x) atomicAdd(&g_prof[i], (unsigned long long)(x))
#else
#define PROF_STAMP(v)
#define PROF_ADD(i, x)
#endif

// Chunked schedule for many-key / mixed-length batches. The lockstep kernel above gives each G-lane group a whole
// record, so a wave runs as long as its longest record and a key run (~64 records of a connection) as long as its
// longest record too; with U[64 B, 16 KiB] lengths and a workgroup barrier per key that halves throughput twice.
// Here a run's records are cut into units of at most CHUNK_BLOCKS GHASH-stream blocks, counted from the END of the
// stream (so every unit but a record's first is exactly CHUNK_BLOCKS long), and waves pull units from a per-run LDS
// counter. A unit's group computes the partial P_k = sum over its blocks of X_i * H^(end_k - i) (k = units after it);
// GHASH = sum_k P_k * H^(k * CHUNK_BLOCKS). The group that completes a record's last outstanding unit (LDS counter per
// record) evaluates that sum by Horner with the H^CHUNK_BLOCKS table and finishes the tag, inside the unit loop.
// Single-unit records finish inside their unit as in the lockstep kernel.
template <int NR, bool OPEN, int FRAME>
__global__ __launch_bounds__(ENGINE_WG) __attribute__((amdgpu_waves_per_eu(ENGINE_WAVES_PER_SIMD, ENGINE_WAVES_PER_SIMD))) void gcm_chunked_kernel(BatchArgs args)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    PROF_STAMP(tk);
    // s_ctl: [1] next unit, [4..7] per-wave unit totals, [8..11] per-wave key boundary, [12..15] per-wave unit cut,
    // [16..19] / [20..23] per-wave min / max steps, [32 + 16 w + b] per-wave count of front-unit bucket b
    lds_u32 *s_front = (lds_u32 *)(lds + CLDS_FRONT);
    lds_u32 *s_ctl = (lds_u32 *)(lds + CLDS_CTL);
    lds_u32 *s_ubase = (lds_u32 *)(lds + CLDS_UBASE);
    lds_u32 *s_done = (lds_u32 *)(lds + CLDS_DONE);
    lds_u32x4 *s_ek0 = (lds_u32x4 *)(lds + CLDS_EK0);
    lds_u32x4 *s_part = (lds_u32x4 *)(lds + CLDS_PART);
    constexpr int G = ENGINE_G;
    constexpr int RPW = 64 / G;
    constexpr u32 SCAN_WAVES = CRUN_RECS / 64;

    const u32 lane = threadIdx.x & 63;
    const u32 j = lane % G;
    const u32 slot = lane / G;
    const u32 laneoff = (lane & 31) * 4;
    const u32 wave = threadIdx.x >> 6;
    const u32 tsel_horner = 0x10000u + (u32)(G - 1) * GHASH_TABLE_BYTES;
    const u32 tsel_last = 0x10000u + (u32)(G - 1 - j) * GHASH_TABLE_BYTES;
    const u32 tsel_chunk = 0x10000u + 8u * GHASH_TABLE_BYTES;
    // unit length in steps (a power of two <= CHUNK_STEPS) and the key element of its combine power H^(G * ustep)
    const u32 ustep = 1u << args.unit_log2;
    const u32 usrc = ustep == CHUNK_STEPS ? 8u : args.unit_log2 == 0 ? 7u : 8u + args.unit_log2;

    const u64 n = args.nrecs;
    const u64 beg = n * blockIdx.x / gridDim.x, end = n * (blockIdx.x + 1) / gridDim.x;
    u32 loaded_key = 0xffffffffu;
    // the descriptors in batch order, or (an ungrouped many-key batch) the key-grouped copy built on the device; ok
    // bytes go to the record's batch index either way
    const ptls_mi355x_record_t *recs = args.recs;
    const u32 *perm = nullptr;
    if (args.perm_on != nullptr && *args.perm_on)
        recs = args.grouped, perm = args.perm;
    auto ok_at = [&](u64 i) -> u64 { return perm != nullptr ? (u64)perm[i] : i; };

    build_aes_tables(lds);

    for (u64 pos = beg; pos < end;) {
        PROF_STAMP(t0);
        // ---- the run: records [pos, pos + run_n) with one key, at most CRUN_RECS records and CRUN_UNITS units.
        // Threads 0..CRUN_RECS-1 read one descriptor each: the key boundary and the unit counts come from one pass.
        const u32 key_idx = args.multi_key ? recs[pos].key_idx : 0u;
        const u32 lim = (u32)min(end - pos, (u64)CRUN_RECS);
        u32 nc = 0, incl = 0, bkt = 0;
        if (wave < SCAN_WAVES) {
            const u32 t = threadIdx.x;
            bool other_key = false;
            u32 smin = 0xffffffffu, smax = 0;
            if (t < lim) {
                ptls_mi355x_record_t r = recs[pos + t];
                if (!record_ok(args, r))  // rejected: one empty unit (see the unit loop)
                    r.len = 0, r.aad_len = 0;
                const u32 steps = gcm_steps<OPEN, FRAME>(r);
                // front-unit size bucket: 0 = a record too long for CHUNK_MAX_UNITS units (it takes units of a
                // multiple length, unit_mul), else ustep + 1 - size of the record's first unit (1 = a full unit, ustep =
                // one step)
                const u32 mul = unit_mul(steps, args.unit_log2);
                nc = (steps + ustep - 1) >> args.unit_log2;
                if (mul > 1)  // rare: the only division
                    nc = (steps + mul * ustep - 1) / (mul * ustep);
                bkt = mul > 1 ? 0u : ustep + 1 - (steps - (nc - 1) * ustep);
                other_key = args.multi_key && r.key_idx != key_idx;
                if (!other_key)
                    smin = smax = steps;
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                smin = min(smin, (u32)__shfl_xor((int)smin, off, 64));
                smax = max(smax, (u32)__shfl_xor((int)smax, off, 64));
            }
            const u64 kb = __ballot(other_key || t >= lim);
            incl = nc;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const u32 y = (u32)__shfl_up((int)incl, off, 64);
                if (lane >= (u32)off)
                    incl += y;
            }
            if (lane == 63) {
                s_ctl[4 + wave] = incl;
                s_ctl[8 + wave] = kb ? 64 * wave + (u32)__builtin_ctzll(kb) : 0xffffffffu;
                s_ctl[16 + wave] = smin;
                s_ctl[20 + wave] = smax;
            }
            s_done[t] = 0;
            if (t == 0)
                s_ctl[1] = 0;
        }
        __syncthreads();
        u32 run_n = lim, smin = 0xffffffffu, smax = 0;
#pragma unroll
        for (u32 w = 0; w < SCAN_WAVES; ++w) {
            run_n = min(run_n, s_ctl[8 + w]);
            smin = min(smin, s_ctl[16 + w]);
            smax = max(smax, s_ctl[20 + w]);
        }
        // uniform run: every record is one unit (no partials), and a one-key batch may take a much longer run. A
        // workgroup with fewer records left than it has groups cuts them into units instead, so that a small batch
        // (the per-record picotls path is a batch of one) spreads over the workgroup's waves.
        const bool whole = smax <= smin + UNIFORM_SLACK && end - pos >= WHOLE_MIN_RECS;
        if (whole && !args.multi_key)
            run_n = (u32)min(end - pos, (u64)WHOLE_RUN_RECS);
        if (!whole && wave < SCAN_WAVES) {
            for (u32 w = 0; w < wave; ++w)
                incl += s_ctl[4 + w];
            s_ubase[threadIdx.x + 1] = incl;
            if (threadIdx.x == 0)
                s_ubase[0] = 0;
            // the first record whose units overflow the run's partial slots ends the run (never the first record)
            const u64 cut = __ballot(incl > CRUN_UNITS);
            if (lane == 0)
                s_ctl[12 + wave] = cut ? 64 * wave + (u32)__builtin_ctzll(cut) : 0xffffffffu;
        }
        u32 nhuge = 0;
        if (!whole) {
            __syncthreads();
#pragma unroll
            for (u32 w = 0; w < SCAN_WAVES; ++w)
                run_n = min(run_n, max(s_ctl[12 + w], 1u));
            // Unit order: [front units of very long records][all full units, record-major][the other front units by
            // size, largest first]. Lockstep waves then draw units of equal or similar length, and the run ends on
            // its shortest units. Counting sort of the front units by bucket: per-wave counts, then positions.
            u32 rank = 0;
            if (wave < SCAN_WAVES) {
                const bool in = threadIdx.x < run_n;
#pragma unroll
                for (u32 b = 0; b <= CHUNK_STEPS; ++b) {
                    const u64 m = __ballot(in && bkt == b);
                    if (lane == 0)
                        s_ctl[32 + BKT_STRIDE * wave + b] = (u32)__popcll(m);
                    if (in && bkt == b)
                        rank = (u32)__popcll(m & ((1ull << lane) - 1));
                }
            }
            __syncthreads();
            if (wave < SCAN_WAVES) {
                // lane b: first slot of this wave's bucket-b records = all records of earlier buckets (prefix over
                // lanes) + bucket b of earlier waves; a record then takes lane bkt's value (no serial walk)
                u32 tot = 0, mine = 0;
#pragma unroll
                for (u32 w = 0; w < SCAN_WAVES; ++w) {
                    const u32 c = lane < BKT_STRIDE ? s_ctl[32 + BKT_STRIDE * w + lane] : 0u;
                    tot += c;
                    mine += w < wave ? c : 0u;
                }
                u32 before = tot;
#pragma unroll
                for (int off = 1; off < 32; off <<= 1) {
                    const u32 y = (u32)__shfl_up((int)before, off, 64);
                    if (lane >= (u32)off)
                        before += y;
                }
                const u32 first_slot = before - tot + mine;
                const u32 base = (u32)__shfl((int)first_slot, (int)bkt, 64);
                if (threadIdx.x < run_n)
                    s_front[base + rank] = threadIdx.x;
            }
#pragma unroll
            for (u32 w = 0; w < SCAN_WAVES; ++w)
                nhuge += s_ctl[32 + BKT_STRIDE * w];
            __syncthreads();
        }
        const u32 total_units = whole ? run_n : s_ubase[run_n];
        const u32 nfull = total_units - run_n;
        const u64 run_end = pos + run_n;
        PROF_STAMP(t1);

        if (key_idx >= args.nkeys) {  // invalid key: nothing is written except a failed ok byte
            if (OPEN)
                for (u64 t = pos + threadIdx.x; t < run_end; t += blockDim.x)
                    args.ok[ok_at(t)] = 0;
            __syncthreads();
            pos = run_end;
            continue;
        }
        if (key_idx != loaded_key) {
            build_ghash_tables(lds, args.keys + key_idx, 9, usrc);  // H^1..H^8 and the unit combine power
            __syncthreads();
            loaded_key = key_idx;
            if (threadIdx.x == 0)
                PROF_ADD(7, 1);
        }
        PROF_STAMP(t2);
        const KeyEntry *key = args.keys + key_idx;
        u32 rk[NR + 1][4];
#pragma unroll
        for (int r = 0; r <= NR; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                rk[r][c] = __builtin_amdgcn_readfirstlane(key->rk[r][c]);
        const u32 iv0 = __builtin_amdgcn_readfirstlane(key->iv[0]), iv1 = __builtin_amdgcn_readfirstlane(key->iv[1]),
                  iv2 = __builtin_amdgcn_readfirstlane(key->iv[2]);

        // ---- units: each wave takes RPW consecutive units (one per group) at a time
        for (;;) {
            u32 ub = 0;
            if (lane == 0)
                ub = atomicAdd((u32 *)&s_ctl[1], (u32)RPW);
            ub = __builtin_amdgcn_readfirstlane(ub);
            if (ub >= total_units)
                break;
            const u32 u = ub + slot;
            const bool valid = u < total_units;
            u32 lo = u, first = u, unc = 1, k_back = 0;
            if (!whole && valid) {
                if (u < nhuge || u >= nhuge + nfull) {  // a front unit
                    lo = s_front[u < nhuge ? u : u - nfull];
                    first = s_ubase[lo];
                    unc = s_ubase[lo + 1] - first;
                    k_back = unc - 1;
                } else {  // full unit f: record lo with s_ubase[lo] - lo <= f < s_ubase[lo + 1] - (lo + 1)
                    const u32 f = u - nhuge;
                    u32 hi = run_n;
                    lo = 0;
                    while (hi - lo > 1) {
                        const u32 mid = (lo + hi) >> 1;
                        if (s_ubase[mid] - mid <= f)
                            lo = mid;
                        else
                            hi = mid;
                    }
                    first = s_ubase[lo];
                    unc = s_ubase[lo + 1] - first;
                    k_back = f - (first - lo);
                }
            }
            const u32 ri = lo;
            ptls_mi355x_record_t r = {};
            if (valid)
                r = recs[pos + ri];
            const u64 rid = OPEN && valid ? ok_at(pos + ri) : pos + ri;  // the record's batch index (ok byte)
            const bool live = valid && record_ok(args, r);
            if (valid && !live) {  // rejected descriptor: the scan gave it one unit; nothing is written
                r.len = 0, r.aad_len = 0;
                if (OPEN && j == 0)
                    args.ok[rid] = 0;
            }
            const u32 steps = gcm_steps<OPEN, FRAME>(r);
            // unit [m_lo, m_hi) of the record's steps (whole mode: the record); huge records take longer units
            const u32 mul = whole ? 1u : unit_mul(steps, args.unit_log2);
            u32 m_hi = steps, m_lo = 0;
            if (!whole) {
                const u32 ulen = mul * ustep;
                m_hi = steps - k_back * ulen;
                m_lo = k_back + 1 == unc ? 0u : m_hi - ulen;
            }
            if (!live)
                m_lo = m_hi = 0;
            u32x4 acc, ek0;
            gcm_segment<NR, OPEN, 1, FRAME>(args, lds, rk, iv0, iv1, iv2, r, live, m_lo, m_hi, j, laneoff, tsel_horner,
                                     tsel_last, acc, ek0, unc == 1, rid);
            if (live && unc > 1) {  // uniform over the group
                u32 last = 0;
                if (j == G - 1) {
                    s_part[first + unc - 1 - k_back] = acc;  // stream order: the front unit first
                    if (k_back == 0)
                        s_ek0[ri] = ek0;
                    __threadfence_block();  // partial and E(K, J0) land before the count that publishes them
                    last = atomicAdd((u32 *)&s_done[ri], 1u) == unc - 1;
                }
                last = dpp_bcast7(last, lane);
                if (last) {
                    // last unit of the record: GHASH = Horner over the partials with H^(G * ulen) = (H^(G * ustep))^mul
                    // (whole group)
                    u32x4 g = s_part[first];
                    for (u32 i = 1; i < unc; ++i) {
                        g = gmul_group(lds, g, tsel_chunk, j);
                        for (u32 t = 1; t < mul; ++t)  // huge records only
                            g = gmul_group(lds, g, tsel_chunk, j);
                        g ^= s_part[first + i];
                    }
                    const u32x4 tag = g ^ s_ek0[ri];
                    if (j != G - 1) {
                    } else if (OPEN) {
                        const u32x4 rt = *(const u32x4_u *)(args.in + r.in_off + frame_in_skip<OPEN, FRAME>() +
                                                            gcm_text_len<OPEN, FRAME>(r));
                        const u32x4 d = rt ^ tag;
                        args.ok[rid] = (d[0] | d[1] | d[2] | d[3]) == 0;
                    } else {
                        *(u32x4_u *)(args.out + r.out_off + frame_out_skip<OPEN, FRAME>() + gcm_text_len<OPEN, FRAME>(r)) = tag;
                    }
                }
            }
        }
        PROF_STAMP(tw);
        __syncthreads();  // the run's tables, partials and counters are free again
        PROF_STAMP(t3);
#if ENGINE_PROFILE
        if (lane == 0)
            PROF_ADD(4, t3 - tw);
        if (threadIdx.x == 0) {
            PROF_ADD(0, t1 - t0);
            PROF_ADD(1, t2 - t1);
            PROF_ADD(2, t3 - t2);
            PROF_ADD(5, total_units);
            PROF_ADD(6, 1);
            if (pos == beg)
                PROF_ADD(3, t0 - tk);
        }
#endif
        pos = run_end;
    }
}

// ------------------------------------------------------------------------------------------------ key grouping
// A many-key batch whose records are not grouped by connection would give the chunked kernel one-record key runs, each
// with its own table build and barrier (15 GiB/s on 4M records over 64K keys in random order against 724 grouped).
// Small kernels group it on the device first: the number of key changes between neighbours (regroup when runs would
// average under 8 records; a grouped batch stops here), key counts, their exclusive scan, and a scatter of record
// indices into key order. The chunked kernel then walks the permutation; descriptors, outputs and ok bytes stay
// at each record's own index, so the results are those of the batch order. ctl[0] = key changes, ctl[1] = regroup.
#define KEY_GROUP_MAX_KEYS (1u << 20)

// ctl[0]: key changes between neighbouring records (a wave sum per atomic)
__global__ __launch_bounds__(256) void key_changes_kernel(const ptls_mi355x_record_t *recs, u64 n, u32 *ctl)
{
    u32 changes = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += (u64)gridDim.x * blockDim.x)
        changes += recs[i - 1].key_idx != recs[i].key_idx;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
        changes += (u32)__shfl_xor((int)changes, off, 64);
    if ((threadIdx.x & 63) == 0 && changes != 0)
        atomicAdd(&ctl[0], changes);
}

__device__ __forceinline__ bool key_regroup(const u32 *ctl, u64 n) { return (u64)ctl[0] * 8 > n; }

// key counts (only when regrouping): each thread counts a contiguous stretch of records and adds one count per key run
__global__ __launch_bounds__(256) void key_hist_kernel(const ptls_mi355x_record_t *recs, u64 n, u32 nkeys, u32 *cnt, const u32 *ctl)
{
    if (!key_regroup(ctl, n))
        return;
    const u64 nthr = (u64)gridDim.x * blockDim.x, t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 per = (n + nthr - 1) / nthr, i0 = min(n, t * per), i1 = min(n, i0 + per);
    u32 run_key = 0xffffffffu, run_len = 0;
    for (u64 i = i0; i < i1; ++i) {
        u32 k = recs[i].key_idx;
        k = k < nkeys ? k : nkeys;  // out-of-range keys share the last bucket
        if (k != run_key) {
            if (run_len != 0)
                atomicAdd(&cnt[run_key], run_len);
            run_key = k, run_len = 0;
        }
        ++run_len;
    }
    if (run_len != 0)
        atomicAdd(&cnt[run_key], run_len);
}

// exclusive scan of the counts in place (one workgroup), then ctl[1] = regroup
__global__ __launch_bounds__(1024) void key_scan_kernel(u32 *cnt, u32 nb, u64 n, u32 *ctl)
{
    __shared__ u32 wsum[16];
    const bool regroup = key_regroup(ctl, n);
    if (threadIdx.x == 0)
        ctl[1] = regroup;
    if (!regroup)
        return;
    const u32 t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const u32 per = (nb + blockDim.x - 1) / blockDim.x, b0 = min(nb, t * per), b1 = min(nb, b0 + per);
    u32 sum = 0;
#pragma unroll 8
    for (u32 i = b0; i < b1; ++i)
        sum += cnt[i];
    u32 incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = (u32)__shfl_up((int)incl, off, 64);
        if (lane >= (u32)off)
            incl += y;
    }
    if (lane == 63)
        wsum[wave] = incl;
    __syncthreads();
    u32 run = incl - sum;
    for (u32 w = 0; w < wave; ++w)
        run += wsum[w];
#pragma unroll 8
    for (u32 i = b0; i < b1; ++i) {
        const u32 c = cnt[i];
        cnt[i] = run;
        run += c;
    }
}

__global__ __launch_bounds__(256) void key_scatter_kernel(const ptls_mi355x_record_t *recs, u64 n, u32 nkeys, u32 *cur, u32 *perm,
                                                          ptls_mi355x_record_t *grouped, const u32 *ctl)
{
    if (ctl[1] == 0)
        return;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_record_t r = recs[i];
        const u32 slot = atomicAdd(&cur[r.key_idx < nkeys ? r.key_idx : nkeys], 1u);
        perm[slot] = (u32)i;
        grouped[slot] = r;
    }
}

// AES-ECB of independent blocks (one block per thread, keys from the keyset). Blocks whose key index is out of range
// produce zeros.
template <int NR>
__global__ __launch_bounds__(256) void ecb_kernel(const KeyEntry *keys, u32 nkeys, const u32 *key_idx, const uint8_t *in,
                                                  uint8_t *out, u64 nblocks)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    build_aes_tables(lds);
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nblocks; i += (u64)gridDim.x * blockDim.x) {
        const u32 ki = key_idx != nullptr ? key_idx[i] : 0u;
        u32x4 o = {0, 0, 0, 0};
        if (ki < nkeys) {
            const KeyEntry *k = keys + ki;
            u32 rk[NR + 1][4];
            for (int r = 0; r <= NR; ++r)
                for (int c = 0; c < 4; ++c)
                    rk[r][c] = k->rk[r][c];
            const u32x4 v = *(const u32x4_u *)(in + 16 * i);
            u32 s0 = v[0] ^ rk[0][0], s1 = v[1] ^ rk[0][1], s2 = v[2] ^ rk[0][2], s3 = v[3] ^ rk[0][3];
            aes_encrypt_tt<NR>(lds, laneoff, rk, s0, s1, s2, s3);
            o = u32x4{s0, s1, s2, s3};
        }
        *(u32x4_u *)(out + 16 * i) = o;
    }
}

// QUIC header-protection masks (fusion's supp, lib/fusion.c:425-430,636-651): mask[i] = AES-ECB(hp key, the 16-byte
// sample at base + hp[i].sample_off). Runs after the seal kernel on the same stream, so the sample may cover the tag.
template <int NR>
__global__ __launch_bounds__(256) void hp_kernel(const KeyEntry *keys, u32 nkeys, const ptls_mi355x_hp_t *hp, const uint8_t *base,
                                                 uint8_t *masks, u64 n)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    build_aes_tables(lds);
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_hp_t h = hp[i];
        u32x4 o = {0, 0, 0, 0};
        if (h.key_idx < nkeys) {
            const KeyEntry *k = keys + h.key_idx;
            u32 rk[NR + 1][4];
            for (int r = 0; r <= NR; ++r)
                for (int c = 0; c < 4; ++c)
                    rk[r][c] = k->rk[r][c];
            const u32x4 v = *(const u32x4_u *)(base + h.sample_off);
            u32 s0 = v[0] ^ rk[0][0], s1 = v[1] ^ rk[0][1], s2 = v[2] ^ rk[0][2], s3 = v[3] ^ rk[0][3];
            aes_encrypt_tt<NR>(lds, laneoff, rk, s0, s1, s2, s3);
            o = u32x4{s0, s1, s2, s3};
        }
        *(u32x4_u *)(masks + 16 * i) = o;
    }
}

// QUIC-LB connection-ID cipher (lib/quiclb-impl.h:100-162, behind ptls_fusion_quiclb lib/fusion.c:2186-2233): a 4-round
// Feistel network over the two halves of a 7..19-byte CID, each round X ^ AES-ECB((Y & mask) | len_pass) with
// len_pass = {0 x 14, len, round} (:134-135, :47-70). One thread per CID; blocks are LE words (byte i of the block in
// word i/4). The middle byte of an odd-length CID belongs to both halves, split by nibble masks (:107-125).
template <int NR>
__device__ __forceinline__ u32x4 quiclb_f(const lds_u8 *lds, u32 laneoff, const u32 (*rk)[4], u32x4 y, u32x4 m, u32 len, u32 rnd)
{
    u32 s0 = (y[0] & m[0]) ^ rk[0][0], s1 = (y[1] & m[1]) ^ rk[0][1], s2 = (y[2] & m[2]) ^ rk[0][2];
    u32 s3 = ((y[3] & m[3]) | len << 16 | rnd << 24) ^ rk[0][3];
    aes_encrypt_tt<NR>(lds, laneoff, rk, s0, s1, s2, s3);
    return u32x4{s0, s1, s2, s3};
}

__device__ __forceinline__ void set_byte(u32x4 &v, u32 i, u32 b) { v[i >> 2] |= (b & 0xffu) << (8 * (i & 3)); }
__device__ __forceinline__ u32 get_byte(const u32x4 &v, u32 i) { return (v[i >> 2] >> (8 * (i & 3))) & 0xffu; }

template <int NR>
__global__ __launch_bounds__(256) void quiclb_kernel(const KeyEntry *keys, u32 nkeys, const ptls_mi355x_cid_t *cids,
                                                     const uint8_t *in, uint8_t *out, u64 n)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    build_aes_tables(lds);
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_cid_t c = cids[i];
        const u32 L = c.len;
        if (c.key_idx >= nkeys || L < PTLS_MI355X_QUICLB_MIN_LEN || L > PTLS_MI355X_QUICLB_MAX_LEN)
            continue;  // invalid entries are not written
        const KeyEntry *k = keys + c.key_idx;
        u32 rk[NR + 1][4];
        for (int r = 0; r <= NR; ++r)
            for (int w = 0; w < 4; ++w)
                rk[r][w] = k->rk[r][w];
        const u32 half = L / 2, odd = L & 1, hl = half + odd;  // bytes per side: (L + 1) / 2
        // masks (:107-125): left keeps bytes [0, half) and the high nibble of the middle byte; right keeps its low nibble
        // (byte 0) and the bytes after it
        u32x4 ml = {0, 0, 0, 0}, mr = {0, 0, 0, 0};
        for (u32 b = 0; b < half; ++b)
            set_byte(ml, b, 0xff), set_byte(mr, b + odd, 0xff);
        if (odd)
            set_byte(ml, half, 0xf0), set_byte(mr, 0, 0x0f);
        // split (:72-84): l = in[0, hl), r = in[half, half + hl), zero padded
        const uint8_t *src = in + c.in_off;
        u32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
        for (u32 t = 0; t < hl; ++t)
            set_byte(a, t, src[t]), set_byte(b, t, src[half + t]);
        u32x4 l, r;
        if (c.encrypt) {  // (:149-154) l0 = a, r0 = b
            const u32x4 r1 = b ^ quiclb_f<NR>(lds, laneoff, rk, a, ml, L, 1);
            const u32x4 l1 = a ^ quiclb_f<NR>(lds, laneoff, rk, r1, mr, L, 2);
            r = r1 ^ quiclb_f<NR>(lds, laneoff, rk, l1, ml, L, 3);
            l = l1 ^ quiclb_f<NR>(lds, laneoff, rk, r, mr, L, 4);
        } else {  // (:155-161) l2 = a, r2 = b
            const u32x4 l1 = a ^ quiclb_f<NR>(lds, laneoff, rk, b, mr, L, 4);
            const u32x4 r1 = b ^ quiclb_f<NR>(lds, laneoff, rk, l1, ml, L, 3);
            l = l1 ^ quiclb_f<NR>(lds, laneoff, rk, r1, mr, L, 2);
            r = r1 ^ quiclb_f<NR>(lds, laneoff, rk, l, ml, L, 1);
        }
        // merge (:86-100)
        uint8_t *dst = out + c.out_off;
        for (u32 t = 0; t < half; ++t)
            dst[t] = (uint8_t)get_byte(l, t);
        if (odd)
            dst[half] = (uint8_t)((get_byte(l, half) & 0xf0u) | (get_byte(r, 0) & 0x0fu));
        for (u32 t = 0; t < half; ++t)
            dst[half + odd + t] = (uint8_t)get_byte(r, t + odd);
    }
}

// After opening framed TLS records: outer header check, then the receive-side padding strip of lib/picotls.c:5960-5968
// (the inner content type is the last non-zero plaintext byte; an all-zero plaintext, or an empty alert / handshake
// record, is an unexpected message). One thread per record; ok[i] becomes 1 only for status 0.
__global__ __launch_bounds__(256) void tls_unpad_kernel(const ptls_mi355x_record_t *recs, u64 n, const uint8_t *in,
                                                        const uint8_t *out, uint8_t *ok, ptls_mi355x_tls_result_t *res)
{
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_record_t r = recs[i];
        ptls_mi355x_tls_result_t o = {0, 0, 0, 0};
        const uint8_t *h = in + r.in_off;
        if (!ok[i]) {
            o.status = PTLS_MI355X_TLS_BAD_MAC;
        } else if (h[0] != 23 || h[1] != 3 || h[2] != 3 || ((u32)h[3] << 8 | h[4]) != r.len + 16) {
            o.status = PTLS_MI355X_TLS_BAD_HEADER;
        } else {
            const uint8_t *p = out + r.out_off;
            u32 len = r.len;
            while (len != 0 && p[len - 1] == 0)
                --len;
            if (len == 0) {
                o.status = PTLS_MI355X_TLS_UNEXPECTED_MESSAGE;
            } else {
                o.content_type = p[len - 1];
                o.plain_len = len - 1;
                if (o.plain_len == 0 && (o.content_type == 21 || o.content_type == 22))
                    o.status = PTLS_MI355X_TLS_UNEXPECTED_MESSAGE;
            }
        }
        ok[i] = o.status == 0;
        if (res != nullptr)
            res[i] = o;
    }
}

// After opening TLS 1.2 records: the record header must be {type, 3, 3, BE16(8 + len + 16)} (parse_record /
// handle_input_tls12, lib/picotls.c:6019-6045); TLS 1.2 has no inner content type or padding, so the content is the
// whole plaintext and the type is the (authenticated) outer one. ok[i] becomes 1 only for status 0.
__global__ __launch_bounds__(256) void tls12_check_kernel(const ptls_mi355x_record_t *recs, u64 n, const uint8_t *in, uint8_t *ok,
                                                          ptls_mi355x_tls_result_t *res)
{
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_record_t r = recs[i];
        ptls_mi355x_tls_result_t o = {0, 0, 0, 0};
        const uint8_t *h = in + r.in_off;
        if (!ok[i])
            o.status = PTLS_MI355X_TLS_BAD_MAC;
        else if (h[1] != 3 || h[2] != 3 || ((u32)h[3] << 8 | h[4]) != r.len + TLS12_RECORD_IV_SIZE + 16)
            o.status = PTLS_MI355X_TLS_BAD_HEADER;
        o.content_type = h[0];
        o.plain_len = o.status == 0 ? r.len : 0;
        ok[i] = o.status == 0;
        if (res != nullptr)
            res[i] = o;
    }
}

// ------------------------------------------------------------------------------------------------ host side

static thread_local char g_err[256];

static int fail(const char *fmt, const char *detail)
{
    snprintf(g_err, sizeof(g_err), fmt, detail);
    return -1;
}

#define HIP_TRY(expr)                                                                                                         \
    do {                                                                                                                      \
        hipError_t e_ = (expr);                                                                                               \
        if (e_ != hipSuccess)                                                                                                 \
            return fail(#expr ": %s", hipGetErrorString(e_));                                                                 \
    } while (0)

struct st_ptls_mi355x_keyset_t {
    int device;
    size_t nkeys, key_size;
    int nr;
    KeyEntry *d_keys;
    int ncu;
    int schedule;
    // staging for the synchronous host-buffer helpers (the per-record picotls path): one pinned host buffer and one
    // device buffer, grown on demand, and a stream of their own, so a call is one H2D copy, one launch, one D2H copy
    uint8_t *d_stage, *h_stage;
    size_t stage_cap;
    hipStream_t stream;
    // key grouping of ungrouped many-key batches (key_group_*): scratch for key counts and the record permutation,
    // grown on demand; group_ev orders its users when batches on several streams share the keyset
    u32 *d_group;
    size_t group_cap;
    hipEvent_t group_ev;
};

static int stage_reserve(ptls_mi355x_keyset_t *ks, size_t bytes)
{
    if (bytes <= ks->stage_cap)
        return 0;
    size_t cap = ks->stage_cap * 2 > bytes ? ks->stage_cap * 2 : bytes;
    cap = cap < 4096 ? 4096 : (cap + 4095) & ~(size_t)4095;
    if (ks->stream == NULL)
        HIP_TRY(hipStreamCreateWithFlags(&ks->stream, hipStreamNonBlocking));
    if (ks->d_stage != NULL) {
        HIP_TRY(hipStreamSynchronize(ks->stream));
        hipFree(ks->d_stage);
        hipHostFree(ks->h_stage);
        ks->d_stage = ks->h_stage = NULL;
        ks->stage_cap = 0;
    }
    HIP_TRY(hipMalloc((void **)&ks->d_stage, cap));
    if (hipHostMalloc((void **)&ks->h_stage, cap, hipHostMallocDefault) != hipSuccess) {
        hipFree(ks->d_stage);
        ks->d_stage = NULL;
        return fail("%s", "stage: pinned host allocation failed");
    }
    ks->stage_cap = cap;
    return 0;
}

// H2D of the first `up` staged bytes, the launch (run by the caller's lambda), D2H of [down_off, down_off + down),
// then wait: the synchronous round trip of the host-buffer helpers
template <typename Launch>
static int stage_roundtrip(ptls_mi355x_keyset_t *ks, size_t up, size_t down_off, size_t down, Launch launch)
{
    HIP_TRY(hipMemcpyAsync(ks->d_stage, ks->h_stage, up, hipMemcpyHostToDevice, ks->stream));
    if (launch() != 0)
        return -1;
    HIP_TRY(hipMemcpyAsync(ks->h_stage + down_off, ks->d_stage + down_off, down, hipMemcpyDeviceToHost, ks->stream));
    HIP_TRY(hipStreamSynchronize(ks->stream));
    return 0;
}

static int engine_init_attrs(void)
{
    static int done = 0;
    if (done)
        return 0;
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<10, false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<10, true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<14, false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<14, true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
#define CHUNKED_ATTR(nr, open, frame)                                                                                  \
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_chunked_kernel<nr, open, frame>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                CLDS_ALLOC))
    CHUNKED_ATTR(10, false, 0);
    CHUNKED_ATTR(10, true, 0);
    CHUNKED_ATTR(14, false, 0);
    CHUNKED_ATTR(14, true, 0);
    CHUNKED_ATTR(10, false, 1);
    CHUNKED_ATTR(10, true, 1);
    CHUNKED_ATTR(14, false, 1);
    CHUNKED_ATTR(14, true, 1);
    CHUNKED_ATTR(10, false, 2);
    CHUNKED_ATTR(10, true, 2);
    CHUNKED_ATTR(14, false, 2);
    CHUNKED_ATTR(14, true, 2);
#undef CHUNKED_ATTR
    HIP_TRY(hipFuncSetAttribute((const void *)ecb_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)ecb_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)hp_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)hp_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)quiclb_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    done = 1;
    return 0;
}

extern "C" {

const char *ptls_mi355x_last_error(void) { return g_err; }

int ptls_mi355x_is_supported(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return 0;
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return 0;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

ptls_mi355x_keyset_t *ptls_mi355x_keyset_new(const void *keys, const void *ivs, size_t nkeys, size_t key_size)
{
    if (keys == NULL || ivs == NULL || nkeys == 0 || (key_size != 16 && key_size != 32) || nkeys > (1u << 30)) {
        fail("%s", "ptls_mi355x_keyset_new: invalid arguments");
        return NULL;
    }
    if (engine_init_attrs() != 0)
        return NULL;
    ptls_mi355x_keyset_t *ks = (ptls_mi355x_keyset_t *)calloc(1, sizeof(*ks));
    uint8_t *d_raw = NULL;
    if (ks == NULL)
        return NULL;
    ks->nkeys = nkeys, ks->key_size = key_size, ks->nr = key_size == 16 ? 10 : 14;
    if (hipGetDevice(&ks->device) != hipSuccess || hipDeviceGetAttribute(&ks->ncu, hipDeviceAttributeMultiprocessorCount, ks->device) != hipSuccess)
        goto Fail;
    if (hipMalloc((void **)&ks->d_keys, nkeys * sizeof(KeyEntry)) != hipSuccess)
        goto Fail;
    if (hipMalloc((void **)&d_raw, nkeys * (key_size + 12)) != hipSuccess)
        goto Fail;
    if (hipMemcpy(d_raw, keys, nkeys * key_size, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_raw + nkeys * key_size, ivs, nkeys * 12, hipMemcpyHostToDevice) != hipSuccess)
        goto Fail;
    keyset_setup_kernel<<<(unsigned)((nkeys + 127) / 128), 128>>>(d_raw, d_raw + nkeys * key_size, ks->d_keys, (u32)nkeys, (u32)key_size);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        goto Fail;
    hipMemset(d_raw, 0, nkeys * (key_size + 12));
    hipFree(d_raw);
    return ks;
Fail:
    fail("%s", "ptls_mi355x_keyset_new: device setup failed");
    if (d_raw != NULL)
        hipFree(d_raw);
    if (ks->d_keys != NULL)
        hipFree(ks->d_keys);
    free(ks);
    return NULL;
}

int ptls_mi355x_keyset_update(ptls_mi355x_keyset_t *ks, const uint32_t *key_idx, const void *keys, const void *ivs, size_t n)
{
    if (ks == NULL || (n != 0 && (key_idx == NULL || keys == NULL || ivs == NULL)))
        return fail("%s", "keyset_update: invalid arguments");
    std::vector<bool> seen(n != 0 ? ks->nkeys : 0);
    for (size_t i = 0; i < n; ++i) {
        if (key_idx[i] >= ks->nkeys)
            return fail("%s", "keyset_update: key index out of range");
        if (seen[key_idx[i]])
            return fail("%s", "keyset_update: key index listed twice");
        seen[key_idx[i]] = true;
    }
    if (n == 0)
        return 0;
    uint8_t *d = NULL;
    const size_t kb = n * ks->key_size, ib = n * 12, sb = n * 4;
    HIP_TRY(hipMalloc((void **)&d, kb + ib + sb));
    int ret = -1;
    if (hipDeviceSynchronize() == hipSuccess &&  // no launch in flight still reads the old entries
        hipMemcpy(d, keys, kb, hipMemcpyHostToDevice) == hipSuccess && hipMemcpy(d + kb, ivs, ib, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(d + kb + ib, key_idx, sb, hipMemcpyHostToDevice) == hipSuccess) {
        keyset_setup_kernel<<<(unsigned)((n + 127) / 128), 128>>>(d, d + kb, ks->d_keys, (u32)n, (u32)ks->key_size,
                                                                 (const u32 *)(d + kb + ib));
        if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess)
            ret = 0;
    }
    hipMemset(d, 0, kb + ib);
    hipDeviceSynchronize();
    hipFree(d);
    if (ret != 0)
        fail("%s", "keyset_update: device setup failed");
    return ret;
}

void ptls_mi355x_keyset_free(ptls_mi355x_keyset_t *ks)
{
    if (ks == NULL)
        return;
    hipMemset(ks->d_keys, 0, ks->nkeys * sizeof(KeyEntry));
    hipDeviceSynchronize();
    hipFree(ks->d_keys);
    if (ks->d_stage != NULL) {
        hipMemset(ks->d_stage, 0, ks->stage_cap);
        memset(ks->h_stage, 0, ks->stage_cap);  // staged plaintext and keystream-derived bytes
        hipDeviceSynchronize();
        hipFree(ks->d_stage);
        hipHostFree(ks->h_stage);
    }
    if (ks->stream != NULL)
        hipStreamDestroy(ks->stream);
    if (ks->group_ev != NULL) {
        hipEventSynchronize(ks->group_ev);
        hipEventDestroy(ks->group_ev);
    }
    hipFree(ks->d_group);
    free(ks);
}

#if ENGINE_PROFILE
int ptls_mi355x_debug_profile(unsigned long long *out, int reset)
{
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(g_prof)));
    if (reset) {
        static const unsigned long long z[8] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)));
    }
    return 0;
}
#endif

int ptls_mi355x_keyset_set_schedule(ptls_mi355x_keyset_t *ks, int schedule)
{
    if (ks == NULL || schedule < PTLS_MI355X_SCHEDULE_AUTO || schedule > PTLS_MI355X_SCHEDULE_CHUNKED)
        return fail("%s", "set_schedule: invalid arguments");
    ks->schedule = schedule;
    return 0;
}

size_t ptls_mi355x_keyset_size(const ptls_mi355x_keyset_t *ks) { return ks->nkeys; }
size_t ptls_mi355x_keyset_key_size(const ptls_mi355x_keyset_t *ks) { return ks->key_size; }

int ptls_mi355x_keyset_get_iv(ptls_mi355x_keyset_t *ks, size_t key_idx, void *iv)
{
    if (ks == NULL || key_idx >= ks->nkeys)
        return fail("%s", "get_iv: bad key index");
    u32 w[3];
    HIP_TRY(hipMemcpy(w, ks->d_keys[key_idx].iv, 12, hipMemcpyDeviceToHost));
    memcpy(iv, w, 12);
    return 0;
}

int ptls_mi355x_keyset_set_iv(ptls_mi355x_keyset_t *ks, size_t key_idx, const void *iv)
{
    if (ks == NULL || key_idx >= ks->nkeys)
        return fail("%s", "set_iv: bad key index");
    u32 w[3];
    memcpy(w, iv, 12);
    HIP_TRY(hipMemcpy(ks->d_keys[key_idx].iv, w, 12, hipMemcpyHostToDevice));
    return 0;
}

// Schedule choice (ptls_mi355x_keyset_set_schedule): AUTO = chunked. Its uniform runs take the whole-record path,
// which measured at or above the lockstep kernel on one-key uniform batches (929 vs 841 GiB/s on 16 KiB records,
// 784 vs 751 on 1200 B), and its chunked runs balance mixed lengths and short key runs.
static bool use_chunked(const ptls_mi355x_keyset_t *ks) { return ks->schedule != PTLS_MI355X_SCHEDULE_LOCKSTEP; }

static int launch_batch(ptls_mi355x_keyset_t *ks, bool open, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                        const void *aad, void *out, uint8_t *ok, void *stream, int frame = 0, u32 unit_log2 = CHUNK_LOG2)
{
    if (ks == NULL || (nrecs != 0 && (recs == NULL || in == NULL || out == NULL || (open && ok == NULL))))
        return fail("%s", "batch: invalid arguments");
    if (nrecs == 0)
        return 0;
    BatchArgs a = {ks->d_keys, recs, (u64)nrecs, (const uint8_t *)in, (const uint8_t *)aad, (uint8_t *)out, ok,
                   ks->nkeys > 1 ? 1u : 0u, (u32)ks->nkeys, unit_log2, nullptr, nullptr, nullptr};
    if (a.aad == NULL)
        a.aad = a.in;
    const u64 groups = (nrecs + (64 / ENGINE_G) - 1) / (64 / ENGINE_G);
    // one persistent workgroup per CU; small batches use fewer workgroups so each still gets >= 4 record groups
    u64 grid = (u64)ks->ncu;
    if (grid > (groups + 3) / 4)
        grid = (groups + 3) / 4;
    if (grid < 1)
        grid = 1;
    hipStream_t s = (hipStream_t)stream;
    // ungrouped many-key batches: group the records by key on the device first (see key_hist_kernel)
#ifndef KEY_GROUP_DISABLE
    const bool group = use_chunked(ks) && ks->nkeys > 1 && ks->nkeys <= KEY_GROUP_MAX_KEYS && nrecs > 1 &&
                       nrecs <= 0xffffffffu;
#else
    const bool group = false;
#endif
    if (group) {
        // scratch: ctl[2] | counts[nkeys + 1] | perm[n] | (8-byte aligned) grouped descriptors[n]
        const size_t nb = ks->nkeys + 1, words = ((2 + nb + nrecs + 1) & ~(size_t)1) + nrecs * (sizeof(ptls_mi355x_record_t) / 4);
        if (ks->group_ev == NULL)
            HIP_TRY(hipEventCreateWithFlags(&ks->group_ev, hipEventDisableTiming));
        if (words > ks->group_cap) {
            HIP_TRY(hipEventSynchronize(ks->group_ev));
            hipFree(ks->d_group);
            ks->d_group = NULL;
            ks->group_cap = 0;
            HIP_TRY(hipMalloc((void **)&ks->d_group, words * 4));
            ks->group_cap = words;
        }
        HIP_TRY(hipStreamWaitEvent(s, ks->group_ev, 0));  // a batch on another stream may still use the scratch
        u32 *ctl = ks->d_group, *cnt = ctl + 2, *perm = cnt + nb;
        HIP_TRY(hipMemsetAsync(ctl, 0, (2 + nb) * 4, s));
        const unsigned gh = (unsigned)min((nrecs + 255) / 256, (size_t)ks->ncu * 8);
        key_changes_kernel<<<gh, 256, 0, s>>>(recs, nrecs, ctl);
        key_hist_kernel<<<gh, 256, 0, s>>>(recs, nrecs, (u32)ks->nkeys, cnt, ctl);
        key_scan_kernel<<<1, 1024, 0, s>>>(cnt, (u32)nb, nrecs, ctl);
        ptls_mi355x_record_t *grouped = (ptls_mi355x_record_t *)(ctl + ((2 + nb + nrecs + 1) & ~(size_t)1));
        key_scatter_kernel<<<gh, 256, 0, s>>>(recs, nrecs, (u32)ks->nkeys, cnt, perm, grouped, ctl);
        a.grouped = grouped;
        a.perm = perm;
        a.perm_on = ctl + 1;
    }
#define CHUNKED_LAUNCH(nr, op, frame) gcm_chunked_kernel<nr, op, frame><<<(unsigned)grid, ENGINE_WG, CLDS_ALLOC, s>>>(a)
    if (frame == 1) {
        if (ks->nr == 10) {
            if (open)
                CHUNKED_LAUNCH(10, true, 1);
            else
                CHUNKED_LAUNCH(10, false, 1);
        } else {
            if (open)
                CHUNKED_LAUNCH(14, true, 1);
            else
                CHUNKED_LAUNCH(14, false, 1);
        }
    } else if (frame == 2) {
        if (ks->nr == 10) {
            if (open)
                CHUNKED_LAUNCH(10, true, 2);
            else
                CHUNKED_LAUNCH(10, false, 2);
        } else {
            if (open)
                CHUNKED_LAUNCH(14, true, 2);
            else
                CHUNKED_LAUNCH(14, false, 2);
        }
    } else if (use_chunked(ks)) {
        if (ks->nr == 10) {
            if (open)
                CHUNKED_LAUNCH(10, true, 0);
            else
                CHUNKED_LAUNCH(10, false, 0);
        } else {
            if (open)
                CHUNKED_LAUNCH(14, true, 0);
            else
                CHUNKED_LAUNCH(14, false, 0);
        }
    } else if (ks->nr == 10) {
        if (open)
            gcm_batch_kernel<10, true><<<(unsigned)grid, ENGINE_WG, LDS_ALLOC, s>>>(a);
        else
            gcm_batch_kernel<10, false><<<(unsigned)grid, ENGINE_WG, LDS_ALLOC, s>>>(a);
    } else {
        if (open)
            gcm_batch_kernel<14, true><<<(unsigned)grid, ENGINE_WG, LDS_ALLOC, s>>>(a);
        else
            gcm_batch_kernel<14, false><<<(unsigned)grid, ENGINE_WG, LDS_ALLOC, s>>>(a);
    }
    HIP_TRY(hipGetLastError());
    if (group)
        HIP_TRY(hipEventRecord(ks->group_ev, s));
    return 0;
}

int ptls_mi355x_seal_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                           const void *aad, void *out, void *stream)
{
    return launch_batch(ks, false, recs, nrecs, in, aad, out, NULL, stream);
}

int ptls_mi355x_open_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                           const void *aad, void *out, uint8_t *ok, void *stream)
{
    return launch_batch(ks, true, recs, nrecs, in, aad, out, ok, stream);
}

int ptls_mi355x_ecb_batch(ptls_mi355x_keyset_t *ks, const uint32_t *key_idx, const void *in, void *out, size_t nblocks,
                          void *stream)
{
    if (ks == NULL || (nblocks != 0 && (in == NULL || out == NULL)))
        return fail("%s", "ecb: invalid arguments");
    if (nblocks == 0)
        return 0;
    u64 grid = (nblocks + 255) / 256;
    if (grid > (u64)ks->ncu * 4)
        grid = (u64)ks->ncu * 4;
    hipStream_t s = (hipStream_t)stream;
    if (ks->nr == 10)
        ecb_kernel<10><<<(unsigned)grid, 256, LDS_AES_BYTES, s>>>(ks->d_keys, (u32)ks->nkeys, key_idx, (const uint8_t *)in,
                                                                  (uint8_t *)out, nblocks);
    else
        ecb_kernel<14><<<(unsigned)grid, 256, LDS_AES_BYTES, s>>>(ks->d_keys, (u32)ks->nkeys, key_idx, (const uint8_t *)in,
                                                                  (uint8_t *)out, nblocks);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_seal_tls_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                 void *out, void *stream)
{
    return launch_batch(ks, false, recs, nrecs, in, NULL, out, NULL, stream, 1);
}

int ptls_mi355x_open_tls_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                 void *out, uint8_t *ok, ptls_mi355x_tls_result_t *results, void *stream)
{
    if (launch_batch(ks, true, recs, nrecs, in, NULL, out, ok, stream, 1) != 0)
        return -1;
    if (nrecs == 0)
        return 0;
    u64 grid = (nrecs + 255) / 256;
    if (grid > (u64)ks->ncu * 4)
        grid = (u64)ks->ncu * 4;
    tls_unpad_kernel<<<(unsigned)grid, 256, 0, (hipStream_t)stream>>>(recs, nrecs, (const uint8_t *)in, (const uint8_t *)out,
                                                                       ok, results);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_seal_tls12_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                   void *out, void *stream)
{
    return launch_batch(ks, false, recs, nrecs, in, NULL, out, NULL, stream, 2);
}

int ptls_mi355x_open_tls12_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                   void *out, uint8_t *ok, ptls_mi355x_tls_result_t *results, void *stream)
{
    if (launch_batch(ks, true, recs, nrecs, in, NULL, out, ok, stream, 2) != 0)
        return -1;
    if (nrecs == 0)
        return 0;
    u64 grid = (nrecs + 255) / 256;
    if (grid > (u64)ks->ncu * 4)
        grid = (u64)ks->ncu * 4;
    tls12_check_kernel<<<(unsigned)grid, 256, 0, (hipStream_t)stream>>>(recs, nrecs, (const uint8_t *)in, ok, results);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_hp_mask_batch(ptls_mi355x_keyset_t *hp_ks, const ptls_mi355x_hp_t *hp, size_t n, const void *base,
                              void *masks, void *stream)
{
    if (hp_ks == NULL || (n != 0 && (hp == NULL || base == NULL || masks == NULL)))
        return fail("%s", "hp_mask: invalid arguments");
    if (n == 0)
        return 0;
    u64 grid = (n + 255) / 256;
    if (grid > (u64)hp_ks->ncu * 4)
        grid = (u64)hp_ks->ncu * 4;
    hipStream_t s = (hipStream_t)stream;
    if (hp_ks->nr == 10)
        hp_kernel<10><<<(unsigned)grid, 256, LDS_AES_BYTES, s>>>(hp_ks->d_keys, (u32)hp_ks->nkeys, hp, (const uint8_t *)base,
                                                                 (uint8_t *)masks, n);
    else
        hp_kernel<14><<<(unsigned)grid, 256, LDS_AES_BYTES, s>>>(hp_ks->d_keys, (u32)hp_ks->nkeys, hp, (const uint8_t *)base,
                                                                 (uint8_t *)masks, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_seal_batch_hp(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                              const void *aad, void *out, ptls_mi355x_keyset_t *hp_ks, const ptls_mi355x_hp_t *hp,
                              void *masks, void *stream)
{
    if (hp_ks == NULL || (nrecs != 0 && (hp == NULL || masks == NULL)))
        return fail("%s", "seal_batch_hp: invalid arguments");
    if (launch_batch(ks, false, recs, nrecs, in, aad, out, NULL, stream) != 0)
        return -1;
    return ptls_mi355x_hp_mask_batch(hp_ks, hp, nrecs, out, masks, stream);
}

int ptls_mi355x_quiclb_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_cid_t *cids, size_t n, const void *in, void *out,
                             void *stream)
{
    if (ks == NULL || (n != 0 && (cids == NULL || in == NULL || out == NULL)))
        return fail("%s", "quiclb: invalid arguments");
    if (ks->key_size != 16)
        return fail("%s", "quiclb: the QUIC-LB cipher is keyed with AES-128 (PTLS_QUICLB_KEY_SIZE)");
    if (n == 0)
        return 0;
    u64 grid = (n + 255) / 256;
    if (grid > (u64)ks->ncu * 4)
        grid = (u64)ks->ncu * 4;
    quiclb_kernel<10><<<(unsigned)grid, 256, LDS_AES_BYTES, (hipStream_t)stream>>>(ks->d_keys, (u32)ks->nkeys, cids,
                                                                                    (const uint8_t *)in, (uint8_t *)out, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_quiclb_transform(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t len, int encrypt)
{
    if (ks == NULL || key_idx >= ks->nkeys || output == NULL || input == NULL || len < PTLS_MI355X_QUICLB_MIN_LEN ||
        len > PTLS_MI355X_QUICLB_MAX_LEN)
        return fail("%s", "quiclb_transform: invalid arguments");
    if (stage_reserve(ks, 96) != 0)
        return -1;
    // staging: [0, 32) CID in, [32, 56) descriptor | [64, 96) CID out
    const ptls_mi355x_cid_t c = {0, 64, (uint32_t)key_idx, (uint8_t)len, (uint8_t)(encrypt != 0), 0};
    memcpy(ks->h_stage, input, len);
    memcpy(ks->h_stage + 32, &c, sizeof(c));
    uint8_t *d = ks->d_stage;
    if (stage_roundtrip(ks, 64, 64, 32, [&] {
            return ptls_mi355x_quiclb_batch(ks, (const ptls_mi355x_cid_t *)(d + 32), 1, d, d, ks->stream);
        }) != 0)
        return -1;
    memcpy(output, ks->h_stage + 64, len);
    return 0;
}

int ptls_mi355x_encrypt_block(ptls_mi355x_keyset_t *ks, size_t key_idx, void *out, const void *in)
{
    if (ks == NULL || key_idx >= ks->nkeys || out == NULL || in == NULL)
        return fail("%s", "encrypt_block: invalid arguments");
    if (stage_reserve(ks, 64) != 0)
        return -1;
    // staging: [0, 16) block in, [16, 20) key index | [32, 48) block out
    const u32 idx = (u32)key_idx;
    memcpy(ks->h_stage, in, 16);
    memcpy(ks->h_stage + 16, &idx, 4);
    uint8_t *d = ks->d_stage;
    if (stage_roundtrip(ks, 32, 32, 16, [&] {
            return ptls_mi355x_ecb_batch(ks, (const uint32_t *)(d + 16), d, d + 32, 1, ks->stream);
        }) != 0)
        return -1;
    memcpy(out, ks->h_stage + 32, 16);
    return 0;
}

// single record on host buffers: a batch of one through the keyset's staging buffers
static int single(ptls_mi355x_keyset_t *ks, size_t key_idx, bool open, void *output, const void *input, size_t len, uint64_t seq,
                  const void *aad, size_t aadlen, int *verified)
{
    if (ks == NULL || key_idx >= ks->nkeys || aadlen > 0xffff || len > PTLS_MI355X_MAX_RECORD_LEN)
        return fail("%s", "single: invalid arguments");
    const size_t inbytes = len + (open ? 16 : 0), outbytes = len + (open ? 0 : 16);
    // staging: [in | aad | descriptor] goes up, [out | ok] comes back
    const size_t off_in = 0, off_aad = (inbytes + 15) & ~(size_t)15, off_rec = off_aad + ((aadlen + 15) & ~(size_t)15),
                 off_out = off_rec + 64, off_ok = off_out + ((outbytes + 15) & ~(size_t)15), total = off_ok + 16;
    if (stage_reserve(ks, total) != 0)
        return -1;
    const ptls_mi355x_record_t r = {0, 0, seq, 0, (u32)len, 0, (uint16_t)aadlen, 0};  // offsets relative to the arenas below
    ptls_mi355x_keyset_t view = *ks;
    view.d_keys = ks->d_keys + key_idx;
    view.nkeys = 1;
    uint8_t *h = ks->h_stage, *d = ks->d_stage;
    if (inbytes != 0)
        memcpy(h + off_in, input, inbytes);
    if (aadlen != 0)
        memcpy(h + off_aad, aad, aadlen);
    memcpy(h + off_rec, &r, sizeof(r));
    // one record on one workgroup: shorter units put more of its waves to work (a unit step costs a lone wave ~2 us of
    // latency, a unit combine ~0.15 us); steps / 2^k units balance the two
    const size_t steps = ((aadlen + 15) / 16 + (len + 15) / 16 + 1 + ENGINE_G - 1) / ENGINE_G;
    const u32 unit_log2 = steps <= 24 ? 0 : steps <= 96 ? 1 : steps <= 400 ? 2 : steps <= 1600 ? 3 : CHUNK_LOG2;
    if (stage_roundtrip(ks, off_out, off_out, total - off_out, [&] {
            return launch_batch(&view, open, (const ptls_mi355x_record_t *)(d + off_rec), 1, d + off_in, d + off_aad,
                                d + off_out, d + off_ok, ks->stream, 0, unit_log2 < CHUNK_LOG2 ? unit_log2 : CHUNK_LOG2);
        }) != 0)
        return -1;
    if (outbytes != 0)
        memcpy(output, h + off_out, outbytes);
    if (open)
        *verified = h[off_ok];
    return 0;
}

int ptls_mi355x_encrypt(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                        const void *aad, size_t aadlen)
{
    return single(ks, key_idx, false, output, input, inlen, seq, aad, aadlen, NULL);
}

size_t ptls_mi355x_decrypt(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                           const void *aad, size_t aadlen)
{
    if (inlen < 16)
        return SIZE_MAX;
    int verified = 0;
    if (single(ks, key_idx, true, output, input, inlen - 16, seq, aad, aadlen, &verified) != 0)
        return SIZE_MAX;
    return verified ? inlen - 16 : SIZE_MAX;
}

}  // extern "C"
