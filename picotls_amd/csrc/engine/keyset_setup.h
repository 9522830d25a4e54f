// picotls_amd/csrc/engine/keyset_setup.h -- On-device key schedule, H and H-power setup of a keyset (keyset_setup_kernel).
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_KEYSET_SETUP_H
#define PTLS_MI355X_ENGINE_KEYSET_SETUP_H

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

// S-box lookups: from the constant table (one thread per key of a many-key setup), or from a 256-byte LDS copy (the
// one-wave setup of a picotls context, where each lookup is on the launch's critical path)
struct SboxConst {
    __device__ __forceinline__ u32 operator()(u32 i) const { return c_sbox.v[i]; }
};
struct SboxLds {
    const lds_u8 *t;
    __device__ __forceinline__ u32 operator()(u32 i) const { return t[i]; }
};

template <typename S>
__device__ __forceinline__ u32 sub_word(const S &sb, u32 w)
{
    return sb(w & 0xff) | sb((w >> 8) & 0xff) << 8 | sb((w >> 16) & 0xff) << 16 | sb(w >> 24) << 24;
}

__device__ __forceinline__ u32 xtime_w(u32 w) { return ((w & 0x7f7f7f7fu) << 1) ^ (((w >> 7) & 0x01010101u) * 0x1bu); }

// plain word-level AES (setup only: H = E_K(0^128))
template <int NR, typename S>
__device__ __forceinline__ void aes_plain(const S &sb, const u32 (&rk)[15][4], u32 (&s)[4])
{
    constexpr int nr = NR;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        s[c] ^= rk[0][c];
#pragma unroll
    for (int r = 1; r <= nr; ++r) {
        u32 t[4];
        for (int c = 0; c < 4; ++c)
            t[c] = sub_word(sb, s[c]);
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

// x = x * y on one whole wave (x and y uniform across its 64 lanes, and so is the result): lane L adds the terms of
// bits 2L and 2L+1 of x, y * x^(2L) formed in closed form (gf_mulxs_be: at most three 32-bit steps and one shorter one),
// then an XOR over the wave. ~20x shorter than the 128-step serial loop on the launch's critical path.
__device__ void gf_mul_be_wave(u32 (&x)[4], const u32 (&y)[4])
{
    const u32 bit = 2 * (threadIdx.x & 63);
    u32 b0 = y[0], b1 = y[1], b2 = y[2], b3 = y[3];
    for (u32 k = 0; k < (bit >> 5); ++k)
        gf_mulxs_be(b0, b1, b2, b3, 32);
    if (bit & 31)
        gf_mulxs_be(b0, b1, b2, b3, bit & 31);
    const u32 xw = x[bit >> 5];
    u32 z[4] = {0, 0, 0, 0};
    if ((xw >> (31 - (bit & 31))) & 1)
        z[0] ^= b0, z[1] ^= b1, z[2] ^= b2, z[3] ^= b3;
    gf_mulxs_be(b0, b1, b2, b3, 1);
    if ((xw >> (30 - (bit & 31))) & 1)
        z[0] ^= b0, z[1] ^= b1, z[2] ^= b2, z[3] ^= b3;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1)
            z[c] ^= (u32)__shfl_xor((int)z[c], m, 64);
        x[c] = z[c];
    }
}

// FIPS-197 key expansion, H = E_K(0), the H powers and the static IV of one keyset entry (WAVE: all 64 lanes of a wave
// compute it together, with uniform inputs; lane 0 writes the entry)
// (NK = key words, 4 or 8: the loops unroll and the schedule stays in registers)
template <bool WAVE, int NK, typename S>
__device__ void setup_entry(const S &sb, const uint8_t *k, const uint8_t *v, KeyEntry *e)
{
    constexpr int nk = NK, nr = NK + 6;
    u32 w[4 * (nr + 1)];
#pragma unroll
    for (int j = 0; j < nk; ++j)
        w[j] = (u32)k[4 * j] | (u32)k[4 * j + 1] << 8 | (u32)k[4 * j + 2] << 16 | (u32)k[4 * j + 3] << 24;
    u32 rcon = 1;
#pragma unroll
    for (int j = nk; j < 4 * (nr + 1); ++j) {
        u32 t = w[j - 1];
        if (j % nk == 0) {
            t = sub_word(sb, (t >> 8) | (t << 24)) ^ rcon;
            rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0)) & 0xff;
        } else if (nk > 6 && j % nk == 4) {
            t = sub_word(sb, t);
        }
        w[j] = w[j - nk] ^ t;
    }
    u32 rk[15][4];
#pragma unroll
    for (int r = 0; r < 15; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            rk[r][c] = r <= nr ? w[4 * r + c] : 0;
    const bool writer = !WAVE || (threadIdx.x & 63) == 0;
    if (writer) {
#pragma unroll
        for (int r = 0; r < 15; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                e->rk[r][c] = r >= 1 && r < nr ? rotr8(rk[r][c]) : rk[r][c];
        for (int c = 0; c < 3; ++c)
            e->iv[c] = (u32)v[4 * c] | (u32)v[4 * c + 1] << 8 | (u32)v[4 * c + 2] << 16 | (u32)v[4 * c + 3] << 24;
        e->iv[3] = 0;
    }

    u32 s[4] = {0, 0, 0, 0};
    aes_plain<nr>(sb, rk, s);
    // H as big-endian words for the bitwise multiply (SP 800-38D Algorithm 1): H^1..H^8 by multiplication, then
    // H^16 .. H^1024 by squaring (14 products instead of a walk over every power); H^256..H^1024 are the piece
    // multipliers of long records over many workgroups (spread_pieces)
    const u32 hb[4] = {bswap32(s[0]), bswap32(s[1]), bswap32(s[2]), bswap32(s[3])};
    u32 p[4] = {hb[0], hb[1], hb[2], hb[3]};  // current power, big-endian words
    u32 out[16][4];
#pragma unroll
    for (int n = 1; n <= 8; ++n) {
        for (int c = 0; c < 4; ++c)
            out[n - 1][c] = bswap32(p[c]);
        if (n < 8) {
            if (WAVE)
                gf_mul_be_wave(p, hb);
            else
                gf_mul_be(p, hb);
        }
    }
    static_assert(CHUNK_BLOCKS >= 8 && (CHUNK_BLOCKS & (CHUNK_BLOCKS - 1)) == 0, "unit powers are squarings of H^8");
    for (int c = 0; c < 4; ++c)
        out[8][c] = out[7][c], out[12][c] = 0;  // CHUNK_BLOCKS == 8
#pragma unroll
    for (int n = 16; n <= 1024; n *= 2) {
        const u32 q[4] = {p[0], p[1], p[2], p[3]};
        if (WAVE)
            gf_mul_be_wave(p, q);  // p = H^n
        else
            gf_mul_be(p, q);
        if (n == CHUNK_BLOCKS)
            for (int c = 0; c < 4; ++c)
                out[8][c] = bswap32(p[c]);
        const int slot = n == 16 ? 9 : n == 32 ? 10 : n == 64 ? 11 : n == 128 ? 12 : n == 256 ? 13 : n == 512 ? 14 : 15;
        for (int c = 0; c < 4; ++c)
            out[slot][c] = bswap32(p[c]);
    }
    if (writer) {
#pragma unroll
        for (int n = 0; n < 16; ++n)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                e->h[n][c] = out[n][c];
    }
}

// one thread per key (slot: entry i goes to out[slot[i]] when slot != nullptr: a rekey of some connections of a keyset)
__global__ void keyset_setup_kernel(const uint8_t *__restrict__ keys, const uint8_t *__restrict__ ivs, KeyEntry *__restrict__ out,
                                    u32 nkeys, u32 key_size, const u32 *__restrict__ slot = nullptr)
{
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkeys)
        return;
    KeyEntry *e = out + (slot != nullptr ? slot[i] : i);
    if (key_size == 16)
        setup_entry<false, 4>(SboxConst{}, keys + (size_t)i * 16, ivs + (size_t)i * 12, e);
    else
        setup_entry<false, 8>(SboxConst{}, keys + (size_t)i * 32, ivs + (size_t)i * 12, e);
}

// one key passed by value in the kernel arguments (a picotls context: ptls_aead_new_direct), so that creating it needs
// no host buffer that must outlive the launch; one wave, with the S-box in LDS
struct RawKey {
    uint8_t key[32];
    uint8_t iv[12];
    u32 key_size;
};
__global__ __launch_bounds__(64) void keyset_setup_one_kernel(RawKey k, KeyEntry *out)
{
    __shared__ uint8_t sbox[256];
    const u32 l = threadIdx.x;
    sbox[4 * l] = c_sbox.v[4 * l], sbox[4 * l + 1] = c_sbox.v[4 * l + 1], sbox[4 * l + 2] = c_sbox.v[4 * l + 2],
    sbox[4 * l + 3] = c_sbox.v[4 * l + 3];
    __syncthreads();
    if (k.key_size == 16)
        setup_entry<true, 4>(SboxLds{(const lds_u8 *)sbox}, k.key, k.iv, out);
    else
        setup_entry<true, 8>(SboxLds{(const lds_u8 *)sbox}, k.key, k.iv, out);
}

// do_set_iv (lib/fusion.c:1181-1187): the static IV of one entry, by value
__global__ void keyset_set_iv_kernel(KeyEntry *e, u32 iv0, u32 iv1, u32 iv2)
{
    e->iv[0] = iv0, e->iv[1] = iv1, e->iv[2] = iv2;
}

#endif  // PTLS_MI355X_ENGINE_KEYSET_SETUP_H
