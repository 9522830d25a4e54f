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

#endif  // PTLS_MI355X_ENGINE_KEYSET_SETUP_H
