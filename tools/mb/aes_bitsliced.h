// Bitsliced AES, eight blocks per 32-bit lane: the VALU-only alternative to the LDS T-table rounds of
// aesgcm_engine.hip (DESIGN.md §5 compares the two). Plain C++ so the same code is unit-tested on the host
// (tests/c/test_bitsliced.cpp) and compiled into the gfx950 kernels.
//
// State layout. q[i][n] (row i = 0..3, n = 0..7) is one bit-plane of state row i: it holds bit (7 - n) of each of the
// row's bytes (q[i][0] = the most significant bits, the S-box circuit's input U0), and bit 8c + k of the plane
// belongs to column c (0..3) of block k (0..7). So:
//   SubBytes   = the Boyar-Peralta circuit (aes_bs_sbox.inc) on the 8 planes of each row,
//   ShiftRows  = rotate the planes of row i right by 8i bits (column c takes column c + i),
//   MixColumns = XORs between the planes of the four rows (same bit positions = same column),
//   AddRoundKey= XOR with key planes whose byte c is 0x00 or 0xff (bsk_planes).
// Loading eight blocks (LE column words, byte i = row i) is a 4x4 byte transpose per block and an 8x8 bit
// transpose per row (bs_ortho, its own inverse); storing is the reverse.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define BS_FN __host__ __device__ inline __attribute__((always_inline))
#else
#define BS_FN static inline
#endif

namespace bs {

typedef uint32_t u32;

BS_FN u32 rotr(u32 x, int n) { return n == 0 ? x : (x >> n) | (x << (32 - n)); }

BS_FN void swapmove(u32 &a, u32 &b, u32 m, int n)
{
    const u32 t = ((a >> n) ^ b) & m;
    b ^= t;
    a ^= t << n;
}

// r[7 - k] = word k (byte c at bits 8c..8c+7)  <->  r[n] = bit (7 - n) of every byte, at bit 8c + k
BS_FN void ortho(u32 (&r)[8])
{
    swapmove(r[1], r[0], 0x55555555u, 1);
    swapmove(r[3], r[2], 0x55555555u, 1);
    swapmove(r[5], r[4], 0x55555555u, 1);
    swapmove(r[7], r[6], 0x55555555u, 1);
    swapmove(r[2], r[0], 0x33333333u, 2);
    swapmove(r[3], r[1], 0x33333333u, 2);
    swapmove(r[6], r[4], 0x33333333u, 2);
    swapmove(r[7], r[5], 0x33333333u, 2);
    swapmove(r[4], r[0], 0x0f0f0f0fu, 4);
    swapmove(r[5], r[1], 0x0f0f0f0fu, 4);
    swapmove(r[6], r[2], 0x0f0f0f0fu, 4);
    swapmove(r[7], r[3], 0x0f0f0f0fu, 4);
}

// 4x4 byte transpose: out[j] byte i = in[i] byte j
BS_FN void transpose4(u32 (&o)[4], u32 a, u32 b, u32 c, u32 d)
{
    const u32 ab_lo = (a & 0x00ff00ffu) | ((b & 0x00ff00ffu) << 8);  // a0 b0 a2 b2
    const u32 ab_hi = ((a >> 8) & 0x00ff00ffu) | (b & 0xff00ff00u);  // a1 b1 a3 b3
    const u32 cd_lo = (c & 0x00ff00ffu) | ((d & 0x00ff00ffu) << 8);  // c0 d0 c2 d2
    const u32 cd_hi = ((c >> 8) & 0x00ff00ffu) | (d & 0xff00ff00u);  // c1 d1 c3 d3
    o[0] = (ab_lo & 0xffffu) | (cd_lo << 16);
    o[1] = (ab_hi & 0xffffu) | (cd_hi << 16);
    o[2] = (ab_lo >> 16) | (cd_lo & 0xffff0000u);
    o[3] = (ab_hi >> 16) | (cd_hi & 0xffff0000u);
}

// eight blocks (w[k][c]: block k, column word c) -> bit-planes
BS_FN void load(u32 (&q)[4][8], const u32 (&w)[8][4])
{
    u32 rows[8][4];  // rows[k][i]: byte c = state byte (i, c) of block k
    for (int k = 0; k < 8; ++k)
        transpose4(rows[k], w[k][0], w[k][1], w[k][2], w[k][3]);
    for (int i = 0; i < 4; ++i) {
        for (int k = 0; k < 8; ++k)
            q[i][7 - k] = rows[k][i];
        ortho(q[i]);
    }
}

BS_FN void store(u32 (&w)[8][4], const u32 (&q)[4][8])
{
    u32 rows[4][8];
    for (int i = 0; i < 4; ++i) {
        u32 r[8];
        for (int n = 0; n < 8; ++n)
            r[n] = q[i][n];
        ortho(r);
        for (int k = 0; k < 8; ++k)
            rows[i][k] = r[7 - k];
    }
    for (int k = 0; k < 8; ++k) {
        u32 o[4];
        transpose4(o, rows[0][k], rows[1][k], rows[2][k], rows[3][k]);
        for (int c = 0; c < 4; ++c)
            w[k][c] = o[c];
    }
}

BS_FN void sub_bytes_row(u32 (&v)[8])
{
    const u32 U0 = v[0], U1 = v[1], U2 = v[2], U3 = v[3], U4 = v[4], U5 = v[5], U6 = v[6], U7 = v[7];
#include "aes_bs_sbox.inc"
    v[0] = S0, v[1] = S1, v[2] = S2, v[3] = S3, v[4] = S4, v[5] = S5, v[6] = S6, v[7] = S7;
}

BS_FN void shift_rows(u32 (&q)[4][8])
{
    for (int i = 1; i < 4; ++i)
        for (int n = 0; n < 8; ++n)
            q[i][n] = rotr(q[i][n], 8 * i);
}

// out_i = a_i ^ t ^ xtime(a_i ^ a_(i+1)), t = a_0 ^ a_1 ^ a_2 ^ a_3 (plane n = bit 7 - n; xtime shifts toward the
// MSB plane and folds the old MSB plane into bits 4, 3, 1, 0 = planes 3, 4, 6, 7)
BS_FN void mix_columns(u32 (&q)[4][8])
{
    u32 t[8];
    for (int n = 0; n < 8; ++n)
        t[n] = q[0][n] ^ q[1][n] ^ q[2][n] ^ q[3][n];
    u32 o[4][8];
    for (int i = 0; i < 4; ++i) {
        u32 d[8];
        for (int n = 0; n < 8; ++n)
            d[n] = q[i][n] ^ q[(i + 1) & 3][n];
        const u32 x[8] = {d[1], d[2], d[3], d[4] ^ d[0], d[5] ^ d[0], d[6], d[7] ^ d[0], d[0]};
        for (int n = 0; n < 8; ++n)
            o[i][n] = q[i][n] ^ t[n] ^ x[n];
    }
    for (int i = 0; i < 4; ++i)
        for (int n = 0; n < 8; ++n)
            q[i][n] = o[i][n];
}

BS_FN void add_round_key(u32 (&q)[4][8], const u32 *kp)
{
    for (int i = 0; i < 4; ++i)
        for (int n = 0; n < 8; ++n)
            q[i][n] ^= kp[8 * i + n];
}

// key planes of one round key (LE column words rk[c], byte i = row i): 32 words, plane (i, n) at 8i + n
BS_FN void key_planes(u32 *kp, const u32 (&rk)[4])
{
    for (int i = 0; i < 4; ++i)
        for (int n = 0; n < 8; ++n) {
            u32 m = 0;
            for (int c = 0; c < 4; ++c)
                if ((rk[c] >> (8 * i + 7 - n)) & 1u)
                    m |= 0xffu << (8 * c);
            kp[8 * i + n] = m;
        }
}

// nr rounds on bit-planes; kp = (nr + 1) * 32 key-plane words
BS_FN void encrypt(u32 (&q)[4][8], const u32 *kp, int nr)
{
    add_round_key(q, kp);
    for (int r = 1; r < nr; ++r) {
        for (int i = 0; i < 4; ++i)
            sub_bytes_row(q[i]);
        shift_rows(q);
        mix_columns(q);
        add_round_key(q, kp + 32 * r);
    }
    for (int i = 0; i < 4; ++i)
        sub_bytes_row(q[i]);
    shift_rows(q);
    add_round_key(q, kp + 32 * nr);
}

}  // namespace bs
