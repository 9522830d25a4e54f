// Host unit test of the bitsliced AES core (tools/mb/aes_bitsliced.h) against the oracle's AES
// (oracle/gcm_ref.c): load/store round trip, and AES-128/256 of random 8-block batches. Exit status 0 = pass.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../tools/mb/aes_bitsliced.h"

extern "C" {
int oracle_aes_expand(uint8_t *rk, const uint8_t *key, size_t key_size);
void oracle_aes_encrypt_rk(const uint8_t *rk, int nr, uint8_t out[16], const uint8_t in[16]);
}

static uint64_t s = 0x1234567887654321ull;
static uint32_t rnd(void)
{
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return (uint32_t)s;
}

static uint32_t le32(const uint8_t *p) { return p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

int main(void)
{
    int fails = 0;
    // load/store are inverse
    for (int t = 0; t < 100; ++t) {
        uint32_t w[8][4], q[4][8], back[8][4];
        for (int k = 0; k < 8; ++k)
            for (int c = 0; c < 4; ++c)
                w[k][c] = rnd();
        bs::load(q, w);
        bs::store(back, q);
        fails += memcmp(w, back, sizeof(w)) != 0;
    }
    // bit layout: plane n of row i, bit 8c + k == bit (7 - n) of byte (i, c) of block k
    for (int t = 0; t < 20; ++t) {
        uint32_t w[8][4], q[4][8];
        for (int k = 0; k < 8; ++k)
            for (int c = 0; c < 4; ++c)
                w[k][c] = rnd();
        bs::load(q, w);
        for (int i = 0; i < 4; ++i)
            for (int n = 0; n < 8; ++n)
                for (int c = 0; c < 4; ++c)
                    for (int k = 0; k < 8; ++k)
                        fails += ((q[i][n] >> (8 * c + k)) & 1) != ((w[k][c] >> (8 * i + 7 - n)) & 1);
    }
    for (int ks = 16; ks <= 32; ks += 16) {
        for (int t = 0; t < 200; ++t) {
            uint8_t key[32], rkb[240], in[8][16], out[16];
            for (int i = 0; i < ks; ++i)
                key[i] = (uint8_t)rnd();
            const int nr = oracle_aes_expand(rkb, key, ks);
            uint32_t kp[15 * 32];
            for (int r = 0; r <= nr; ++r) {
                const uint32_t rk[4] = {le32(rkb + 16 * r), le32(rkb + 16 * r + 4), le32(rkb + 16 * r + 8), le32(rkb + 16 * r + 12)};
                bs::key_planes(kp + 32 * r, rk);
            }
            uint32_t w[8][4], q[4][8];
            for (int k = 0; k < 8; ++k) {
                for (int i = 0; i < 16; ++i)
                    in[k][i] = (uint8_t)rnd();
                for (int c = 0; c < 4; ++c)
                    w[k][c] = le32(in[k] + 4 * c);
            }
            bs::load(q, w);
            bs::encrypt(q, kp, nr);
            bs::store(w, q);
            for (int k = 0; k < 8; ++k) {
                oracle_aes_encrypt_rk(rkb, nr, out, in[k]);
                for (int c = 0; c < 4; ++c)
                    fails += w[k][c] != le32(out + 4 * c);
            }
        }
    }
    printf("bitsliced AES: %s (%d mismatches)\n", fails ? "FAIL" : "ok", fails);
    return fails != 0;
}
