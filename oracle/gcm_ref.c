/*
 * oracle/gcm_ref.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C, table-free-in-spirit restatement of AES-GCM as picotls' fusion backend computes it, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg to check the HIP engine. Nothing under
 * picotls_amd/ links or calls this file.
 *
 * What it restates (reference file:line into h2o/picotls):
 *   - AES block encryption, 10/14 rounds      lib/fusion.c:323-335 (aesecb_encrypt), key expansion :847-917
 *   - GHASH over GF(2^128)                    lib/fusion.c:114-321 (fusion uses PCLMUL + Karatsuba + deferred
 *                                             reduction; here: SP 800-38D Algorithm 1, bit by bit)
 *   - GCM seal                                lib/fusion.c:401-659 (ptls_fusion_aesgcm_encrypt): J0 = nonce||1
 *                                             (:489-490), data counters start at 2, tag = GHASH ^ E(J0),
 *                                             length block = len(A)*8 || len(C)*8 big-endian (:469)
 *   - GCM open                                lib/fusion.c:661-845 (ptls_fusion_aesgcm_decrypt): plaintext is
 *                                             written even when the tag does not verify (:783-828, :839-841)
 *   - TLS 1.3 nonce rule                      lib/picotls.c:6587-6601 (ptls_aead__build_iv) and
 *                                             lib/fusion.c:1127-1134 (calc_counter): nonce = iv ^ (0^32 || seq_be64)
 *   - vtable semantics                        lib/fusion.c:1136-1171 (aead_do_encrypt / aead_do_decrypt:
 *                                             inlen < 16 -> SIZE_MAX)
 *   - QUIC-LB CID cipher                      lib/quiclb-impl.h:47-162 (picotls_quiclb_transform), the cipher of
 *                                             ptls_fusion_quiclb (lib/fusion.c:2186-2233); pinned by t/quiclb.c:27-30
 *
 * Parity pinning: tests/test_oracle.py checks this file against the known-answer vectors held in the
 * reference's own tests (t/fusion.c:80,85,128-227,239-280,310-332,353-359 and t/picotls.c ECB vectors), stored as
 * data in tests/golden/kat.json, and against vectors produced by lib/fusion.c itself compiled from
 * /root/reference (oracle/Makefile -> oracle/_ref, tests/golden/gen_golden.py -> tests/golden/fusion_vectors.json).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

/* ---------------------------------------------------------------- AES (FIPS-197) */

static uint8_t sbox[256];
static int sbox_ready;

static uint8_t gf8_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b != 0) {
        if (b & 1)
            r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

/* S-box derived from its definition (multiplicative inverse in GF(2^8) followed by the affine map), FIPS-197 §5.1.1 */
static void sbox_init(void)
{
    if (sbox_ready)
        return;
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x != 0) {
            for (int y = 1; y < 256; ++y) {
                if (gf8_mul((uint8_t)x, (uint8_t)y) == 1) {
                    inv = (uint8_t)y;
                    break;
                }
            }
        }
        uint8_t s = inv;
        for (int i = 1; i <= 4; ++i)
            s ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
        sbox[x] = s ^ 0x63;
    }
    sbox_ready = 1;
}

/* key expansion, FIPS-197 §5.2; returns number of rounds. rk must hold (rounds+1)*16 bytes */
int oracle_aes_expand(uint8_t *rk, const uint8_t *key, size_t key_size)
{
    sbox_init();
    int nk = (int)(key_size / 4), nr = nk + 6;
    uint8_t rcon = 1;
    memcpy(rk, key, key_size);
    for (int i = nk; i < 4 * (nr + 1); ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            uint8_t t0 = t[0];
            t[0] = sbox[t[1]] ^ rcon;
            t[1] = sbox[t[2]];
            t[2] = sbox[t[3]];
            t[3] = sbox[t0];
            rcon = gf8_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            for (int j = 0; j < 4; ++j)
                t[j] = sbox[t[j]];
        }
        for (int j = 0; j < 4; ++j)
            rk[4 * i + j] = rk[4 * (i - nk) + j] ^ t[j];
    }
    return nr;
}

/* cipher, FIPS-197 §5.1; state byte (r,c) = s[4c + r] */
void oracle_aes_encrypt_rk(const uint8_t *rk, int nr, uint8_t out[16], const uint8_t in[16])
{
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; ++i)
        s[i] = in[i] ^ rk[i];
    for (int round = 1; round <= nr; ++round) {
        for (int i = 0; i < 16; ++i) /* SubBytes */
            s[i] = sbox[s[i]];
        for (int c = 0; c < 4; ++c) /* ShiftRows */
            for (int r = 0; r < 4; ++r)
                t[4 * c + r] = s[4 * ((c + r) % 4) + r];
        if (round != nr) {
            for (int c = 0; c < 4; ++c) { /* MixColumns */
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = gf8_mul(a0, 2) ^ gf8_mul(a1, 3) ^ a2 ^ a3;
                s[4 * c + 1] = a0 ^ gf8_mul(a1, 2) ^ gf8_mul(a2, 3) ^ a3;
                s[4 * c + 2] = a0 ^ a1 ^ gf8_mul(a2, 2) ^ gf8_mul(a3, 3);
                s[4 * c + 3] = gf8_mul(a0, 3) ^ a1 ^ a2 ^ gf8_mul(a3, 2);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; ++i) /* AddRoundKey */
            s[i] ^= rk[16 * round + i];
    }
    memcpy(out, s, 16);
}

/* one-block AES-ECB (mirrors ptls_fusion_aesecb_encrypt, lib/fusion.c:924) */
void oracle_aes_encrypt(const uint8_t *key, size_t key_size, uint8_t out[16], const uint8_t in[16])
{
    uint8_t rk[240];
    int nr = oracle_aes_expand(rk, key, key_size);
    oracle_aes_encrypt_rk(rk, nr, out, in);
}

/* ---------------------------------------------------------------- GHASH (SP 800-38D §6.3, Algorithm 1) */

/* Z = X * Y in GF(2^128) with the GCM bit order (bit 0 = MSB of byte 0) */
void oracle_gf128_mul(uint8_t z[16], const uint8_t x[16], const uint8_t y[16])
{
    uint8_t v[16], acc[16] = {0};
    memcpy(v, y, 16);
    for (int i = 0; i < 128; ++i) {
        if ((x[i / 8] >> (7 - i % 8)) & 1)
            for (int j = 0; j < 16; ++j)
                acc[j] ^= v[j];
        int lsb = v[15] & 1;
        for (int j = 15; j > 0; --j)
            v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
        v[0] >>= 1;
        if (lsb)
            v[0] ^= 0xe1;
    }
    memcpy(z, acc, 16);
}

/* Y = GHASH_H(X_1..X_m) where the data is zero-padded to a multiple of 16 bytes, folded into y */
static void ghash_update(uint8_t y[16], const uint8_t h[16], const uint8_t *data, size_t len)
{
    while (len != 0) {
        size_t n = len < 16 ? len : 16;
        for (size_t i = 0; i < n; ++i)
            y[i] ^= data[i];
        oracle_gf128_mul(y, y, h);
        data += n;
        len -= n;
    }
}

/* plain GHASH over whole 16-byte blocks (used by the GHASH known-answer tests of t/fusion.c:88-234) */
void oracle_ghash(uint8_t out[16], const uint8_t h[16], const uint8_t *data, size_t nblocks)
{
    memset(out, 0, 16);
    ghash_update(out, h, data, nblocks * 16);
}

/* ---------------------------------------------------------------- GCM (SP 800-38D §7) */

/* nonce = static_iv ^ (0^32 || seq big-endian), lib/picotls.c:6587-6601 */
void oracle_build_nonce(uint8_t nonce[12], const uint8_t iv[12], uint64_t seq)
{
    memcpy(nonce, iv, 12);
    for (int i = 0; i < 8; ++i)
        nonce[4 + i] ^= (uint8_t)(seq >> (56 - 8 * i));
}

static void gcm_core(const uint8_t *rk, int nr, const uint8_t nonce[12], const uint8_t *aad, size_t aadlen, const uint8_t *in,
                     size_t len, uint8_t *out, int is_enc, uint8_t tag[16])
{
    uint8_t h[16] = {0}, zero[16] = {0}, j0[16], ctr[16], ks[16], y[16] = {0}, lenblk[16];
    oracle_aes_encrypt_rk(rk, nr, h, zero);
    memcpy(j0, nonce, 12);
    j0[12] = 0, j0[13] = 0, j0[14] = 0, j0[15] = 1;

    ghash_update(y, h, aad, aadlen);

    /* GCTR starting at inc32(J0); GHASH over the ciphertext (input when opening, output when sealing) */
    memcpy(ctr, j0, 16);
    uint8_t cblk[16];
    for (size_t off = 0; off < len; off += 16) {
        uint32_t c = ((uint32_t)ctr[12] << 24 | (uint32_t)ctr[13] << 16 | (uint32_t)ctr[14] << 8 | ctr[15]) + 1;
        ctr[12] = (uint8_t)(c >> 24), ctr[13] = (uint8_t)(c >> 16), ctr[14] = (uint8_t)(c >> 8), ctr[15] = (uint8_t)c;
        oracle_aes_encrypt_rk(rk, nr, ks, ctr);
        size_t n = len - off < 16 ? len - off : 16;
        memset(cblk, 0, 16);
        for (size_t i = 0; i < n; ++i) {
            uint8_t x = in[off + i];
            uint8_t o = x ^ ks[i];
            cblk[i] = is_enc ? o : x;
            out[off + i] = o;
        }
        for (size_t i = 0; i < 16; ++i)
            y[i] ^= cblk[i];
        oracle_gf128_mul(y, y, h);
    }

    uint64_t abits = (uint64_t)aadlen * 8, cbits = (uint64_t)len * 8;
    for (int i = 0; i < 8; ++i) {
        lenblk[i] = (uint8_t)(abits >> (56 - 8 * i));
        lenblk[8 + i] = (uint8_t)(cbits >> (56 - 8 * i));
    }
    for (int i = 0; i < 16; ++i)
        y[i] ^= lenblk[i];
    oracle_gf128_mul(y, y, h);

    oracle_aes_encrypt_rk(rk, nr, ks, j0);
    for (int i = 0; i < 16; ++i)
        tag[i] = y[i] ^ ks[i];
}

/* seal: writes len bytes of ciphertext followed by the 16-byte tag into out (ptls_aead_encrypt semantics,
 * include/picotls.h:2102-2107); out may alias in. */
void oracle_gcm_seal(const uint8_t *key, size_t key_size, const uint8_t iv[12], uint64_t seq, const uint8_t *aad, size_t aadlen,
                     const uint8_t *in, size_t len, uint8_t *out)
{
    uint8_t rk[240], nonce[12];
    int nr = oracle_aes_expand(rk, key, key_size);
    oracle_build_nonce(nonce, iv, seq);
    gcm_core(rk, nr, nonce, aad, aadlen, in, len, out, 1, out + len);
}

/* open: in holds inlen bytes = ciphertext || tag. Returns plaintext length, or SIZE_MAX on failure
 * (ptls_aead_decrypt semantics, lib/fusion.c:1154-1171). Plaintext is written even on tag mismatch. */
size_t oracle_gcm_open(const uint8_t *key, size_t key_size, const uint8_t iv[12], uint64_t seq, const uint8_t *aad, size_t aadlen,
                       const uint8_t *in, size_t inlen, uint8_t *out)
{
    if (inlen < 16)
        return SIZE_MAX;
    uint8_t rk[240], nonce[12], tag[16], rtag[16];
    size_t len = inlen - 16;
    memcpy(rtag, in + len, 16);
    int nr = oracle_aes_expand(rk, key, key_size);
    oracle_build_nonce(nonce, iv, seq);
    gcm_core(rk, nr, nonce, aad, aadlen, in, len, out, 0, tag);
    uint8_t diff = 0;
    for (int i = 0; i < 16; ++i)
        diff |= tag[i] ^ rtag[i];
    return diff == 0 ? len : SIZE_MAX;
}

/* ---------------------------------------------------------------- batch helpers (same descriptor layout as the engine) */

/* keep in sync with include/picotls/mi355x.h ptls_mi355x_record_t (40 bytes) */
typedef struct {
    uint64_t in_off, out_off, seq;
    uint32_t aad_off, len, key_idx;
    uint16_t aad_len, flags;
} oracle_record_t;

/* keys: n_keys * key_size bytes; ivs: n_keys * 12 bytes */
void oracle_seal_batch(const uint8_t *keys, const uint8_t *ivs, size_t key_size, const oracle_record_t *recs, size_t nrecs,
                       const uint8_t *in, const uint8_t *aad, uint8_t *out)
{
    uint32_t cur = UINT32_MAX;
    uint8_t rk[240];
    int nr = 0;
    for (size_t i = 0; i < nrecs; ++i) {
        const oracle_record_t *r = recs + i;
        if (r->key_idx != cur) {
            cur = r->key_idx;
            nr = oracle_aes_expand(rk, keys + (size_t)cur * key_size, key_size);
        }
        uint8_t nonce[12];
        oracle_build_nonce(nonce, ivs + (size_t)cur * 12, r->seq);
        gcm_core(rk, nr, nonce, aad + r->aad_off, r->aad_len, in + r->in_off, r->len, out + r->out_off, 1,
                 out + r->out_off + r->len);
    }
}

void oracle_open_batch(const uint8_t *keys, const uint8_t *ivs, size_t key_size, const oracle_record_t *recs, size_t nrecs,
                       const uint8_t *in, const uint8_t *aad, uint8_t *out, uint8_t *ok)
{
    uint32_t cur = UINT32_MAX;
    uint8_t rk[240];
    int nr = 0;
    for (size_t i = 0; i < nrecs; ++i) {
        const oracle_record_t *r = recs + i;
        if (r->key_idx != cur) {
            cur = r->key_idx;
            nr = oracle_aes_expand(rk, keys + (size_t)cur * key_size, key_size);
        }
        uint8_t nonce[12], tag[16], diff = 0;
        oracle_build_nonce(nonce, ivs + (size_t)cur * 12, r->seq);
        gcm_core(rk, nr, nonce, aad + r->aad_off, r->aad_len, in + r->in_off, r->len, out + r->out_off, 0, tag);
        for (int k = 0; k < 16; ++k)
            diff |= tag[k] ^ in[r->in_off + r->len + k];
        ok[i] = diff == 0;
    }
}

/* ---------------------------------------------------------------- QUIC-LB CID cipher (lib/quiclb-impl.h) */

/* One Feistel round (lib/quiclb-impl.h:47-70 picotls_quiclb_one_round): dest = x ^ AES((y & mask) | len_pass), with
 * len_pass = 0^112 || len || round (:133-135). Blocks are 16 bytes; only the first (len + 1) / 2 bytes of a half matter. */
static void quiclb_round(const uint8_t *rk, int nr, uint8_t dest[16], const uint8_t x[16], const uint8_t y[16],
                         const uint8_t mask[16], size_t len, int rnd)
{
    uint8_t t[16];
    for (int i = 0; i < 16; ++i)
        t[i] = y[i] & mask[i];
    t[14] |= (uint8_t)len;
    t[15] |= (uint8_t)rnd;
    oracle_aes_encrypt_rk(rk, nr, t, t);
    for (int i = 0; i < 16; ++i)
        dest[i] = t[i] ^ x[i];
}

/* picotls_quiclb_transform (lib/quiclb-impl.h:107-162) for 7 <= len <= 19 with an AES-128 key; returns -1 otherwise.
 * The masks (:111-125) are derived rather than tabulated: the left half keeps bytes [0, len/2) plus the high nibble of
 * the middle byte when len is odd; the right half keeps that middle byte's low nibble (its byte 0) and the bytes after
 * it. split (:72-84) and merge (:86-100) follow the reference byte for byte. */
int oracle_quiclb_transform(const uint8_t key[16], uint8_t *output, const uint8_t *input, size_t len, int encrypt)
{
    if (len < 7 || len > 19)
        return -1;
    uint8_t rk[240];
    const int nr = oracle_aes_expand(rk, key, 16);
    const size_t half = len / 2, hl = (len + 1) / 2, odd = len & 1;
    uint8_t ml[16] = {0}, mr[16] = {0};
    for (size_t i = 0; i < half; ++i)
        ml[i] = 0xff, mr[i + odd] = 0xff;
    if (odd)
        ml[half] = 0xf0, mr[0] = 0x0f;
    uint8_t a[16] = {0}, b[16] = {0}, l1[16], r1[16], l[16], r[16];
    for (size_t i = 0; i < hl; ++i)
        a[i] = input[i], b[i] = input[i + half];
    if (encrypt) { /* (:149-154): l0 = a, r0 = b */
        quiclb_round(rk, nr, r1, b, a, ml, len, 1);
        quiclb_round(rk, nr, l1, a, r1, mr, len, 2);
        quiclb_round(rk, nr, r, r1, l1, ml, len, 3);
        quiclb_round(rk, nr, l, l1, r, mr, len, 4);
    } else { /* (:155-161): l2 = a, r2 = b */
        quiclb_round(rk, nr, l1, a, b, mr, len, 4);
        quiclb_round(rk, nr, r1, b, l1, ml, len, 3);
        quiclb_round(rk, nr, l, l1, r1, mr, len, 2);
        quiclb_round(rk, nr, r, r1, l, ml, len, 1);
    }
    uint8_t tmp[19];
    size_t o = 0;
    for (size_t i = 0; i < half; ++i)
        tmp[o++] = l[i];
    if (odd)
        tmp[o++] = (l[half] & 0xf0) | (r[0] & 0x0f);
    for (size_t i = 0; i < half; ++i)
        tmp[o++] = r[i + odd];
    memcpy(output, tmp, len); /* output may alias input */
    return 0;
}
