/*
 * picotls_amd/csrc/ptls_mi355x.c -- the picotls plugin objects for the MI355X AES-GCM engine.
 *
 * Mirrors fusion's vtable layer (lib/fusion.c:1103-1261) on top of the engine's C ABI (include/picotls/mi355x.h):
 *   aesgcm_setup        lib/fusion.c:1189-1211  (key == NULL: IV-only update; callbacks; context tail)
 *   aead_do_encrypt     lib/fusion.c:1136-1146  -> ptls_mi355x_encrypt (+ the supplementary block, as
 *                                                  ptls_aead__do_encrypt does, include/picotls.h:2136-2146)
 *   aead_do_decrypt     lib/fusion.c:1154-1171  -> ptls_mi355x_decrypt (inlen < 16 -> SIZE_MAX)
 *   aesgcm_get/set_iv   lib/fusion.c:1173-1187
 *   ctr cipher          lib/fusion.c:1051-1101  (one 16-byte AES-CTR block per init, for QUIC header protection)
 *   quiclb cipher       lib/fusion.c:2186-2233  (QUIC-LB CID encryption, lib/quiclb-impl.h)
 * Unlike fusion, do_encrypt_v (TLS over TCP) is implemented: the iovecs are gathered straight into the staging buffer and
 * sealed as one record.
 *
 * Constant time. fusion's AES and GHASH are AES-NI / PCLMUL (lib/fusion.c:157-186, :323-335): their timing does not depend on
 * keys or data. The AEAD objects here therefore put their keysets in the engine's constant-time mode (every LDS access
 * with a data-independent bank pattern, include/picotls/mi355x.h ptls_mi355x_keyset_set_constant_time) unless the
 * environment sets PTLS_MI355X_CONSTANT_TIME=0. Since round 4 that is also the engine's own default for every keyset
 * (ptls_mi355x_keyset_new creates them constant-time, batch keysets included), and both settings run the same kernels
 * at the same rate; the explicit call here keeps the objects constant-time whatever that default is.
 *
 * Failure behaviour. picotls' encrypt callbacks cannot report errors (fusion asserts on OOM, lib/fusion.c:1143), so
 * every engine failure fails closed in every build: a failed seal overwrites the whole output (inlen + 16 bytes) with
 * zeros, which no peer authenticates and which holds no plaintext even when sealing in place; a cipher that cannot
 * produce its keystream (CTR / header protection, QUIC-LB) aborts, because any output it could return would leak its
 * input. Decrypt reports failures as SIZE_MAX, as for a bad tag; ptls_mi355x_last_error() tells them apart.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "picotls/mi355x_picotls.h"

_Static_assert(sizeof(ptls_iovec_t) == sizeof(ptls_mi355x_iovec_t), "ptls_iovec_t and ptls_mi355x_iovec_t share a layout");

static void engine_fatal(const char *what)
{
    fprintf(stderr, "picotls MI355X engine: %s failed: %s\n", what, ptls_mi355x_last_error());
    abort();
}

struct mi355x_aead_context {
    ptls_aead_context_t super;
    ptls_mi355x_keyset_t *ks;
    uint8_t static_iv[PTLS_AESGCM_IV_SIZE];
};

struct mi355x_ctr_context {
    ptls_cipher_context_t super;
    ptls_mi355x_keyset_t *ks;
    uint8_t bits[16];
    int is_ready;
};

/* ------------------------------------------------------------------ AES-CTR (<= 16 bytes per init) */

static void ctr_dispose(ptls_cipher_context_t *_ctx)
{
    struct mi355x_ctr_context *ctx = (struct mi355x_ctr_context *)_ctx;
    ptls_mi355x_keyset_free(ctx->ks);
    ptls_clear_memory(ctx->bits, sizeof(ctx->bits));
}

static void ctr_init(ptls_cipher_context_t *_ctx, const void *iv)
{
    struct mi355x_ctr_context *ctx = (struct mi355x_ctr_context *)_ctx;
    if (ptls_mi355x_encrypt_block(ctx->ks, 0, ctx->bits, iv) != 0)
        engine_fatal("AES-CTR keystream");
    ctx->is_ready = 1;
}

static void ctr_transform(ptls_cipher_context_t *_ctx, void *output, const void *input, size_t len)
{
    struct mi355x_ctr_context *ctx = (struct mi355x_ctr_context *)_ctx;
    if (!(ctx->is_ready && len <= 16)) /* fusion asserts the same (lib/fusion.c:1065-1073) */
        engine_fatal("CTR transform (supported once per init, up to 16 bytes)");
    ctx->is_ready = 0;
    const uint8_t *in = input;
    uint8_t *out = output;
    for (size_t i = 0; i < len; ++i)
        out[i] = in[i] ^ ctx->bits[i];
}

static int aesctr_setup(ptls_cipher_context_t *_ctx, int is_enc, const void *key, size_t key_size)
{
    (void)is_enc; /* CTR is its own inverse */
    struct mi355x_ctr_context *ctx = (struct mi355x_ctr_context *)_ctx;
    static const uint8_t zero_iv[PTLS_AESGCM_IV_SIZE] = {0};
    if ((ctx->ks = ptls_mi355x_keyset_new(key, zero_iv, 1, key_size)) == NULL)
        return PTLS_ERROR_LIBRARY;
    ctx->super.do_dispose = ctr_dispose;
    ctx->super.do_init = ctr_init;
    ctx->super.do_transform = ctr_transform;
    ctx->is_ready = 0;
    return 0;
}

static int aes128ctr_setup(ptls_cipher_context_t *ctx, int is_enc, const void *key)
{
    return aesctr_setup(ctx, is_enc, key, PTLS_AES128_KEY_SIZE);
}

static int aes256ctr_setup(ptls_cipher_context_t *ctx, int is_enc, const void *key)
{
    return aesctr_setup(ctx, is_enc, key, PTLS_AES256_KEY_SIZE);
}

/* ------------------------------------------------------------------ AES-GCM */

static int aead_constant_time(void)
{
    const char *e = getenv("PTLS_MI355X_CONSTANT_TIME");
    return !(e != NULL && strcmp(e, "0") == 0);
}

static void aesgcm_dispose_crypto(ptls_aead_context_t *_ctx)
{
    struct mi355x_aead_context *ctx = (struct mi355x_aead_context *)_ctx;
    ptls_mi355x_keyset_free(ctx->ks);
    ctx->ks = NULL;
    ptls_clear_memory(ctx->static_iv, sizeof(ctx->static_iv));
}

static void aesgcm_get_iv(ptls_aead_context_t *_ctx, void *iv)
{
    struct mi355x_aead_context *ctx = (struct mi355x_aead_context *)_ctx;
    memcpy(iv, ctx->static_iv, sizeof(ctx->static_iv));
}

static void aesgcm_set_iv(ptls_aead_context_t *_ctx, const void *iv)
{
    struct mi355x_aead_context *ctx = (struct mi355x_aead_context *)_ctx;
    memcpy(ctx->static_iv, iv, sizeof(ctx->static_iv));
    /* a wrong IV on the device would seal under a nonce the caller did not ask for: nothing safe to return */
    if (ptls_mi355x_keyset_set_iv(ctx->ks, 0, iv) != 0)
        engine_fatal("set_iv");
}

/* a seal that did not happen leaves zeros, never plaintext or a partial result, in the output */
static void seal_failed(void *output, size_t inlen, ptls_aead_supplementary_encryption_t *supp)
{
    memset(output, 0, inlen + PTLS_AESGCM_TAG_SIZE);
    if (supp != NULL)
        memset(supp->output, 0, sizeof(supp->output));
}

static int is_mi355x_ctr(ptls_cipher_context_t *c)
{
    return c->algo == &ptls_mi355x_aes128ctr || c->algo == &ptls_mi355x_aes256ctr;
}

/* a seal of one record on key 0 of ks, with the optional supplementary (header protection) block; fails closed */
static void seal_one(ptls_mi355x_keyset_t *ks, void *output, const void *input, size_t inlen, uint64_t seq, const void *aad,
                     size_t aadlen, ptls_aead_supplementary_encryption_t *supp)
{
    if (supp != NULL && is_mi355x_ctr(supp->ctx) &&
        ptls_mi355x_keyset_device(((struct mi355x_ctr_context *)supp->ctx)->ks) == ptls_mi355x_keyset_device(ks) &&
        (const uint8_t *)supp->input >= (const uint8_t *)output &&
        (const uint8_t *)supp->input + 16 <= (const uint8_t *)output + inlen + PTLS_AESGCM_TAG_SIZE) {
        /* the header-protection mask of a sample inside the sealed output, computed in the seal's round trip (fusion
         * computes it inside the seal, lib/fusion.c:425-430,636-651) */
        struct mi355x_ctr_context *hp = (struct mi355x_ctr_context *)supp->ctx;
        if (ptls_mi355x_encrypt_s(ks, 0, output, input, inlen, seq, aad, aadlen, hp->ks, 0,
                                  (size_t)((const uint8_t *)supp->input - (const uint8_t *)output), supp->output) != 0)
            seal_failed(output, inlen, supp);
        return;
    }
    if (ptls_mi355x_encrypt(ks, 0, output, input, inlen, seq, aad, aadlen) != 0) {
        seal_failed(output, inlen, supp);
        return;
    }
    if (supp != NULL) {
        /* the sample may point into the freshly written ciphertext, so it is read only now (include/picotls.h:446-449) */
        supp->ctx->do_init(supp->ctx, supp->input);
        memset(supp->output, 0, sizeof(supp->output));
        supp->ctx->do_transform(supp->ctx, supp->output, supp->output, sizeof(supp->output));
    }
}

static void aead_do_encrypt(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                            const void *aad, size_t aadlen, ptls_aead_supplementary_encryption_t *supp)
{
    seal_one(((struct mi355x_aead_context *)_ctx)->ks, output, input, inlen, seq, aad, aadlen, supp);
}

static void aead_do_encrypt_v(ptls_aead_context_t *_ctx, void *output, ptls_iovec_t *input, size_t incnt, uint64_t seq,
                              const void *aad, size_t aadlen)
{
    struct mi355x_aead_context *ctx = (struct mi355x_aead_context *)_ctx;
    if (ptls_mi355x_encrypt_v(ctx->ks, 0, output, (const ptls_mi355x_iovec_t *)input, incnt, seq, aad, aadlen) != 0) {
        size_t total = 0;
        for (size_t i = 0; i < incnt; ++i)
            total += input[i].len;
        seal_failed(output, total, NULL);
    }
}

static size_t aead_do_decrypt(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                              const void *aad, size_t aadlen)
{
    struct mi355x_aead_context *ctx = (struct mi355x_aead_context *)_ctx;
    if (inlen < 16)
        return SIZE_MAX;
    return ptls_mi355x_decrypt(ctx->ks, 0, output, input, inlen, seq, aad, aadlen);
}

static int aesgcm_setup(ptls_aead_context_t *_ctx, int is_enc, const void *key, const void *iv, size_t key_size)
{
    (void)is_enc; /* one context type serves both directions */
    struct mi355x_aead_context *ctx = (struct mi355x_aead_context *)_ctx;

    memcpy(ctx->static_iv, iv, sizeof(ctx->static_iv));
    if (key == NULL)
        return 0;

    if ((ctx->ks = ptls_mi355x_keyset_new(key, iv, 1, key_size)) == NULL)
        return PTLS_ERROR_LIBRARY;
    if (ptls_mi355x_keyset_set_constant_time(ctx->ks, aead_constant_time()) != 0) {
        ptls_mi355x_keyset_free(ctx->ks);
        ctx->ks = NULL;
        return PTLS_ERROR_LIBRARY;
    }
    ctx->super.dispose_crypto = aesgcm_dispose_crypto;
    ctx->super.do_get_iv = aesgcm_get_iv;
    ctx->super.do_set_iv = aesgcm_set_iv;
    ctx->super.do_encrypt_init = NULL;
    ctx->super.do_encrypt_update = NULL;
    ctx->super.do_encrypt_final = NULL;
    ctx->super.do_encrypt = aead_do_encrypt;
    ctx->super.do_encrypt_v = aead_do_encrypt_v;
    ctx->super.do_decrypt = aead_do_decrypt;
    return 0;
}

static int aes128gcm_setup(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv)
{
    return aesgcm_setup(ctx, is_enc, key, iv, PTLS_AES128_KEY_SIZE);
}

static int aes256gcm_setup(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv)
{
    return aesgcm_setup(ctx, is_enc, key, iv, PTLS_AES256_KEY_SIZE);
}

/* ------------------------------------------------------------------ QUIC-LB CID cipher (lib/fusion.c:2186-2233) */

struct mi355x_quiclb_context {
    ptls_cipher_context_t super;
    ptls_mi355x_keyset_t *ks;
    int is_enc;
};

static void quiclb_dispose(ptls_cipher_context_t *_ctx)
{
    struct mi355x_quiclb_context *ctx = (struct mi355x_quiclb_context *)_ctx;
    ptls_mi355x_keyset_free(ctx->ks);
}

static void quiclb_init(ptls_cipher_context_t *ctx, const void *iv)
{
    (void)ctx, (void)iv;
    /* no-op, as picotls_quiclb_do_init (lib/quiclb-impl.h:102-105) */
}

static void quiclb_transform(ptls_cipher_context_t *_ctx, void *output, const void *input, size_t len)
{
    struct mi355x_quiclb_context *ctx = (struct mi355x_quiclb_context *)_ctx;
    /* the reference asserts PTLS_QUICLB_MIN_BLOCK_SIZE <= len <= PTLS_QUICLB_MAX_BLOCK_SIZE (lib/quiclb-impl.h:127) */
    if (ptls_mi355x_quiclb_transform(ctx->ks, 0, output, input, len, ctx->is_enc) != 0)
        engine_fatal("QUIC-LB transform");
}

static int quiclb_setup(ptls_cipher_context_t *_ctx, int is_enc, const void *key)
{
    struct mi355x_quiclb_context *ctx = (struct mi355x_quiclb_context *)_ctx;
    static const uint8_t zero_iv[PTLS_AESGCM_IV_SIZE] = {0};
    if ((ctx->ks = ptls_mi355x_keyset_new(key, zero_iv, 1, PTLS_QUICLB_KEY_SIZE)) == NULL)
        return PTLS_ERROR_LIBRARY;
    ctx->super.do_dispose = quiclb_dispose;
    ctx->super.do_init = quiclb_init;
    ctx->super.do_transform = quiclb_transform;
    ctx->is_enc = is_enc;
    return 0;
}

ptls_cipher_algorithm_t ptls_mi355x_quiclb = {"QUICLB", PTLS_QUICLB_KEY_SIZE, PTLS_QUICLB_DEFAULT_BLOCK_SIZE, 0,
                                              sizeof(struct mi355x_quiclb_context), quiclb_setup};

ptls_mi355x_keyset_t *ptls_mi355x_aead_get_keyset(ptls_aead_context_t *ctx)
{
    return ((struct mi355x_aead_context *)ctx)->ks;
}

/* ------------------------------------------------------------------ raw contexts (include/picotls/fusion.h:40-94) */

struct ptls_mi355x_aesgcm_context {
    ptls_mi355x_keyset_t *ks; /* key 0; its IV holds the first 4 nonce bytes of the last call, the rest zero */
    uint8_t iv_hi[4];
    size_t capacity;
    uint8_t *bounce; /* decrypt: ciphertext || tag, contiguous as the engine's open takes them (capacity + 16 bytes) */
};

ptls_mi355x_aesgcm_context_t *ptls_mi355x_aesgcm_new(const void *key, size_t key_size, size_t capacity)
{
    static const uint8_t zero_iv[PTLS_AESGCM_IV_SIZE] = {0};
    ptls_mi355x_aesgcm_context_t *ctx = calloc(1, sizeof(*ctx));
    if (ctx == NULL)
        return NULL;
    if ((ctx->bounce = malloc(capacity + PTLS_AESGCM_TAG_SIZE)) == NULL ||
        (ctx->ks = ptls_mi355x_keyset_new(key, zero_iv, 1, key_size)) == NULL ||
        ptls_mi355x_keyset_set_constant_time(ctx->ks, aead_constant_time()) != 0) {
        ptls_mi355x_aesgcm_free(ctx);
        return NULL;
    }
    ctx->capacity = capacity;
    return ctx;
}

ptls_mi355x_aesgcm_context_t *ptls_mi355x_aesgcm_set_capacity(ptls_mi355x_aesgcm_context_t *ctx, size_t capacity)
{
    if (capacity <= ctx->capacity)
        return ctx;
    uint8_t *b = malloc(capacity + PTLS_AESGCM_TAG_SIZE);
    if (b == NULL)
        return NULL;
    ptls_clear_memory(ctx->bounce, ctx->capacity + PTLS_AESGCM_TAG_SIZE);
    free(ctx->bounce);
    ctx->bounce = b;
    ctx->capacity = capacity;
    return ctx;
}

void ptls_mi355x_aesgcm_free(ptls_mi355x_aesgcm_context_t *ctx)
{
    if (ctx == NULL)
        return;
    if (ctx->ks != NULL)
        ptls_mi355x_keyset_free(ctx->ks);
    if (ctx->bounce != NULL) {
        ptls_clear_memory(ctx->bounce, ctx->capacity + PTLS_AESGCM_TAG_SIZE);
        free(ctx->bounce);
    }
    ptls_clear_memory(ctx, sizeof(*ctx));
    free(ctx);
}

/* fusion's counter register as stored -> the engine's (IV, seq) form: nonce byte i is ctr byte 15 - i; the keyset IV
 * carries nonce bytes 0-3 (updated on device only when they change: a connection's static IV keeps them), seq the
 * big-endian nonce bytes 4-11, and iv ^ (0^32 || BE64(seq)) is the nonce again (lib/picotls.c:6587-6601) */
static int raw_nonce(ptls_mi355x_aesgcm_context_t *ctx, const void *ctr, uint64_t *seq)
{
    const uint8_t *c = ctr;
    uint8_t nonce[PTLS_AESGCM_IV_SIZE];
    for (int i = 0; i < PTLS_AESGCM_IV_SIZE; ++i)
        nonce[i] = c[15 - i];
    if (memcmp(nonce, ctx->iv_hi, 4) != 0) {
        uint8_t iv[PTLS_AESGCM_IV_SIZE] = {0};
        memcpy(iv, nonce, 4);
        if (ptls_mi355x_keyset_set_iv(ctx->ks, 0, iv) != 0)
            return -1;
        memcpy(ctx->iv_hi, nonce, 4);
    }
    uint64_t s = 0;
    for (int i = 4; i < PTLS_AESGCM_IV_SIZE; ++i)
        s = s << 8 | nonce[i];
    *seq = s;
    return 0;
}

void ptls_mi355x_aesgcm_encrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                                const void *ctr, const void *aad, size_t aadlen, ptls_aead_supplementary_encryption_t *supp)
{
    uint64_t seq;
    if (inlen + aadlen > ctx->capacity || raw_nonce(ctx, ctr, &seq) != 0) { /* fusion asserts the capacity */
        seal_failed(output, inlen, supp);
        return;
    }
    seal_one(ctx->ks, output, input, inlen, seq, aad, aadlen, supp);
}

/* fusion's decrypt with a counter whose low dword is not zero (lib/fusion.c:679-682, :741): the register's low 64 bits
 * v = LE64(ctr[0..7]) advance by a 64-bit add, so E(K, J0) is taken at v + 1 and data block b at v + 2 + b, each block
 * the register byte-reversed. The output is that keystream XOR the input (written whatever the tag says); the tag
 * holds iff tag == GHASH(aad, input) ^ E(K, ctr_J0). The engine's open checks GHASH ^ E(K, nonce || 1) instead, so it is
 * handed tag ^ E(K, ctr_J0) ^ E(K, nonce || 1): it accepts exactly when fusion's decrypt would. All AES blocks are one
 * ECB launch (ptls_mi355x_encrypt_blocks); GHASH is the engine's open of the record. */
static int raw_decrypt_offset_counter(ptls_mi355x_aesgcm_context_t *ctx, uint8_t *output, const uint8_t *input, size_t inlen,
                                      const uint8_t *c, const void *aad, size_t aadlen, const uint8_t *tag)
{
    const size_t nb = (inlen + 15) / 16, nblk = nb + 2;
    uint8_t *blk = malloc(nblk * 16), *ks = malloc(nblk * 16);
    uint64_t seq, v = 0;
    int ok = 0, done = 0;
    if (blk == NULL || ks == NULL || raw_nonce(ctx, c, &seq) != 0)
        goto Exit;
    for (int i = 7; i >= 0; --i)
        v = v << 8 | c[i];
    for (size_t j = 0; j <= nb; ++j) { /* j = 0: J0 at v + 1; j = 1 + b: data block b at v + 2 + b */
        uint8_t *p = blk + 16 * j;
        const uint64_t x = v + 1 + j;
        for (int i = 0; i < 8; ++i)
            p[i] = c[15 - i], p[8 + i] = (uint8_t)(x >> (56 - 8 * i));
    }
    { /* the engine's J0 for (iv, seq): nonce || 0x00000001 */
        uint8_t *p = blk + 16 * (nb + 1);
        for (int i = 0; i < 12; ++i)
            p[i] = c[15 - i];
        p[12] = 0, p[13] = 0, p[14] = 0, p[15] = 1;
    }
    if (ptls_mi355x_encrypt_blocks(ctx->ks, 0, ks, blk, nblk) != 0)
        goto Exit;
    /* the input is staged first, so that output may alias it */
    memcpy(ctx->bounce, input, inlen);
    for (size_t i = 0; i < inlen; ++i)
        output[i] = ctx->bounce[i] ^ ks[16 + i];
    for (int i = 0; i < PTLS_AESGCM_TAG_SIZE; ++i)
        ctx->bounce[inlen + i] = tag[i] ^ ks[i] ^ ks[16 * (nb + 1) + i];
    ok = ptls_mi355x_decrypt(ctx->ks, 0, ctx->bounce, ctx->bounce, inlen + PTLS_AESGCM_TAG_SIZE, seq, aad, aadlen) == inlen;
    done = 1;
Exit:
    if (!done) /* the engine could not run: nothing decrypted, fail closed */
        memset(output, 0, inlen);
    if (ks != NULL)
        ptls_clear_memory(ks, nblk * 16);
    ptls_clear_memory(ctx->bounce, inlen + PTLS_AESGCM_TAG_SIZE);
    free(blk);
    free(ks);
    return ok;
}

int ptls_mi355x_aesgcm_decrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                               const void *ctr, const void *aad, size_t aadlen, const void *tag)
{
    uint64_t seq;
    const uint8_t *c = ctr;
    if (inlen + aadlen > ctx->capacity)
        return 0;
    if ((c[0] | c[1] | c[2] | c[3]) != 0)
        return raw_decrypt_offset_counter(ctx, output, input, inlen, c, aad, aadlen, tag);
    if (raw_nonce(ctx, ctr, &seq) != 0)
        return 0;
    memcpy(ctx->bounce, input, inlen);
    memcpy(ctx->bounce + inlen, tag, PTLS_AESGCM_TAG_SIZE);
    const size_t r = ptls_mi355x_decrypt(ctx->ks, 0, output, ctx->bounce, inlen + PTLS_AESGCM_TAG_SIZE, seq, aad, aadlen);
    ptls_clear_memory(ctx->bounce, inlen + PTLS_AESGCM_TAG_SIZE);
    return r == inlen;
}

int ptls_mi355x_aesecb_init(ptls_mi355x_aesecb_context_t *ctx, int is_enc, const void *key, size_t key_size)
{
    static const uint8_t zero_iv[PTLS_AESGCM_IV_SIZE] = {0};
    ctx->ks = NULL;
    if (!is_enc) /* fusion: assert(is_enc && "decryption is not supported (yet)"), lib/fusion.c */
        return PTLS_ERROR_NOT_AVAILABLE;
    if ((ctx->ks = ptls_mi355x_keyset_new(key, zero_iv, 1, key_size)) == NULL)
        return PTLS_ERROR_LIBRARY;
    return 0;
}

void ptls_mi355x_aesecb_dispose(ptls_mi355x_aesecb_context_t *ctx)
{
    if (ctx->ks != NULL)
        ptls_mi355x_keyset_free(ctx->ks);
    ctx->ks = NULL;
}

void ptls_mi355x_aesecb_encrypt(ptls_mi355x_aesecb_context_t *ctx, void *dst, const void *src)
{
    if (ptls_mi355x_encrypt_block(ctx->ks, 0, dst, src) != 0)
        engine_fatal("AES-ECB block");
}

ptls_cipher_algorithm_t ptls_mi355x_aes128ctr = {"AES128-CTR", PTLS_AES128_KEY_SIZE, 1, PTLS_AES_IV_SIZE,
                                                 sizeof(struct mi355x_ctr_context), aes128ctr_setup};
ptls_cipher_algorithm_t ptls_mi355x_aes256ctr = {"AES256-CTR", PTLS_AES256_KEY_SIZE, 1, PTLS_AES_IV_SIZE,
                                                 sizeof(struct mi355x_ctr_context), aes256ctr_setup};
ptls_aead_algorithm_t ptls_mi355x_aes128gcm = {"AES128-GCM",
                                               PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                               PTLS_AESGCM_INTEGRITY_LIMIT,
                                               &ptls_mi355x_aes128ctr,
                                               NULL,
                                               PTLS_AES128_KEY_SIZE,
                                               PTLS_AESGCM_IV_SIZE,
                                               PTLS_AESGCM_TAG_SIZE,
                                               {0},
                                               0,
                                               0,
                                               sizeof(struct mi355x_aead_context),
                                               aes128gcm_setup};
ptls_aead_algorithm_t ptls_mi355x_aes256gcm = {"AES256-GCM",
                                               PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                               PTLS_AESGCM_INTEGRITY_LIMIT,
                                               &ptls_mi355x_aes256ctr,
                                               NULL,
                                               PTLS_AES256_KEY_SIZE,
                                               PTLS_AESGCM_IV_SIZE,
                                               PTLS_AESGCM_TAG_SIZE,
                                               {0},
                                               0,
                                               0,
                                               sizeof(struct mi355x_aead_context),
                                               aes256gcm_setup};

/* The TLS-1.2-capable objects, counterparts of ptls_non_temporal_aes{128,256}gcm (lib/fusion.c:2159-2184): same GCM
 * callbacks, record IV sizes {4, 8} so that picotls' TLS 1.2 record layer (lib/picotls.c:779-799, :6019-6060) can use
 * them, non_temporal = 1 and 64-byte buffer alignment as fusion declares (on the GPU these are hints only: records are
 * staged through device memory either way). Unlike fusion's, both directions are available on every context. */
#define MI355X_CACHE_LINE_ALIGN_BITS 6
ptls_aead_algorithm_t ptls_mi355x_non_temporal_aes128gcm = {"AES128-GCM",
                                                            PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                                            PTLS_AESGCM_INTEGRITY_LIMIT,
                                                            &ptls_mi355x_aes128ctr,
                                                            NULL,
                                                            PTLS_AES128_KEY_SIZE,
                                                            PTLS_AESGCM_IV_SIZE,
                                                            PTLS_AESGCM_TAG_SIZE,
                                                            {PTLS_TLS12_AESGCM_FIXED_IV_SIZE, PTLS_TLS12_AESGCM_RECORD_IV_SIZE},
                                                            1,
                                                            MI355X_CACHE_LINE_ALIGN_BITS,
                                                            sizeof(struct mi355x_aead_context),
                                                            aes128gcm_setup};
ptls_aead_algorithm_t ptls_mi355x_non_temporal_aes256gcm = {"AES256-GCM",
                                                            PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                                            PTLS_AESGCM_INTEGRITY_LIMIT,
                                                            &ptls_mi355x_aes256ctr,
                                                            NULL,
                                                            PTLS_AES256_KEY_SIZE,
                                                            PTLS_AESGCM_IV_SIZE,
                                                            PTLS_AESGCM_TAG_SIZE,
                                                            {PTLS_TLS12_AESGCM_FIXED_IV_SIZE, PTLS_TLS12_AESGCM_RECORD_IV_SIZE},
                                                            1,
                                                            MI355X_CACHE_LINE_ALIGN_BITS,
                                                            sizeof(struct mi355x_aead_context),
                                                            aes256gcm_setup};
