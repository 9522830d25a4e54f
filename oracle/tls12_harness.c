/*
 * oracle/tls12_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives picotls' own TLS 1.2 record layer (lib/picotls.c, compiled unmodified from /root/reference) with fusion's
 * TLS-1.2-capable AEADs ptls_non_temporal_aes{128,256}gcm (lib/fusion.c:2159-2184, record IV sizes {4, 8}), so that
 * the MI355X batch TLS 1.2 framing (ptls_mi355x_seal_tls12_records / _open_tls12_records) can be compared with the
 * reference's own wire bytes:
 *   send:    ptls_build_tls12_export_params (is_server = 1) -> ptls_import -> ptls_send
 *            (buffer_push_encrypted_records, lib/picotls.c:770-817, tls12 branch :779-799)
 *   receive: the same params for the client side (is_server = 0) -> ptls_import -> ptls_receive
 *            (handle_input_tls12, lib/picotls.c:6019-6080)
 * The key block is the reference's own ptls_tls12_phash over SHA-256 / SHA-384 from lib/openssl.c (also compiled
 * unmodified), as in ptls_build_tls12_export_params (:5308-5340). Built by oracle/Makefile into
 * oracle/_ref/libtls12_ref.so (links the system libcrypto); never linked by the product.
 */
#include <stdlib.h>
#include <string.h>
#include "picotls.h"
#include "picotls/fusion.h"
#include "picotls/openssl.h"

static ptls_cipher_suite_t suite128 = {0xc02f, &ptls_non_temporal_aes128gcm, &ptls_openssl_sha256, "tls12-aes128gcm-sha256"},
                           suite256 = {0xc030, &ptls_non_temporal_aes256gcm, &ptls_openssl_sha384, "tls12-aes256gcm-sha384"};

static ptls_t *import(size_t key_size, int is_server, const uint8_t *master_secret, const uint8_t *hello_randoms,
                      uint64_t next_send_record_iv, ptls_context_t *ctx, ptls_cipher_suite_t **suites)
{
    ptls_cipher_suite_t *suite = key_size == 32 ? &suite256 : &suite128;
    suites[0] = suite;
    suites[1] = NULL;
    memset(ctx, 0, sizeof(*ctx));
    ctx->random_bytes = ptls_openssl_random_bytes;
    ctx->get_time = &ptls_get_time;
    ctx->tls12_cipher_suites = suites;
    ptls_buffer_t params;
    ptls_buffer_init(&params, "", 0);
    ptls_t *tls = NULL;
    if (ptls_build_tls12_export_params(ctx, &params, is_server, 0, suite, master_secret, hello_randoms, next_send_record_iv,
                                       NULL, ptls_iovec_init(NULL, 0)) == 0)
        ptls_import(ctx, &tls, ptls_iovec_init(params.base, params.off));
    ptls_buffer_dispose(&params);
    return tls;
}

/* The server's key and fixed IV of the key block (client key | server key | client IV | server IV), :5327-5335. */
int ref_tls12_server_keys(size_t key_size, const uint8_t *master_secret, const uint8_t *hello_randoms, uint8_t *key,
                          uint8_t *fixed_iv)
{
    ptls_cipher_suite_t *suite = key_size == 32 ? &suite256 : &suite128;
    uint8_t kb[2 * (32 + 4)];
    size_t len = 2 * (key_size + PTLS_TLS12_AESGCM_FIXED_IV_SIZE);
    int ret = ptls_tls12_phash(suite->hash, kb, len, ptls_iovec_init(master_secret, PTLS_TLS12_MASTER_SECRET_SIZE),
                               "key expansion", ptls_iovec_init(hello_randoms, PTLS_HELLO_RANDOM_SIZE * 2));
    if (ret != 0)
        return ret;
    memcpy(key, kb + key_size, key_size);
    memcpy(fixed_iv, kb + 2 * key_size + PTLS_TLS12_AESGCM_FIXED_IV_SIZE, PTLS_TLS12_AESGCM_FIXED_IV_SIZE);
    return 0;
}

/* Server sends inlen application-data bytes; the wire records go to out (capacity outcap). Returns the number of
 * bytes written, or 0 on failure. The first record has sequence number 1 and explicit nonce next_send_record_iv. */
size_t ref_tls12_send(size_t key_size, const uint8_t *master_secret, const uint8_t *hello_randoms, uint64_t next_send_record_iv,
                      const uint8_t *input, size_t inlen, uint8_t *out, size_t outcap)
{
    ptls_context_t ctx;
    ptls_cipher_suite_t *suites[2];
    ptls_t *tls = import(key_size, 1, master_secret, hello_randoms, next_send_record_iv, &ctx, suites);
    size_t n = 0;
    if (tls == NULL)
        return 0;
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    if (ptls_send(tls, &buf, input, inlen) == 0 && buf.off <= outcap) {
        memcpy(out, buf.base, buf.off);
        n = buf.off;
    }
    ptls_buffer_dispose(&buf);
    ptls_free(tls);
    return n;
}

/* Client receives the server's wire records; the plaintext goes to out. Returns the plaintext length, or -(ret) of the
 * first failing ptls_receive (e.g. -PTLS_ALERT_BAD_RECORD_MAC). */
long ref_tls12_receive(size_t key_size, const uint8_t *master_secret, const uint8_t *hello_randoms, const uint8_t *input,
                       size_t inlen, uint8_t *out, size_t outcap)
{
    ptls_context_t ctx;
    ptls_cipher_suite_t *suites[2];
    ptls_t *tls = import(key_size, 0, master_secret, hello_randoms, 0, &ctx, suites);
    if (tls == NULL)
        return -1;
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    long ret = 0;
    size_t off = 0;
    while (off < inlen) {
        size_t consumed = inlen - off;
        int r = ptls_receive(tls, &buf, input + off, &consumed);
        if (r != 0) {
            ret = -(long)r;
            break;
        }
        off += consumed;
    }
    if (ret == 0) {
        if (buf.off <= outcap) {
            memcpy(out, buf.base, buf.off);
            ret = (long)buf.off;
        } else {
            ret = -1;
        }
    }
    ptls_buffer_dispose(&buf);
    ptls_free(tls);
    return ret;
}

/* ---------------------------------------------------------------- TLS 1.3 record layer
 * ptls_import of TLS 1.3 traffic secrets in the serialization of ptls_export (export_tls_params, lib/picotls.c:5262-5282,
 * TLS 1.3 block :5359-5365), then ptls_send (aead_encrypt / buffer_push_encrypted_records :728-738, :770-817) and
 * ptls_receive (:5952-5974) over fusion's ptls_non_temporal_aes{128,256}gcm: the TLS 1.3 sender seals with
 * ptls_aead_encrypt_v (payload || content type), which ptls_fusion_aes{128,256}gcm leave unimplemented
 * (aead_do_encrypt_v asserts "FIXME", lib/fusion.c:1148-1152) and the non-temporal objects implement
 * (non_temporal_encrypt_v128/256, :1345-2112). The traffic key and IV come from ptls_get_traffic_keys (the
 * HKDF-Expand-Label of setup_traffic_protection). */
static ptls_cipher_suite_t tls13_128 = {PTLS_CIPHER_SUITE_AES_128_GCM_SHA256, &ptls_non_temporal_aes128gcm, &ptls_openssl_sha256,
                                        "TLS_AES_128_GCM_SHA256"},
                           tls13_256 = {PTLS_CIPHER_SUITE_AES_256_GCM_SHA384, &ptls_non_temporal_aes256gcm, &ptls_openssl_sha384,
                                        "TLS_AES_256_GCM_SHA384"};

static ptls_t *import13(size_t key_size, int is_server, const uint8_t *enc_secret, uint64_t enc_seq, const uint8_t *dec_secret,
                        uint64_t dec_seq, ptls_context_t *ctx, ptls_cipher_suite_t **suites)
{
    ptls_cipher_suite_t *suite = key_size == 32 ? &tls13_256 : &tls13_128;
    const size_t dsz = suite->hash->digest_size;
    static const uint8_t client_random[PTLS_HELLO_RANDOM_SIZE] = {0};
    suites[0] = suite;
    suites[1] = NULL;
    memset(ctx, 0, sizeof(*ctx));
    ctx->random_bytes = ptls_openssl_random_bytes;
    ctx->get_time = &ptls_get_time;
    ctx->cipher_suites = suites;
    ptls_buffer_t p;
    ptls_buffer_init(&p, "", 0);
    ptls_t *tls = NULL;
    int ret;
    ptls_buffer_push_block(&p, 2, {
        ptls_buffer_push(&p, (uint8_t)is_server);
        ptls_buffer_push(&p, 0);
        ptls_buffer_push16(&p, PTLS_PROTOCOL_VERSION_TLS13);
        ptls_buffer_push16(&p, suite->id);
        ptls_buffer_pushv(&p, client_random, PTLS_HELLO_RANDOM_SIZE);
        ptls_buffer_push_block(&p, 2, {});
        ptls_buffer_push_block(&p, 2, {});
        ptls_buffer_push_block(&p, 2, {
            ptls_buffer_pushv(&p, enc_secret, dsz);
            ptls_buffer_push64(&p, enc_seq);
            ptls_buffer_pushv(&p, dec_secret, dsz);
            ptls_buffer_push64(&p, dec_seq);
        });
        ptls_buffer_push_block(&p, 2, {});
    });
    ret = ptls_import(ctx, &tls, ptls_iovec_init(p.base, p.off));
    if (ret != 0)
        tls = NULL;
Exit:
    ptls_buffer_dispose(&p);
    return tls;
}

/* key and IV of the send direction of a server holding traffic secret `secret` (32 / 48 bytes) */
int ref_tls13_traffic_keys(size_t key_size, const uint8_t *secret, uint8_t *key, uint8_t *iv)
{
    ptls_context_t ctx;
    ptls_cipher_suite_t *suites[2];
    uint8_t other[64] = {0};
    ptls_t *tls = import13(key_size, 1, secret, 0, other, 0, &ctx, suites);
    uint64_t seq;
    if (tls == NULL)
        return -1;
    int ret = ptls_get_traffic_keys(tls, 1, key, iv, &seq);
    ptls_free(tls);
    return ret;
}

/* server sends `inlen` application-data bytes with traffic secret `secret`, first record sequence number `seq` */
size_t ref_tls13_send(size_t key_size, const uint8_t *secret, uint64_t seq, const uint8_t *input, size_t inlen, uint8_t *out,
                      size_t outcap)
{
    ptls_context_t ctx;
    ptls_cipher_suite_t *suites[2];
    uint8_t other[64] = {0};
    ptls_t *tls = import13(key_size, 1, secret, seq, other, 0, &ctx, suites);
    size_t n = 0;
    if (tls == NULL)
        return 0;
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    if (ptls_send(tls, &buf, input, inlen) == 0 && buf.off <= outcap) {
        memcpy(out, buf.base, buf.off);
        n = buf.off;
    }
    ptls_buffer_dispose(&buf);
    ptls_free(tls);
    return n;
}

/* client receives the server's records (its decrypt secret = the server's `secret`); plaintext length or -(error) */
long ref_tls13_receive(size_t key_size, const uint8_t *secret, uint64_t seq, const uint8_t *input, size_t inlen, uint8_t *out,
                       size_t outcap)
{
    ptls_context_t ctx;
    ptls_cipher_suite_t *suites[2];
    uint8_t other[64] = {0};
    ptls_t *tls = import13(key_size, 0, other, 0, secret, seq, &ctx, suites);
    if (tls == NULL)
        return -1;
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    long ret = 0;
    size_t off = 0;
    while (off < inlen) {
        size_t consumed = inlen - off;
        int r = ptls_receive(tls, &buf, input + off, &consumed);
        if (r != 0) {
            ret = -(long)r;
            break;
        }
        off += consumed;
    }
    if (ret == 0) {
        if (buf.off <= outcap) {
            memcpy(out, buf.base, buf.off);
            ret = (long)buf.off;
        } else {
            ret = -1;
        }
    }
    ptls_buffer_dispose(&buf);
    ptls_free(tls);
    return ret;
}

/* as ref_tls13_send, then the send direction's key, IV and next sequence number afterwards (ptls_get_traffic_keys): from
 * seq >= 2^24 ptls_send first emits a KeyUpdate under the old key and moves to the next traffic secret
 * (lib/picotls.c:6220-6232, update_send_key :6193-6211) */
size_t ref_tls13_send_rekeyed(size_t key_size, const uint8_t *secret, uint64_t seq, const uint8_t *input, size_t inlen,
                              uint8_t *out, size_t outcap, uint8_t *key_after, uint8_t *iv_after, uint64_t *seq_after)
{
    ptls_context_t ctx;
    ptls_cipher_suite_t *suites[2];
    uint8_t other[64] = {0};
    ptls_t *tls = import13(key_size, 1, secret, seq, other, 0, &ctx, suites);
    size_t n = 0;
    if (tls == NULL)
        return 0;
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    if (ptls_send(tls, &buf, input, inlen) == 0 && buf.off <= outcap &&
        ptls_get_traffic_keys(tls, 1, key_after, iv_after, seq_after) == 0) {
        memcpy(out, buf.base, buf.off);
        n = buf.off;
    }
    ptls_buffer_dispose(&buf);
    ptls_free(tls);
    return n;
}
