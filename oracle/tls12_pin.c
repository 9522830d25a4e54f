/*
 * oracle/tls12_pin.c -- TEST INFRASTRUCTURE ONLY (a checker, never linked by the product).
 *
 * Pins the expected TLS 1.2 wire bytes of `tests/c/test_vtable.c`'s tls12_test with
 * references that do not share fusion's non-temporal code:
 *   - picotls' own TLS 1.2 record layer (ptls_build_tls12_export_params -> ptls_import -> ptls_send,
 *     lib/picotls.c:770-817, tls12 branch :779-799) over ptls_openssl_aes{128,256}gcm (lib/openssl.c:2457-2488);
 *   - the bitwise SP 800-38D restatement oracle/gcm_ref.c, per record, with the key block of lib/picotls.c:5308-5346
 *     (nonce = fixed IV || explicit record IV, AAD = seq || type || version || length, :753-762, first seq 1);
 * and then sweeps fusion's non-temporal seal (lib/fusion.c:1345-1614 non_temporal_encrypt_v128, :1808-2112
 * non_temporal_encrypt_v256, chosen by ptls_fusion_can_aesni256 at context setup, :2114-2147) over
 * ptls_fusion_can_aesni256 in {0, 1}, input alignments 0..63 and output alignments 0..63, naming every combination
 * whose tag or ciphertext differs from the two references.
 *
 * Inputs: the xorshift stream of test_vtable.c:31-41 from 0x1234567, drawn as `test_vtable lasterr` draws them
 * (tls12_test, test_vtable.c:350-357: ms[48], randoms[64], data[40000], first for AES-128 then for AES-256).
 *
 * Usage: tls12_pin            the tags of record 0 from every reference + the sweep summary; exit 0 iff the OpenSSL
 *                             record layer and gcm_ref agree on every record of both streams.
 *        tls12_pin --tags     one line per key size: "<key bits> <openssl record-0 tag hex> <stream sha-free digest>"
 * Built by oracle/Makefile into oracle/_ref/tls12_pin (links libtls12_ref.so and libgcm_oracle.so).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "picotls.h"
#include "picotls/fusion.h"
#include "picotls/openssl.h"

int ref_tls12_server_keys(size_t key_size, const uint8_t *master_secret, const uint8_t *hello_randoms, uint8_t *key,
                          uint8_t *fixed_iv);
void oracle_gcm_seal(const uint8_t *key, size_t key_size, const uint8_t iv[12], uint64_t seq, const uint8_t *aad, size_t aadlen,
                     const uint8_t *in, size_t len, uint8_t *out);
extern int ptls_fusion_can_aesni256;

#define NEXT_RECORD_IV 0x1122334455667788ull /* test_vtable.c tls12_import */
#define DATA_LEN 40000

static uint64_t rs = 0x1234567;
static uint8_t rnd8(void)
{
    rs ^= rs << 13, rs ^= rs >> 7, rs ^= rs << 17;
    return (uint8_t)(rs >> 24);
}
static void rnd(void *p, size_t n)
{
    for (size_t i = 0; i < n; ++i)
        ((uint8_t *)p)[i] = rnd8();
}

static void hex(const uint8_t *p, size_t n, char *out)
{
    for (size_t i = 0; i < n; ++i)
        sprintf(out + 2 * i, "%02x", p[i]);
}

/* picotls' TLS 1.2 sender (server side) over `aead`, as test_vtable.c tls12_send */
static int tls12_send(ptls_aead_algorithm_t *aead, ptls_hash_algorithm_t *hash, const uint8_t *ms, const uint8_t *randoms,
                      const uint8_t *data, size_t len, ptls_buffer_t *out)
{
    ptls_context_t ctx;
    ptls_cipher_suite_t suite = {hash == &ptls_openssl_sha384 ? 0xc030 : 0xc02f, aead, hash, "tls12"}, *suites[2] = {&suite, NULL};
    memset(&ctx, 0, sizeof(ctx));
    ctx.random_bytes = ptls_openssl_random_bytes;
    ctx.get_time = &ptls_get_time;
    ctx.tls12_cipher_suites = suites;
    ptls_buffer_t params;
    ptls_buffer_init(&params, "", 0);
    ptls_t *tls = NULL;
    int ret = -1;
    if (ptls_build_tls12_export_params(&ctx, &params, 1, 0, &suite, ms, randoms, NEXT_RECORD_IV, NULL, ptls_iovec_init(NULL, 0)) == 0 &&
        ptls_import(&ctx, &tls, ptls_iovec_init(params.base, params.off)) == 0)
        ret = ptls_send(tls, out, data, len);
    ptls_buffer_dispose(&params);
    if (tls != NULL)
        ptls_free(tls);
    return ret;
}

/* the wire stream record by record from gcm_ref: 16384-byte records, header | explicit IV | ciphertext | tag */
static size_t gcmref_stream(size_t ks, const uint8_t *ms, const uint8_t *randoms, const uint8_t *data, size_t len, uint8_t *out)
{
    uint8_t key[32], fixed[4], iv[12] = {0};
    if (ref_tls12_server_keys(ks, ms, randoms, key, fixed) != 0)
        return 0;
    memcpy(iv, fixed, 4);
    size_t off = 0, o = 0;
    uint64_t seq = 1, riv = NEXT_RECORD_IV;
    while (off < len) {
        size_t n = len - off < 16384 ? len - off : 16384, reclen = 8 + n + 16;
        uint8_t aad[13];
        out[o] = 23, out[o + 1] = 3, out[o + 2] = 3, out[o + 3] = (uint8_t)(reclen >> 8), out[o + 4] = (uint8_t)reclen;
        for (int i = 0; i < 8; ++i)
            out[o + 5 + i] = (uint8_t)(riv >> (56 - 8 * i)), aad[i] = (uint8_t)(seq >> (56 - 8 * i));
        aad[8] = 23, aad[9] = 3, aad[10] = 3, aad[11] = (uint8_t)(n >> 8), aad[12] = (uint8_t)n;
        oracle_gcm_seal(key, ks, iv, riv, aad, 13, data + off, n, out + o + 13);
        o += 5 + reclen, off += n, ++seq, ++riv;
    }
    return o;
}

/* fusion's non-temporal seal of one record at the given alignments, path chosen by `can256` at context setup */
static int fusion_nt_record(ptls_aead_algorithm_t *nt, int can256, const uint8_t *key, const uint8_t *iv12, const uint8_t *aad,
                            const uint8_t *text, size_t n, size_t in_align, size_t out_align, const uint8_t *expect)
{
    static uint8_t inbuf[16384 + 128] __attribute__((aligned(64))), outbuf[16384 + 16 + 128] __attribute__((aligned(64)));
    const int saved = ptls_fusion_can_aesni256;
    ptls_fusion_can_aesni256 = can256;
    ptls_aead_context_t *c = ptls_aead_new_direct(nt, 1, key, iv12);
    ptls_fusion_can_aesni256 = saved;
    if (c == NULL)
        return -1;
    memcpy(inbuf + in_align, text, n);
    memset(outbuf, 0xee, sizeof(outbuf));
    ptls_aead_encrypt(c, outbuf + out_align, inbuf + in_align, n, NEXT_RECORD_IV, aad, 13);
    ptls_aead_free(c);
    return memcmp(outbuf + out_align, expect, n + 16) == 0 ? 0 : memcmp(outbuf + out_align, expect, n) == 0 ? 1 : 2;
}

int main(int argc, char **argv)
{
    const int tags_only = argc > 1 && strcmp(argv[1], "--tags") == 0;
    const int cpu = ptls_fusion_is_supported_by_cpu(); /* as test_vtable.c main: sets ptls_fusion_can_aesni256 on VAES CPUs */
    const int cpu256 = ptls_fusion_can_aesni256;
    static uint8_t data[DATA_LEN], ref[DATA_LEN + 3 * 29];
    int bad = 0;
    for (int k = 0; k < 2; ++k) {
        const size_t ks = k == 0 ? 16 : 32;
        ptls_hash_algorithm_t *hash = k == 0 ? &ptls_openssl_sha256 : &ptls_openssl_sha384;
        ptls_aead_algorithm_t *ossl = k == 0 ? &ptls_openssl_aes128gcm : &ptls_openssl_aes256gcm,
                              *nt = k == 0 ? &ptls_non_temporal_aes128gcm : &ptls_non_temporal_aes256gcm;
        uint8_t ms[48], randoms[64];
        rnd(ms, sizeof(ms)), rnd(randoms, sizeof(randoms)), rnd(data, sizeof(data));
        /* reference 1: picotls' record layer over OpenSSL */
        ptls_buffer_t wo;
        ptls_buffer_init(&wo, "", 0);
        const int so = tls12_send(ossl, hash, ms, randoms, data, sizeof(data), &wo);
        /* reference 2: gcm_ref */
        const size_t nref = gcmref_stream(ks, ms, randoms, data, sizeof(data), ref);
        const int refs_agree = so == 0 && nref == wo.off && memcmp(ref, wo.base, nref) == 0;
        bad += !refs_agree;
        char tag0[33];
        hex(ref + 5 + 8 + 16384, 16, tag0);
        if (tags_only) {
            printf("%zu %s %s\n", ks * 8, tag0, refs_agree ? "refs-agree" : "REFS-DIFFER");
            ptls_buffer_dispose(&wo);
            continue;
        }
        printf("AES-%zu: record 0 tag: openssl record layer == gcm_ref: %s; tag %s\n", ks * 8, refs_agree ? "yes" : "NO", tag0);
        /* fusion's record layer, both paths, as picotls would drive it */
        for (int c256 = 0; c256 <= cpu256; ++c256) {
            ptls_buffer_t wf;
            ptls_buffer_init(&wf, "", 0);
            ptls_fusion_can_aesni256 = c256;
            const int sf = tls12_send(nt, hash, ms, randoms, data, sizeof(data), &wf);
            ptls_fusion_can_aesni256 = cpu256;
            char t[33] = "-";
            if (sf == 0 && wf.off >= 5 + 8 + 16384 + 16)
                hex(wf.base + 5 + 8 + 16384, 16, t);
            printf("  fusion non-temporal record layer, can_aesni256=%d: stream %s, record 0 tag %s\n", c256,
                   sf == 0 && wf.off == nref && memcmp(wf.base, ref, nref) == 0 ? "== references" : "DIFFERS", t);
            ptls_buffer_dispose(&wf);
        }
        /* the alignment sweep of record 0 (and of the 7232-byte record 2) */
        uint8_t key[32], fixed[4], iv12[12] = {0};
        ref_tls12_server_keys(ks, ms, randoms, key, fixed);
        memcpy(iv12, fixed, 4);
        for (int r = 0; r < 3; r += 2) {
            const size_t roff = (size_t)r * 16384, n = r == 2 ? DATA_LEN - 2 * 16384 : 16384, wire = (size_t)r * (16384 + 29);
            uint8_t aad[13];
            for (int i = 0; i < 8; ++i)
                aad[i] = (uint8_t)((uint64_t)(1 + r) >> (56 - 8 * i));
            aad[8] = 23, aad[9] = 3, aad[10] = 3, aad[11] = (uint8_t)(n >> 8), aad[12] = (uint8_t)n;
            for (int c256 = 0; c256 <= cpu256; ++c256) {
                int ntag = 0, nct = 0, first_i = -1, first_o = -1;
                for (size_t ia = 0; ia < 64; ++ia)
                    for (size_t oa = 0; oa < 64; ++oa) {
                        /* record r's explicit IV is NEXT_RECORD_IV + r; the call passes NEXT_RECORD_IV, so the
                         * difference goes into the static IV */
                        uint8_t ivr[12];
                        const uint64_t d = (NEXT_RECORD_IV + (uint64_t)r) ^ NEXT_RECORD_IV;
                        memcpy(ivr, iv12, 12);
                        for (int i = 0; i < 8; ++i)
                            ivr[4 + i] ^= (uint8_t)(d >> (56 - 8 * i));
                        const int v = fusion_nt_record(nt, c256, key, ivr, aad, data + roff, n, ia, oa, ref + wire + 13);
                        if (v != 0 && first_i < 0)
                            first_i = (int)ia, first_o = (int)oa;
                        ntag += v == 1, nct += v == 2;
                    }
                printf("  record %d (%zu B), fusion non-temporal can_aesni256=%d over 64x64 input/output alignments: %d tag-only and %d "
                       "ciphertext differences",
                       r, n, c256, ntag, nct);
                if (first_i >= 0)
                    printf(" (first at input %% 64 = %d, output %% 64 = %d)", first_i, first_o);
                printf("\n");
            }
        }
        ptls_buffer_dispose(&wo);
    }
    if (!tags_only)
        printf("fusion supported by this CPU: %d, ptls_fusion_can_aesni256 after the cpuid check: %d\n", cpu, cpu256);
    return bad == 0 ? 0 : 1;
}
