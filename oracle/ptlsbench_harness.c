/*
 * oracle/ptlsbench_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * BASELINE.json configs[0]: picotls' own benchmark loop (t/ptlsbench.c:88-185 bench_run_one, :187-247
 * bench_run_aead) over fusion (lib/fusion.c, compiled unmodified) with its conventions kept exactly:
 *   - keys: ptls_aead_new(aead, hash, is_enc, secret = 32 x 'z', NULL) (:223-225), the hash ptlsbench pairs with the
 *     AEAD (:271-274: AES-128-GCM / SHA-256, AES-256-GCM / SHA-384; lib/openssl.c's SHA-2 here, the same function as
 *     minicrypto's);
 *   - AAD: uint64_t h[4] (32 bytes, native little endian) with h[0] = the record's sequence number (:130, :141, :156);
 *   - plaintext: all zero (:117), L bytes, BENCH_BATCH = 1000 records per batch (:86), seq counting from 1;
 *   - clock: CPU time in microseconds (bench_time, :67-81), seal and open timed separately. ptlsbench reads
 *     CLOCK_PROCESS_CPUTIME_ID in a single-threaded process; this harness runs inside a multi-threaded host (Python, the
 *     HIP runtime), so it reads the calling thread's CPU clock, which is what ptlsbench's clock measures there.
 * L is a parameter (the config asks for 16384 where :362 hard-codes 1500). Built into oracle/_ref/libtls12_ref.so
 * (links the system libcrypto for SHA-2); never linked by the product.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "picotls.h"
#include "picotls/fusion.h"
#include "picotls/openssl.h"

#define BENCH_BATCH 1000

static double cpu_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static double wall_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void pick(size_t key_size, ptls_aead_algorithm_t **aead, ptls_hash_algorithm_t **hash)
{
    *aead = key_size == 32 ? &ptls_fusion_aes256gcm : &ptls_fusion_aes128gcm;
    *hash = key_size == 32 ? &ptls_openssl_sha384 : &ptls_openssl_sha256;
}

/* The traffic key and IV ptls_aead_new derives from the secret (get_traffic_keys, lib/picotls.c:1634-1646). */
int ref_ptlsbench_keys(size_t key_size, const uint8_t *secret, uint8_t *key, uint8_t *iv)
{
    ptls_aead_algorithm_t *aead;
    ptls_hash_algorithm_t *hash;
    pick(key_size, &aead, &hash);
    int ret;
    if ((ret = ptls_hkdf_expand_label(hash, key, aead->key_size, ptls_iovec_init(secret, hash->digest_size), "key",
                                      ptls_iovec_init(NULL, 0), NULL)) != 0)
        return ret;
    return ptls_hkdf_expand_label(hash, iv, aead->iv_size, ptls_iovec_init(secret, hash->digest_size), "iv",
                                  ptls_iovec_init(NULL, 0), NULL);
}

/* bench_run_aead + bench_run_one for n records of l bytes. first_batch (may be NULL) receives the sealed records of the
 * first batch, record i at i * (l + 16). times[4] = {seal CPU us, open CPU us, seal wall s, open wall s}. Returns 0, or
 * -1 when a record fails to open (PTLS_ALERT_DECRYPT_ERROR in ptlsbench). */
int ref_ptlsbench(size_t key_size, size_t l, size_t n, uint8_t *first_batch, double *times)
{
    ptls_aead_algorithm_t *aead;
    ptls_hash_algorithm_t *hash;
    pick(key_size, &aead, &hash);
    uint8_t secret[PTLS_MAX_DIGEST_SIZE];
    memset(secret, 'z', sizeof(secret));
    ptls_aead_context_t *e = ptls_aead_new(aead, hash, 1, secret, NULL), *d = ptls_aead_new(aead, hash, 0, secret, NULL);
    uint8_t *v_in = malloc(l + 1), *v_dec = malloc(l + 1), **v_enc = calloc(BENCH_BATCH, sizeof(uint8_t *));
    int ret = e != NULL && d != NULL && v_in != NULL && v_dec != NULL && v_enc != NULL ? 0 : -1;
    for (size_t i = 0; ret == 0 && i < BENCH_BATCH; ++i)
        if ((v_enc[i] = malloc(l + PTLS_MAX_DIGEST_SIZE)) == NULL)
            ret = -1;
    uint64_t h[4] = {0, 0, 0, 0};
    double t_enc = 0, t_dec = 0, w_enc = 0, w_dec = 0;
    if (ret == 0)
        memset(v_in, 0, l);
    for (size_t k = 0; ret == 0 && k < n;) {
        size_t e_len = 0, i_max = n - k > BENCH_BATCH ? BENCH_BATCH : n - k;
        uint64_t old_h = h[0];
        double c0 = cpu_us(), w0 = wall_s();
        for (size_t i = 0; i < i_max; ++i) {
            h[0]++;
            e_len = ptls_aead_encrypt(e, v_enc[i], v_in, l, h[0], h, sizeof(h));
        }
        double c1 = cpu_us(), w1 = wall_s();
        h[0] = old_h;
        for (size_t i = 0; i < i_max; ++i) {
            h[0]++;
            if (ptls_aead_decrypt(d, v_dec, v_enc[i], e_len, h[0], h, sizeof(h)) != l) {
                ret = -1;
                break;
            }
        }
        double c2 = cpu_us(), w2 = wall_s();
        t_enc += c1 - c0, t_dec += c2 - c1, w_enc += w1 - w0, w_dec += w2 - w1;
        if (k == 0 && first_batch != NULL)
            for (size_t i = 0; i < i_max; ++i)
                memcpy(first_batch + i * (l + 16), v_enc[i], l + 16);
        k += i_max;
    }
    times[0] = t_enc, times[1] = t_dec, times[2] = w_enc, times[3] = w_dec;
    for (size_t i = 0; v_enc != NULL && i < BENCH_BATCH; ++i)
        free(v_enc[i]);
    free(v_enc);
    free(v_in);
    free(v_dec);
    if (e != NULL)
        ptls_aead_free(e);
    if (d != NULL)
        ptls_aead_free(d);
    return ret;
}
