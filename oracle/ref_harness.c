/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives picotls' own lib/fusion.c (compiled unmodified from /root/reference by oracle/Makefile into
 * oracle/_ref/libfusion_ref.so) through the reference's AEAD plugin surface, exactly as its own benchmark does
 * (t/ptlsbench.c:88-185 bench_run_one: ptls_aead_encrypt / ptls_aead_decrypt per record on one context).
 *
 * Used for two things, never by the product:
 *   1. parity: byte-for-byte reference ciphertext/tags/plaintext for any record batch (tests, smoke);
 *   2. cpu_baseline (bench.py, kind "reference"): the same batches timed on the host cores, CLOCK_MONOTONIC
 *      wall time with one pinned pthread per core and a disjoint contiguous shard per thread
 *      (ptlsbench's CLOCK_PROCESS_CPUTIME_ID, t/ptlsbench.c:70-78, is not used because it sums
 *      the CPU time of all threads).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "picotls.h"
#include "picotls/fusion.h"

/* keep in sync with include/picotls/mi355x.h ptls_mi355x_record_t (40 bytes) */
typedef struct {
    uint64_t in_off, out_off, seq;
    uint32_t aad_off, len, key_idx;
    uint16_t aad_len, flags;
} ref_record_t;

int ref_cpu_supported(void)
{
    return ptls_fusion_is_supported_by_cpu();
}

static ptls_aead_algorithm_t *pick(int nontemporal, size_t key_size)
{
    if (nontemporal)
        return key_size == 32 ? &ptls_non_temporal_aes256gcm : &ptls_non_temporal_aes128gcm;
    return key_size == 32 ? &ptls_fusion_aes256gcm : &ptls_fusion_aes128gcm;
}

struct job {
    int is_seal, nontemporal, cpu;
    const uint8_t *keys, *ivs;
    size_t key_size;
    const ref_record_t *recs;
    size_t begin, end;
    const uint8_t *in, *aad;
    uint8_t *out, *ok;
    pthread_barrier_t *barrier;
    double t0, t1;
    size_t failures;
};

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *run_job(void *_j)
{
    struct job *j = _j;
    if (j->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    ptls_aead_algorithm_t *algo = pick(j->nontemporal, j->key_size);
    ptls_aead_context_t *ctx = NULL;
    uint32_t cur = UINT32_MAX;
    /* contexts are created before the clock starts when the shard uses a single key (the common case) */
    if (j->begin < j->end) {
        cur = j->recs[j->begin].key_idx;
        ctx = ptls_aead_new_direct(algo, j->is_seal, j->keys + (size_t)cur * j->key_size, j->ivs + (size_t)cur * 12);
    }
    if (j->barrier != NULL)
        pthread_barrier_wait(j->barrier);
    j->t0 = now();
    for (size_t i = j->begin; i < j->end; ++i) {
        const ref_record_t *r = j->recs + i;
        if (r->key_idx != cur) {
            ptls_aead_free(ctx);
            cur = r->key_idx;
            ctx = ptls_aead_new_direct(algo, j->is_seal, j->keys + (size_t)cur * j->key_size, j->ivs + (size_t)cur * 12);
        }
        if (j->is_seal) {
            ptls_aead_encrypt(ctx, j->out + r->out_off, j->in + r->in_off, r->len, r->seq, j->aad + r->aad_off, r->aad_len);
        } else {
            size_t ret =
                ptls_aead_decrypt(ctx, j->out + r->out_off, j->in + r->in_off, r->len + 16, r->seq, j->aad + r->aad_off, r->aad_len);
            if (j->ok != NULL)
                j->ok[i] = ret == r->len;
            if (ret != r->len)
                ++j->failures;
        }
    }
    j->t1 = now();
    if (ctx != NULL)
        ptls_aead_free(ctx);
    return NULL;
}

/* Runs seal (is_seal=1) or open over recs[0..n) with nthreads pinned threads (cpus[] lists the cores, may be NULL).
 * Returns the wall time between the common start barrier and the last thread's end, in seconds; *failures gets the number
 * of records whose tag did not verify (open only). */
double ref_run_batch(int is_seal, int nontemporal, const uint8_t *keys, const uint8_t *ivs, size_t key_size, const ref_record_t *recs,
                     size_t n, const uint8_t *in, const uint8_t *aad, uint8_t *out, uint8_t *ok, int nthreads, const int *cpus,
                     size_t *failures)
{
    if (nthreads < 1)
        nthreads = 1;
    struct job *jobs = calloc((size_t)nthreads, sizeof(*jobs));
    pthread_t *th = calloc((size_t)nthreads, sizeof(*th));
    pthread_barrier_t barrier;
    pthread_barrier_init(&barrier, NULL, (unsigned)nthreads);

    /* contiguous shards balanced by bytes */
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i)
        total += recs[i].len + 64;
    size_t pos = 0;
    uint64_t acc = 0;
    for (int t = 0; t < nthreads; ++t) {
        uint64_t target = total * (uint64_t)(t + 1) / (uint64_t)nthreads;
        size_t begin = pos;
        while (pos < n && (acc < target || t == nthreads - 1))
            acc += recs[pos++].len + 64;
        jobs[t] = (struct job){is_seal, nontemporal, cpus != NULL ? cpus[t] : -1, keys, ivs, key_size, recs, begin, pos, in, aad, out,
                               ok, &barrier};
    }
    for (int t = 0; t < nthreads; ++t)
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    double t0 = 1e300, t1 = 0;
    size_t fails = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].t0 < t0)
            t0 = jobs[t].t0;
        if (jobs[t].t1 > t1)
            t1 = jobs[t].t1;
        fails += jobs[t].failures;
    }
    pthread_barrier_destroy(&barrier);
    free(jobs);
    free(th);
    if (failures != NULL)
        *failures = fails;
    return t1 - t0;
}

/* single-record helpers through the picotls vtable (ptls_aead_new_direct / ptls_aead_encrypt / ptls_aead_decrypt) */
void ref_seal(const uint8_t *key, size_t key_size, const uint8_t *iv, uint64_t seq, const uint8_t *aad, size_t aadlen,
              const uint8_t *in, size_t len, uint8_t *out)
{
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(0, key_size), 1, key, iv);
    ptls_aead_encrypt(ctx, out, in, len, seq, aad, aadlen);
    ptls_aead_free(ctx);
}

size_t ref_open(const uint8_t *key, size_t key_size, const uint8_t *iv, uint64_t seq, const uint8_t *aad, size_t aadlen,
                const uint8_t *in, size_t inlen, uint8_t *out)
{
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(0, key_size), 0, key, iv);
    size_t ret = ptls_aead_decrypt(ctx, out, in, inlen, seq, aad, aadlen);
    ptls_aead_free(ctx);
    return ret;
}

/* raw fusion API with an explicit zero counter, as in t/fusion.c:236-344 (gcm_basic / gcm_test_vectors) */
void ref_fusion_raw_seal(const uint8_t *key, size_t key_size, const uint8_t *in, size_t len, const uint8_t *aad, size_t aadlen,
                         uint8_t *out)
{
    ptls_fusion_aesgcm_context_t *ctx = ptls_fusion_aesgcm_new(key, key_size, len + aadlen);
    ptls_fusion_aesgcm_encrypt(ctx, out, in, len, _mm_setzero_si128(), aad, aadlen, NULL);
    ptls_fusion_aesgcm_free(ctx);
}

/* QUIC header-protection mask fused into seal (ptls_aead_encrypt_s with supp, lib/fusion.c:425-430,636-651):
 * seals and writes the 16-byte AES-ECB(hp_key, sample) mask, where sample = out + sample_off (read after sealing). */
void ref_seal_with_hp(const uint8_t *key, size_t key_size, const uint8_t *iv, uint64_t seq, const uint8_t *aad, size_t aadlen,
                      const uint8_t *in, size_t len, uint8_t *out, const uint8_t *hp_key, size_t sample_off, uint8_t *mask)
{
    ptls_aead_context_t *ctx = ptls_aead_new_direct(pick(0, key_size), 1, key, iv);
    ptls_aead_supplementary_encryption_t supp;
    supp.ctx = ptls_cipher_new(key_size == 32 ? &ptls_fusion_aes256ctr : &ptls_fusion_aes128ctr, 1, hp_key);
    supp.input = out + sample_off;
    ptls_aead_encrypt_s(ctx, out, in, len, seq, aad, aadlen, &supp);
    memcpy(mask, supp.output, 16);
    ptls_cipher_free(supp.ctx);
    ptls_aead_free(ctx);
}

void ref_aesecb(const uint8_t *key, size_t key_size, uint8_t *out, const uint8_t *in)
{
    ptls_fusion_aesecb_context_t ecb;
    ptls_fusion_aesecb_init(&ecb, 1, key, key_size, 0);
    ptls_fusion_aesecb_encrypt(&ecb, out, in);
    ptls_fusion_aesecb_dispose(&ecb);
}

/* QUIC-LB through picotls' cipher API on fusion's object (ptls_fusion_quiclb, lib/fusion.c:2226-2233), as t/quiclb.c:36-45 */
void ref_quiclb(const uint8_t *key, uint8_t *out, const uint8_t *in, size_t len, int encrypt)
{
    ptls_cipher_context_t *ctx = ptls_cipher_new(&ptls_fusion_quiclb, encrypt, key);
    ptls_cipher_encrypt(ctx, out, in, len);
    ptls_cipher_free(ctx);
}
