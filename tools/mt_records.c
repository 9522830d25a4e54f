/* tools/mt_records.c -- aggregate rate of the synchronous per-record path under concurrency, without Python in the loop:
 * T pthreads, each with its own one-key keyset (a picotls context), call ptls_mi355x_encrypt on their own buffers for a
 * fixed time (after a barrier). Prints calls/s over all threads and the median / p99 call latency per record length
 * and thread count. PTLS_MI355X_COMBINE (read by the engine) selects how calls are combined across threads.
 *
 *   gcc -O2 -pthread -Iinclude tools/mt_records.c -Lpicotls_amd/_lib -lptls_mi355x -Wl,-rpath,'$ORIGIN/../../picotls_amd/_lib'
 *       -o tools/_bin/mt_records      (tools/mt_build.sh)
 *   usage: mt_records [seconds] [lengths...]
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "picotls/mi355x.h"

#define MAX_THREADS 64
#define MAX_SAMPLES (1 << 20)

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec / 1e3;
}

struct job {
    int t;
    size_t len;
    ptls_mi355x_keyset_t *ks;
    uint8_t *in, *out, aad[13];
    double *lat;
    size_t n, failures;
};

static pthread_barrier_t g_start;
static volatile int g_stop;

static void *worker(void *arg)
{
    struct job *j = arg;
    for (int i = 0; i < 5; ++i) /* setup + warm-up */
        ptls_mi355x_encrypt(j->ks, 0, j->out, j->in, j->len, 1, j->aad, sizeof(j->aad));
    pthread_barrier_wait(&g_start);
    uint64_t seq = 2;
    while (!g_stop && j->n < MAX_SAMPLES) {
        double t0 = now_us();
        if (ptls_mi355x_encrypt(j->ks, 0, j->out, j->in, j->len, seq++, j->aad, sizeof(j->aad)) != 0)
            ++j->failures;
        j->lat[j->n++] = now_us() - t0;
    }
    return NULL;
}

static int cmp(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static int run(int nthreads, size_t len, double seconds)
{
    pthread_t th[MAX_THREADS];
    struct job jobs[MAX_THREADS];
    pthread_barrier_init(&g_start, NULL, nthreads + 1);
    g_stop = 0;
    for (int t = 0; t < nthreads; ++t) {
        struct job *j = &jobs[t];
        memset(j, 0, sizeof(*j));
        j->t = t, j->len = len;
        uint8_t key[16], iv[12];
        for (int i = 0; i < 16; ++i)
            key[i] = (uint8_t)(t * 31 + i * 7 + len);
        for (int i = 0; i < 12; ++i)
            iv[i] = (uint8_t)(t * 17 + i);
        if ((j->ks = ptls_mi355x_keyset_new(key, iv, 1, 16)) == NULL) {
            fprintf(stderr, "keyset_new: %s\n", ptls_mi355x_last_error());
            return 1;
        }
        j->in = calloc(len + 1, 1), j->out = malloc(len + 16), j->lat = malloc(sizeof(double) * MAX_SAMPLES);
        pthread_create(&th[t], NULL, worker, j);
    }
    pthread_barrier_wait(&g_start);
    const double t0 = now_us();
    struct timespec d = {(time_t)seconds, (long)((seconds - (time_t)seconds) * 1e9)};
    nanosleep(&d, NULL);
    g_stop = 1;
    size_t total = 0, failures = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        total += jobs[t].n, failures += jobs[t].failures;
    }
    const double dt = (now_us() - t0) / 1e6;
    double *all = malloc(sizeof(double) * (total + 1));
    size_t k = 0;
    for (int t = 0; t < nthreads; ++t) {
        memcpy(all + k, jobs[t].lat, sizeof(double) * jobs[t].n);
        k += jobs[t].n;
        ptls_mi355x_keyset_free(jobs[t].ks);
        free(jobs[t].in), free(jobs[t].out), free(jobs[t].lat);
    }
    qsort(all, total, sizeof(double), cmp);
    printf("len %6zu threads %2d: %9.0f calls/s %9.1f MiB/s  p50 %7.1f us  p99 %8.1f us%s\n", len, nthreads, total / dt,
           total / dt * len / 1048576.0, total ? all[total / 2] : 0.0, total ? all[total * 99 / 100] : 0.0,
           failures ? "  FAILURES" : "");
    fflush(stdout);
    free(all);
    pthread_barrier_destroy(&g_start);
    return failures != 0;
}

int main(int argc, char **argv)
{
    double seconds = argc > 1 ? atof(argv[1]) : 1.0;
    size_t lens[8] = {16, 1200, 16384};
    int nlens = 3;
    if (argc > 2) {
        nlens = 0;
        for (int i = 2; i < argc && nlens < 8; ++i)
            lens[nlens++] = (size_t)atol(argv[i]);
    }
    const int threads[] = {1, 2, 4, 8, 16, 32};
    const char *only = getenv("MT_THREADS"); /* one thread count instead of the sweep */
    int rc = 0;
    for (int l = 0; l < nlens; ++l)
        for (size_t t = 0; t < sizeof(threads) / sizeof(threads[0]); ++t)
            if (only == NULL || atoi(only) == threads[t])
                rc |= run(threads[t], lens[l], seconds);
    return rc;
}
