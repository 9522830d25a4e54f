// Floor of a launch-free per-record path: a persistent "doorbell" workgroup on one CU polls a
// request word in pinned host memory, reads the staged record over PCIe, does a stand-in amount of work, writes the
// result back to pinned host memory and publishes a completion word; the calling thread spins on that word.
//   hipcc --offload-arch=gfx950 -O2 tools/mb/doorbell.hip -o tools/_bin/doorbell && tools/_bin/doorbell
// Prints medians / p99 of 2000 calls (µs) for 16 B, 1200 B and 16 KiB records at 0 and ~2 µs of in-kernel work, beside
// the launch + stream-sync round trip the per-record path pays today, and the GPU-side split (request seen -> done) from
// the kernel's wall clock (100 MHz). The kernel exits on a stop word, after 200 ms without a request, or after 30 s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <vector>
#include <unistd.h>

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                 \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

typedef unsigned int u32;
typedef unsigned long long u64;

enum { W_REQ = 0, W_LEN = 1, W_WORK = 2, W_STOP = 3, W_DONE = 32, W_T0 = 34, W_T1 = 36, W_EXIT = 48 };
static const u32 STOP = 0xffffffffu;

__global__ void empty_kernel() {}

// ring: control words (request at [0], done at [32], one 128-byte line apart); in / out: staged record and result.
// One wave: every lane polls the same word (one request per poll), so the loop needs no barrier.
__global__ __launch_bounds__(64) void doorbell_kernel(u32 *ring, const uint4 *in, uint4 *out)
{
    __shared__ u32 tab[1024];
    for (u32 i = threadIdx.x; i < 1024; i += 64)
        tab[i] = i * 2654435761u;
    if (threadIdx.x == 0)
        __hip_atomic_store(ring + W_EXIT + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // started
    u32 last = 0;
    const u64 born = wall_clock64();
    u64 idle_from = born;
    for (;;) {
        const u32 v = __hip_atomic_load(ring + W_REQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const u64 now = wall_clock64();
        if (v == STOP || now - idle_from > 20000000ull || now - born > 3000000000ull)  // 200 ms idle / 30 s alive
            break;
        if (v == last)
            continue;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const u32 len = __hip_atomic_load(ring + W_LEN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const u32 work = __hip_atomic_load(ring + W_WORK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const u64 t0 = wall_clock64();
        const u32 n16 = (len + 15) / 16;
        for (u32 i = threadIdx.x; i < n16; i += 64) {
            uint4 x = in[i];
            u32 h = x.x ^ v;
            for (u32 k = 0; k < work; ++k)  // stand-in work: a dependent chain of LDS lookups (~AES rounds)
                h = tab[(h ^ k) & 1023] ^ (h >> 3);
            x.x ^= h;
            out[i] = x;
        }
        if (threadIdx.x == 0) {
            *(u64 *)(out + 4096) = t0;
            *(u64 *)(out + 4097) = wall_clock64();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (threadIdx.x == 0)
            __hip_atomic_store(ring + W_DONE, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last = v;
        idle_from = wall_clock64();
    }
    if (threadIdx.x == 0)
        __hip_atomic_store(ring + W_EXIT, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double pct(std::vector<double> v, double p)
{
    std::sort(v.begin(), v.end());
    return v[(size_t)(p * (v.size() - 1))];
}

int main()
{
    setvbuf(stdout, NULL, _IONBF, 0);
    hipStream_t s, sl;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sl, hipStreamNonBlocking));
    const size_t cap = 1 << 20;
    uint8_t *h, *hd, *src, *dst;
    CK(hipHostMalloc((void **)&h, 3 * cap, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void **)&hd, h, 0));
    src = (uint8_t *)malloc(cap);
    dst = (uint8_t *)malloc(cap);
    memset(h, 0, 3 * cap);
    for (size_t i = 0; i < cap; ++i)
        src[i] = (uint8_t)(i * 7 + 1);
    std::atomic<u32> *ring = (std::atomic<u32> *)h;
    uint8_t *hin = h + cap, *hout = h + 2 * cap;

    {  // today's floor: launch + stream sync
        std::vector<double> t;
        for (int i = 0; i < 2000; ++i) {
            auto a = std::chrono::steady_clock::now();
            empty_kernel<<<1, 64, 0, sl>>>();
            CK(hipStreamSynchronize(sl));
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        printf("empty launch + stream sync: p50 %.1f us  p99 %.1f us\n", pct(t, 0.5), pct(t, 0.99));
    }
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    u32 seq = 0;
    doorbell_kernel<<<1, 64, 0, s>>>((u32 *)hd, (const uint4 *)(hd + cap), (uint4 *)(hd + 2 * cap));
    CK(hipGetLastError());
    const u32 lens[] = {16, 1200, 16384};
    const u32 works[] = {0, 64};
    for (u32 work : works)
        for (u32 len : lens) {
            std::vector<double> t, g, up, down;
            for (int i = 0; i < 2200; ++i) {
                auto a = std::chrono::steady_clock::now();
                memcpy(hin, src, len);
                ring[W_LEN].store(len, std::memory_order_relaxed);
                ring[W_WORK].store(work, std::memory_order_relaxed);
                ++seq;
                ring[W_REQ].store(seq, std::memory_order_release);
                auto b = std::chrono::steady_clock::now();
                while (ring[W_DONE].load(std::memory_order_acquire) != seq) {
                    if (std::chrono::steady_clock::now() - b > std::chrono::seconds(1)) {
                        fprintf(stderr, "no completion for request %u (started %u, exited %u)\n", seq,
                                ring[W_EXIT + 1].load(), ring[W_EXIT].load());
                        ring[W_REQ].store(STOP, std::memory_order_release);
                        _exit(2);
                    }
                }
                memcpy(dst, hout, len);
                auto c = std::chrono::steady_clock::now();
                if (i >= 200) {
                    t.push_back(std::chrono::duration<double, std::micro>(c - a).count());
                    const u64 t0 = *(volatile u64 *)(hout + 65536), t1 = *(volatile u64 *)(hout + 65536 + 16);
                    g.push_back((t1 - t0) / 100.0);
                    (void)b;
                }
            }
            printf("doorbell %5u B work %2u: round trip p50 %.2f us  p99 %.2f us | in-kernel (seen -> done) p50 %.2f us\n",
                   len, work, pct(t, 0.5), pct(t, 0.99), pct(g, 0.5));
        }
    ring[W_REQ].store(STOP, std::memory_order_release);
    CK(hipStreamSynchronize(s));
    printf("doorbell kernel exited: %u (CUs %d)\n", ring[W_EXIT].load(), ncu);
    return 0;
}
