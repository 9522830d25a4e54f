// Latency primitives of the synchronous per-record path on one MI355X: what a batch of one can cost at best.
//   hipcc --offload-arch=gfx950 -O2 tools/mb/lat.hip -o tools/mb/lat && tools/mb/lat
// Medians of 300 calls (µs): empty launch + stream sync, small H2D / D2H copies (SDMA path), a kernel that reads its
// input straight from pinned host memory (all loads in flight at once), a kernel that writes host memory.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                 \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

__global__ void empty_kernel() {}

// n bytes host -> device, 16 B per thread
__global__ void pull_kernel(const uint4 *src, uint4 *dst, size_t n16)
{
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

template <typename F>
static double med(F f, int n = 300)
{
    for (int i = 0; i < 20; ++i)
        f();
    std::vector<double> t(n);
    for (int i = 0; i < n; ++i) {
        auto a = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[n / 2];
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t cap = 4 << 20;
    uint8_t *h, *d, *hd;
    CK(hipHostMalloc((void **)&h, cap, hipHostMallocDefault));
    CK(hipMalloc((void **)&d, cap));
    CK(hipHostGetDevicePointer((void **)&hd, h, 0));
    memset(h, 1, cap);
    printf("host ptr %p device view %p\n", (void *)h, (void *)hd);
    printf("empty launch + sync           %8.1f us\n", med([&] {
               empty_kernel<<<1, 64, 0, s>>>();
               CK(hipStreamSynchronize(s));
           }));
    printf("2 empty launches + sync       %8.1f us\n", med([&] {
               empty_kernel<<<1, 64, 0, s>>>();
               empty_kernel<<<1, 64, 0, s>>>();
               CK(hipStreamSynchronize(s));
           }));
    for (size_t n : {(size_t)64, (size_t)16384, (size_t)1 << 20}) {
        printf("--- %zu B\n", n);
        printf("H2D + sync                    %8.1f us\n", med([&] {
                   CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
                   CK(hipStreamSynchronize(s));
               }));
        printf("D2H + sync                    %8.1f us\n", med([&] {
                   CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s));
                   CK(hipStreamSynchronize(s));
               }));
        printf("H2D + launch + D2H + sync     %8.1f us\n", med([&] {
                   CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
                   empty_kernel<<<1, 64, 0, s>>>();
                   CK(hipMemcpyAsync(h + n, d, n, hipMemcpyDeviceToHost, s));
                   CK(hipStreamSynchronize(s));
               }));
        const size_t n16 = n / 16;
        const unsigned blocks = (unsigned)std::min<size_t>((n16 + 255) / 256, 1024);
        printf("pull kernel (host->dev) + sync %7.1f us\n", med([&] {
                   pull_kernel<<<blocks, 256, 0, s>>>((const uint4 *)hd, (uint4 *)d, n16);
                   CK(hipStreamSynchronize(s));
               }));
        printf("push kernel (dev->host) + sync %7.1f us\n", med([&] {
                   pull_kernel<<<blocks, 256, 0, s>>>((const uint4 *)d, (uint4 *)(hd + n), n16);
                   CK(hipStreamSynchronize(s));
               }));
        printf("pull + empty + push + sync    %8.1f us\n", med([&] {
                   pull_kernel<<<blocks, 256, 0, s>>>((const uint4 *)hd, (uint4 *)d, n16);
                   empty_kernel<<<1, 64, 0, s>>>();
                   pull_kernel<<<blocks, 256, 0, s>>>((const uint4 *)d, (uint4 *)(hd + n), n16);
                   CK(hipStreamSynchronize(s));
               }));
    }
    // correctness of the host-mapped path
    for (size_t i = 0; i < 4096; ++i)
        h[i] = (uint8_t)(i * 7);
    pull_kernel<<<1, 256, 0, s>>>((const uint4 *)hd, (uint4 *)d, 256);
    pull_kernel<<<1, 256, 0, s>>>((const uint4 *)d, (uint4 *)(hd + 8192), 256);
    CK(hipStreamSynchronize(s));
    printf("round trip through host-mapped memory: %s\n", memcmp(h, h + 8192, 4096) == 0 ? "ok" : "MISMATCH");
    return 0;
}
