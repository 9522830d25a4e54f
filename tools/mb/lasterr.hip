// Does a hipErrorNotReady from hipEventQuery / hipStreamQuery stay as the thread's "last error", so that a
// following hipGetLastError() after a correct launch reports it? (round 4: the engine checks each launch with
// hipGetLastError). Prints what hipGetLastError returns after each query.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void spin(unsigned long long cycles, int *out)
{
    const unsigned long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0)
        out[0] = 1;
}
__global__ void nop(int *out) { out[1] = 2; }

int main()
{
    int *d = nullptr;
    if (hipMalloc(&d, 64) != hipSuccess)
        return 2;
    hipStream_t s;
    hipEvent_t e;
    (void)hipStreamCreate(&s);
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    for (int round = 0; round < 2; ++round) {
        spin<<<1, 64, 0, s>>>(200000000ull, d);  // ~0.1 s at ~2 GHz
        (void)hipEventRecord(e, s);
        hipError_t q = round == 0 ? hipEventQuery(e) : hipStreamQuery(s);
        hipError_t peek = hipPeekAtLastError();
        nop<<<1, 1, 0, s>>>(d);
        hipError_t after = hipGetLastError();
        printf("%s returned %s; hipPeekAtLastError then %s; hipGetLastError after a good launch: %s\n",
               round == 0 ? "hipEventQuery" : "hipStreamQuery", hipGetErrorName(q), hipGetErrorName(peek), hipGetErrorName(after));
        (void)hipStreamSynchronize(s);
    }
    // a failing call that the caller handles (an invalid device pointer query), then a good launch
    void *p = nullptr;
    int host = 0;
    hipError_t g = hipHostGetDevicePointer(&p, &host, 0);
    nop<<<1, 1, 0, s>>>(d);
    hipError_t after = hipGetLastError();
    printf("hipHostGetDevicePointer(pageable) returned %s; hipGetLastError after a good launch: %s\n", hipGetErrorName(g),
           hipGetErrorName(after));
    (void)hipStreamSynchronize(s);
    return 0;
}
