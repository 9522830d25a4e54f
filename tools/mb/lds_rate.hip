// tools/mb/lds_rate.hip -- microbenchmark (not product code): how many T-table lookups per CU-cycle can the LDS serve
// with CH independent lookup chains per lane (each chain: rounds of 16 lookups whose results feed the next round's
// indices, like AES)? Clock from s_memtime (constant 100 MHz) against the shader clock counter s_memrealtime is not
// available, so the effective clock is read as hipDeviceProp clockRate and also reported as cycles at 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 tools/mb/lds_rate.hip -o tools/mb/lds_rate && ./tools/mb/lds_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t u32;
typedef __attribute__((address_space(3))) u32 lds_u32;

template <int CH, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void rounds(const u32 *__restrict__ gtab, u32 iters, u32 *out)
{
    extern __shared__ __attribute__((aligned(16))) u32 smem[];
    for (u32 i = threadIdx.x; i < 256 * 64; i += blockDim.x)
        smem[i] = gtab[i >> 6];
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    u32 s[CH][4];
    for (int c = 0; c < CH; ++c)
        s[c][0] = threadIdx.x * 0x9e3779b9u + c, s[c][1] = blockIdx.x * 0x85ebca6bu, s[c][2] = threadIdx.x ^ 0xc2b2ae35u,
        s[c][3] = 0x27d4eb2fu + c;
    for (u32 it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            u32 e[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                e[k] = *(const lds_u32 *)(size_t)(__builtin_amdgcn_perm(s[c][(k + (k >> 2)) & 3], laneoff,
                                                                        0x0c0c0000u | ((4u + (k & 3)) << 8)));
#pragma unroll
            for (int q = 0; q < 4; ++q)
                s[c][q] = __builtin_amdgcn_bitop3_b32(e[4 * q], e[4 * q + 1], e[4 * q + 2], 0x96) ^ e[4 * q + 3] ^ it;
        }
    }
    u32 r = 0;
    for (int c = 0; c < CH; ++c)
        r ^= s[c][0] ^ s[c][1] ^ s[c][2] ^ s[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int CH, int WAVES>
static void run(const u32 *gtab, u32 *out, int cus, double clk_ghz)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const u32 iters = 20000 / CH;
    hipLaunchKernelGGL((rounds<CH, WAVES>), dim3(cus), dim3(WAVES * 64), 65536, 0, gtab, 4u, out);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((rounds<CH, WAVES>), dim3(cus), dim3(WAVES * 64), 65536, 0, gtab, iters, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double lookups = (double)cus * WAVES * 64 * iters * 16 * CH;
    printf("chains/lane %d  waves/CU %2d: %7.3f ms  %6.2f lookups/CU-cycle at %.2f GHz (%5.1f %% of 32)\n", CH, WAVES, ms,
           lookups / (ms * 1e-3) / cus / (clk_ghz * 1e9), clk_ghz, 100.0 * lookups / (ms * 1e-3) / cus / (clk_ghz * 1e9) / 32);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}

int main()
{
    u32 h[256];
    for (int i = 0; i < 256; ++i)
        h[i] = (u32)i * 0x9e3779b1u ^ ((u32)i << 17) ^ 0x5bd1e995u;
    u32 *gtab, *out;
    (void)hipMalloc(&gtab, 4096);
    (void)hipMemcpy(gtab, h, sizeof h, hipMemcpyHostToDevice);
    int cus = 256, khz = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0);
    const double ghz = khz / 1e6;
    printf("CUs %d, clockRate %.3f GHz\n", cus, ghz);
    (void)hipMalloc(&out, (size_t)cus * 1024 * 4);
    run<1, 16>(gtab, out, cus, ghz);
    run<2, 16>(gtab, out, cus, ghz);
    run<4, 16>(gtab, out, cus, ghz);
    run<1, 8>(gtab, out, cus, ghz);
    run<2, 8>(gtab, out, cus, ghz);
    run<4, 8>(gtab, out, cus, ghz);
    run<1, 4>(gtab, out, cus, ghz);
    run<4, 4>(gtab, out, cus, ghz);
    (void)hipFree(gtab);
    (void)hipFree(out);
    return 0;
}
