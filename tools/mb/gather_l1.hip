// tools/mb/gather_l1.hip -- microbenchmark (not product code): can T-table lookups be split between the LDS and the
// vector L1 cache? Each lane runs a chain of "rounds"; a round makes 16 independent 4-byte lookups into a 1 KiB table
// (index = one byte of the state) and XOR-combines them, like an AES T-table round. MODE selects where the lookups go:
// the first NG lookups of a round are global loads (table in HBM, L1/L2 resident), the rest LDS reads (32-bank
// replicated copy, conflict-free). Reports lookups per CU-cycle for each split.
//   hipcc --offload-arch=gfx950 -O3 tools/mb/gather_l1.hip -o tools/mb/gather_l1 && ./tools/mb/gather_l1
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef uint32_t u32;
typedef __attribute__((address_space(3))) u32 lds_u32;

template <int NG>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4))) void rounds(const u32 *__restrict__ gtab, u32 iters, u32 *out)
{
    extern __shared__ __attribute__((aligned(16))) u32 smem[];
    for (u32 i = threadIdx.x; i < 256 * 64; i += blockDim.x)
        smem[i] = gtab[i >> 6];  // entry n replicated at n*256 + bank*4 (banks 0..31 used)
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    u32 s[4] = {threadIdx.x * 0x9e3779b9u, blockIdx.x * 0x85ebca6bu, threadIdx.x ^ 0xc2b2ae35u, 0x27d4eb2fu};
    for (u32 it = 0; it < iters; ++it) {
        u32 e[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const u32 x = (s[(k + (k >> 2)) & 3] >> (8 * (k & 3))) & 0xffu;
            if (k < NG)
                e[k] = __builtin_nontemporal_load(gtab + x) ;
            else
                e[k] = *(const lds_u32 *)(size_t)(__builtin_amdgcn_perm(s[(k + (k >> 2)) & 3], laneoff, 0x0c0c0000u | ((4u + (k & 3)) << 8)) );
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
            s[c] = (e[4 * c] ^ e[4 * c + 1]) ^ (e[4 * c + 2] ^ e[4 * c + 3]) ^ it;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

template <int NG>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4))) void rounds_cached(const u32 *__restrict__ gtab, u32 iters, u32 *out)
{
    extern __shared__ __attribute__((aligned(16))) u32 smem[];
    for (u32 i = threadIdx.x; i < 256 * 64; i += blockDim.x)
        smem[i] = gtab[i >> 6];
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    u32 s[4] = {threadIdx.x * 0x9e3779b9u, blockIdx.x * 0x85ebca6bu, threadIdx.x ^ 0xc2b2ae35u, 0x27d4eb2fu};
    for (u32 it = 0; it < iters; ++it) {
        u32 e[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const u32 x = (s[(k + (k >> 2)) & 3] >> (8 * (k & 3))) & 0xffu;
            if (k < NG)
                e[k] = gtab[x];
            else
                e[k] = *(const lds_u32 *)(size_t)(__builtin_amdgcn_perm(s[(k + (k >> 2)) & 3], laneoff, 0x0c0c0000u | ((4u + (k & 3)) << 8)) );
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
            s[c] = (e[4 * c] ^ e[4 * c + 1]) ^ (e[4 * c + 2] ^ e[4 * c + 3]) ^ it;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

template <typename K>
static void run(const char *name, K kern, const u32 *gtab, u32 *out, int grid, u32 iters, int ng)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), 65536, 0, gtab, 4u, out);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), 65536, 0, gtab, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double lookups = (double)grid * 1024 * iters * 16;
    const double clk = 2.0e9;  // nominal; compare rows, not absolutes
    printf("%-16s NG=%2d  %8.3f ms  %7.2f G lookups/s  %6.2f lookups/CU-clk@2GHz (LDS part %5.2f, L1 part %5.2f)\n", name, ng, ms,
           lookups / ms / 1e6, lookups / (ms * 1e-3) / grid / clk, lookups * (16 - ng) / 16 / (ms * 1e-3) / grid / clk,
           lookups * ng / 16 / (ms * 1e-3) / grid / clk);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main()
{
    u32 h[256];
    for (int i = 0; i < 256; ++i)
        h[i] = (u32)i * 0x9e3779b1u ^ ((u32)i << 17) ^ 0x5bd1e995u;
    u32 *gtab, *out;
    hipMalloc(&gtab, 4096);
    hipMemcpy(gtab, h, sizeof h, hipMemcpyHostToDevice);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipMalloc(&out, (size_t)cus * 1024 * 4);
    const u32 iters = 20000;
#define R(N) run("nt-global", rounds<N>, gtab, out, cus, iters, N); run("global", rounds_cached<N>, gtab, out, cus, iters, N);
    R(0) R(1) R(2) R(4) R(6) R(8) R(16)
    hipFree(gtab);
    hipFree(out);
    return 0;
}
