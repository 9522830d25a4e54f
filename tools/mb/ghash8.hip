// Upper-bound probe for 8-bit GHASH windows in the Horner step: the engine's AES-CTR step (counter cache,
// T-table rounds, 16-byte loads and stores) plus one Horner multiply per block and lane, with
//   mode 0: gmul_tab on a 4-bit nibble-major H^8 table (32 ds_read_b128 per block: the engine's steady loop), or
//   mode 1: gmul8 on an 8-bit window-major table (16 ds_read_b128 per block, 64 KiB): entry (byte w, value n) at
//           0x10000 + n * 256 + w * 16; lane l = lane & 15 takes byte i ^ l of the operand at its i-th lookup (a
//           per-lane byte permutation of the operand, 12 VALU operations), so the 16 lanes of a ds_read_b128 phase read
//           16 distinct bank groups for any data.
// The 8-bit table is derived from the 4-bit one (entry(w, n) = e4(2w, n >> 4) ^ e4(2w + 1, n & 15)), so both modes must
// leave the same GHASH accumulators: the host compares them.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -mllvm -amdgpu-sched-strategy=iterative-ilp \
//       tools/mb/ghash8.hip -o tools/_bin/ghash8 && tools/_bin/ghash8 [steps]
#include "../../picotls_amd/csrc/aesgcm_engine.hip"

#include <chrono>
#include <vector>

#define MB_CK(x)                                                                                                       \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                 \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

__device__ __forceinline__ u32x4 gmul8(const lds_u8 *, u32x4 t, u32 lane, const u32 (&wreg)[8], u32 psel)
{
    const u32 l = lane & 15;
    const bool s2 = (l & 8) != 0, s1 = (l & 4) != 0;
    const u32 a0 = s2 ? t[2] : t[0], a1 = s2 ? t[3] : t[1], a2 = s2 ? t[0] : t[2], a3 = s2 ? t[1] : t[3];
    const u32 b[4] = {s1 ? a1 : a0, s1 ? a0 : a1, s1 ? a3 : a2, s1 ? a2 : a3};
    u32 p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        p[k] = __builtin_amdgcn_perm(b[k], b[k], psel);  // byte c <- byte c ^ (l & 3)
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (u32 i = 0; i < 16; i += 2) {
        const u32x4 e0 = lds_load128(__builtin_amdgcn_perm(p[i >> 2], wreg[i >> 1], 0x0c020000u | ((4u + (i & 3)) << 8)));
        const u32x4 e1 =
            lds_load128(__builtin_amdgcn_perm(p[i >> 2], wreg[i >> 1], 0x0c020001u | ((4u + ((i + 1) & 3)) << 8)));
#pragma unroll
        for (int c = 0; c < 4; ++c)
            acc[c] = xor3(acc[c], e0[c], e1[c]);
    }
    return acc;
}

template <int MODE>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4))) void mb_gcm(const u32x4 *in, u32x4 *out, u32 steps,
                                                                                          u32x4 *sink, const u32 *rkg,
                                                                                          const u32x4 *tab4)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    build_aes_tables(lds);
    if (MODE == 0) {
        for (u32 i = threadIdx.x; i < 512; i += blockDim.x)
            ((lds_u32x4 *)(lds + 0x10000 + 7 * 8192))[i] = tab4[i];
    } else {
        for (u32 i = threadIdx.x; i < 4096; i += blockDim.x) {
            const u32 w = i & 15, n = i >> 4;
            ((lds_u32x4 *)(lds + 0x10000))[i] = tab4[(2 * w) * 16 + (n >> 4)] ^ tab4[(2 * w + 1) * 16 + (n & 15)];
        }
    }
    __syncthreads();
    u32 rk[11][4];
#pragma unroll
    for (int r = 0; r <= 10; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            rk[r][c] = __builtin_amdgcn_readfirstlane(rkg[4 * r + c]);
    const u32 lane = lane_here(), laneoff = (lane & 31) * 4, l = lane & 15;
    u32 wreg[8];
#pragma unroll
    for (u32 k = 0; k < 8; ++k)
        wreg[k] = (((2 * k) ^ l) << 4) | ((((2 * k + 1) ^ l) << 4) << 8) | 0x010000u;
    const u32 lb = l & 3, psel = lb | ((1 ^ lb) << 8) | ((2 ^ lb) << 16) | ((3 ^ lb) << 24);
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nthr = (size_t)gridDim.x * blockDim.x;
    const u32 n0 = 0x01234567u ^ (u32)(gid >> 3) ^ rk[0][0], n1 = 0x89abcdefu ^ rk[0][1], n2 = 0x0badf00du ^ rk[0][2];
    u32x4 acc = {0, 0, 0, 0};
    u32 ctr = 2 + (lane & 7);
    CtrCache1 cc = {};
    u32 cc_key = 0xffffffffu;
    for (u32 m = 0; m < steps; ++m) {
        const u32x4 x = in[(size_t)m * nthr + gid];
        u32 st[1][4] = {{n0, n1, n2, bswap32(ctr) ^ rk[0][3]}};
        if ((ctr >> 8) != cc_key) {
            cc = ctr_cache1_init<10>(lds, laneoff, rk, n0, n1, n2, st[0][3]);
            cc_key = ctr >> 8;
        }
        aes_ctr_cached1<10>(lds, laneoff, rk, cc, st);
        __builtin_amdgcn_sched_barrier(0);
        const u32x4 o = x ^ u32x4{st[0][0], st[0][1], st[0][2], st[0][3]};
        out[(size_t)m * nthr + gid] = o;
        __builtin_amdgcn_sched_barrier(0);
        acc = MODE == 0 ? gmul_tab(lds, acc ^ o, 0x10000u + 7u * 8192u) : gmul8(lds, acc ^ o, lane, wreg, psel);
        __builtin_amdgcn_sched_barrier(0);
        ctr += 8;
    }
    sink[gid] = acc;
}

int main(int argc, char **argv)
{
    setvbuf(stdout, NULL, _IONBF, 0);
    const u32 steps = argc > 1 ? (u32)atoi(argv[1]) : 512;
    int ncu = 0;
    MB_CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t nthr = (size_t)ncu * 1024, n = nthr * steps;
    u32x4 *in, *out, *sink0, *sink1, *tab4;
    u32 *rk;
    MB_CK(hipMalloc(&in, n * 16));
    MB_CK(hipMalloc(&out, n * 16));
    MB_CK(hipMalloc(&sink0, nthr * 16));
    MB_CK(hipMalloc(&sink1, nthr * 16));
    MB_CK(hipMalloc(&tab4, 8192));
    MB_CK(hipMalloc(&rk, 44 * 4));
    MB_CK(hipMemset(in, 0x5a, n * 16));
    std::vector<u32> h(2048);
    u32 s = 12345;
    for (auto &v : h)
        v = (s = s * 1664525u + 1013904223u);
    MB_CK(hipMemcpy(tab4, h.data(), 8192, hipMemcpyHostToDevice));
    MB_CK(hipMemcpy(rk, h.data() + 100, 44 * 4, hipMemcpyHostToDevice));
    MB_CK(hipFuncSetAttribute((const void *)mb_gcm<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 0x20000));
    MB_CK(hipFuncSetAttribute((const void *)mb_gcm<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 0x20000));
    hipEvent_t e0, e1;
    MB_CK(hipEventCreate(&e0));
    MB_CK(hipEventCreate(&e1));
    double best[2] = {1e30, 1e30}, sum[2] = {0, 0};
    const int reps = 7;
    for (int r = 0; r <= reps; ++r)
        for (int mode = 0; mode < 2; ++mode) {
            MB_CK(hipEventRecord(e0));
            if (mode == 0)
                mb_gcm<0><<<ncu, 1024, 0x20000>>>(in, out, steps, sink0, rk, tab4);
            else
                mb_gcm<1><<<ncu, 1024, 0x20000>>>(in, out, steps, sink1, rk, tab4);
            MB_CK(hipGetLastError());
            MB_CK(hipEventRecord(e1));
            MB_CK(hipEventSynchronize(e1));
            float ms = 0;
            MB_CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) {
                best[mode] = std::min(best[mode], (double)ms);
                sum[mode] += ms;
            }
        }
    std::vector<u32> a(nthr * 4), b(nthr * 4);
    MB_CK(hipMemcpy(a.data(), sink0, nthr * 16, hipMemcpyDeviceToHost));
    MB_CK(hipMemcpy(b.data(), sink1, nthr * 16, hipMemcpyDeviceToHost));
    const bool same = a == b;
    for (int mode = 0; mode < 2; ++mode) {
        const double ms = sum[mode] / reps;
        printf("mode %d (%s): %.3f ms avg, %.3f ms best, %.1f GB/s in+out, %.3e blocks/s\n", mode,
               mode == 0 ? "4-bit gmul_tab, 32 lookups" : "8-bit window-major gmul8, 16 lookups", ms, best[mode],
               2.0 * n * 16 / (ms * 1e-3) / 1e9, n / (ms * 1e-3));
    }
    printf("speedup mode 1 / mode 0: %.3f (avg)  accumulators equal: %s  (%zu lanes x %u steps)\n", sum[0] / sum[1],
           same ? "yes" : "NO", nthr, steps);
    return same ? 0 : 1;
}
