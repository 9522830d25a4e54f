// tools/mb/microbench.hip -- component microbenchmarks (not product code): how fast can the engine's LDS-table AES
// rounds and GHASH folds run in isolation on a CU, with NB independent blocks per lane in flight?
#include "../../picotls_amd/csrc/aesgcm_engine.hip"

template <int NB>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4))) void mb_aes(const KeyEntry *keys, u32 iters, u32 *out)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    build_aes_tables(lds);
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    u32 rk[11][4];
    for (int r = 0; r <= 10; ++r)
        for (int c = 0; c < 4; ++c)
            rk[r][c] = __builtin_amdgcn_readfirstlane(keys->rk[r][c]);
    u32 acc = 0;
    u32 st[NB][4];
    for (int i = 0; i < NB; ++i)
        st[i][0] = threadIdx.x ^ rk[0][0], st[i][1] = blockIdx.x ^ rk[0][1], st[i][2] = i ^ rk[0][2], st[i][3] = rk[0][3];
    for (u32 it = 0; it < iters; ++it) {
        aes_rounds_n<10, 1, NB>(lds, laneoff, rk, st);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            acc ^= st[i][0] ^ st[i][1] ^ st[i][2] ^ st[i][3];
            st[i][3] ^= it;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NB>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4))) void mb_ghash(const KeyEntry *keys, u32 iters, u32 *out)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    build_ghash_tables(lds, keys);
    __syncthreads();
    const u32 tsel = 0x10000u | 7u * GHASH_TABLE_BYTES;
    u32x4 acc[NB];
    for (int i = 0; i < NB; ++i)
        acc[i] = u32x4{threadIdx.x, blockIdx.x, (u32)i, 0x12345678u};
    for (u32 it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            acc[i] = gmul_tab(lds, acc[i], tsel);
            acc[i][0] ^= it;
        }
    }
    u32 r = 0;
    for (int i = 0; i < NB; ++i)
        r ^= acc[i][0] ^ acc[i][1] ^ acc[i][2] ^ acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

extern "C" int mb_run(int which, int nb, const void *keys, unsigned iters, void *out, int grid, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    static int init = 0;
    if (!init) {
        hipFuncSetAttribute((const void *)mb_aes<1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC);
        hipFuncSetAttribute((const void *)mb_aes<2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC);
        hipFuncSetAttribute((const void *)mb_aes<4>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC);
        hipFuncSetAttribute((const void *)mb_ghash<1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC);
        hipFuncSetAttribute((const void *)mb_ghash<2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC);
        init = 1;
    }
    const KeyEntry *k = (const KeyEntry *)keys;
    u32 *o = (u32 *)out;
    if (which == 0) {
        if (nb == 1) mb_aes<1><<<grid, 1024, LDS_ALLOC, s>>>(k, iters, o);
        else if (nb == 2) mb_aes<2><<<grid, 1024, LDS_ALLOC, s>>>(k, iters, o);
        else mb_aes<4><<<grid, 1024, LDS_ALLOC, s>>>(k, iters, o);
    } else {
        if (nb == 1) mb_ghash<1><<<grid, 1024, LDS_ALLOC, s>>>(k, iters, o);
        else mb_ghash<2><<<grid, 1024, LDS_ALLOC, s>>>(k, iters, o);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" void *mb_keyptr(ptls_mi355x_keyset_t *ks) { return ks->d_keys; }
