// AES-CTR keystream microbenchmark: the engine's two AES implementations side by side on the same data.
//   ctr_tt  LDS T-tables (the rounds of aesgcm_engine.hip: Te0/Te2 replicated over 32 banks, v_perm addressing), one
//           block per lane per iteration
//   ctr_bs  bitsliced (tools/mb/aes_bitsliced.h), eight blocks per lane per iteration, VALU only; key
//           planes read with scalar loads
// out[i] = in[i] ^ AES_K(nonce || BE32(i + 2)) for 16-byte blocks i (the GCM counter numbering). Both kernels must give
// identical output (checked by tools/mb/aes_ctr.py). Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include tools/mb/aes_ctr.hip -o tools/mb/libaesctr.so
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aes_bitsliced.h"

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4_u;
typedef __attribute__((address_space(3))) u32 lds_u32;

__constant__ uint8_t c_sbox[256];

__device__ __forceinline__ u32 rotl8(u32 x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wint-to-pointer-cast"
__device__ __forceinline__ u32 lds32(u32 a) { return *(const lds_u32 *)a; }
#pragma clang diagnostic pop
#define TE(w, r, lo) lds32(__builtin_amdgcn_perm((w), (lo), 0x0c0c0000u | ((4u + (r)) << 8)))
#define TE2(w, r, lo) lds32(__builtin_amdgcn_perm((w), (lo), 0x0c0c0000u | ((4u + (r)) << 8)) + 128)

template <int NR>
__global__ __launch_bounds__(1024) void ctr_tt(const u32 *rkg, const uint8_t *in, uint8_t *out, u64 nblocks, u32 n0, u32 n1,
                                               u32 n2)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u32 *t = (lds_u32 *)smem;
    for (u32 idx = threadIdx.x; idx < 256 * 64; idx += blockDim.x) {
        const u32 n = idx >> 6, slot = idx & 63, s = c_sbox[n];
        const u32 s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
        const u32 te0 = s2 | s << 8 | s << 16 | (s2 ^ s) << 24;
        t[idx] = slot < 32 ? te0 : ((te0 << 16) | (te0 >> 16));
    }
    __syncthreads();
    u32 rk[NR + 1][4];
    for (int r = 0; r <= NR; ++r)
        for (int c = 0; c < 4; ++c)
            rk[r][c] = __builtin_amdgcn_readfirstlane(rkg[4 * r + c]);
    const u32 lo = (threadIdx.x & 31) * 4;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nblocks; i += (u64)gridDim.x * blockDim.x) {
        u32 s0 = n0 ^ rk[0][0], s1 = n1 ^ rk[0][1], s2 = n2 ^ rk[0][2], s3 = __builtin_bswap32((u32)i + 2) ^ rk[0][3];
#pragma unroll
        for (int r = 1; r < NR; ++r) {
            const u32 a0 = xor3(TE(s0, 0, lo), TE2(s2, 2, lo), rk[r][0]) ^ rotl8(TE(s1, 1, lo) ^ TE2(s3, 3, lo));
            const u32 a1 = xor3(TE(s1, 0, lo), TE2(s3, 2, lo), rk[r][1]) ^ rotl8(TE(s2, 1, lo) ^ TE2(s0, 3, lo));
            const u32 a2 = xor3(TE(s2, 0, lo), TE2(s0, 2, lo), rk[r][2]) ^ rotl8(TE(s3, 1, lo) ^ TE2(s1, 3, lo));
            const u32 a3 = xor3(TE(s3, 0, lo), TE2(s1, 2, lo), rk[r][3]) ^ rotl8(TE(s0, 1, lo) ^ TE2(s2, 3, lo));
            s0 = a0, s1 = a1, s2 = a2, s3 = a3;
        }
        const u32 st[4] = {s0, s1, s2, s3};
        u32 o[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const u32 x = __builtin_amdgcn_perm(TE(st[(c + 1) & 3], 1, lo), TE2(st[c], 0, lo), 0x0c0c0500u);
            const u32 y = __builtin_amdgcn_perm(TE2(st[(c + 3) & 3], 3, lo), TE(st[(c + 2) & 3], 2, lo), 0x07020c0cu);
            o[c] = __builtin_amdgcn_bitop3_b32(x, y, rk[NR][c], 0x56);
        }
        const u32x4 v = *(const u32x4_u *)(in + 16 * i);
        const u32x4 ks = {o[0], o[1], o[2], o[3]};
        *(u32x4_u *)(out + 16 * i) = v ^ ks;
    }
}

template <int NR>
__global__ __launch_bounds__(256) void ctr_bs(const u32 *__restrict__ kp, const uint8_t *in, uint8_t *out, u64 nblocks,
                                              u32 n0, u32 n1, u32 n2)
{
    const u64 ngroups = nblocks / 8;
    for (u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += (u64)gridDim.x * blockDim.x) {
        u32 w[8][4];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            w[k][0] = n0, w[k][1] = n1, w[k][2] = n2;
            w[k][3] = __builtin_bswap32((u32)(8 * g + k) + 2);
        }
        u32 q[4][8];
        bs::load(q, w);
        bs::encrypt(q, kp, NR);
        bs::store(w, q);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const u64 i = 8 * g + k;
            const u32x4 v = *(const u32x4_u *)(in + 16 * i);
            const u32x4 ks = {w[k][0], w[k][1], w[k][2], w[k][3]};
            *(u32x4_u *)(out + 16 * i) = v ^ ks;
        }
    }
}

// ---- host: key expansion (FIPS-197), key planes, launchers
static uint8_t h_sbox[256];
static void init_sbox()
{
    uint8_t p = 1, q = 1;
    h_sbox[0] = 0x63;
    do {
        p = p ^ (uint8_t)(p << 1) ^ (p & 0x80 ? 0x1b : 0);
        q ^= q << 1, q ^= q << 2, q ^= q << 4;
        if (q & 0x80)
            q ^= 0x09;
        const uint8_t x = q ^ (uint8_t)(q << 1 | q >> 7) ^ (uint8_t)(q << 2 | q >> 6) ^ (uint8_t)(q << 3 | q >> 5) ^
                          (uint8_t)(q << 4 | q >> 4);
        h_sbox[p] = x ^ 0x63;
    } while (p != 1);
}

static int expand(u32 (*rk)[4], const uint8_t *key, int ks)
{
    const int nk = ks / 4, nr = nk + 6;
    u32 w[60];
    for (int j = 0; j < nk; ++j)
        w[j] = key[4 * j] | (u32)key[4 * j + 1] << 8 | (u32)key[4 * j + 2] << 16 | (u32)key[4 * j + 3] << 24;
    u32 rcon = 1;
    auto sub = [](u32 x) {
        return (u32)h_sbox[x & 0xff] | (u32)h_sbox[(x >> 8) & 0xff] << 8 | (u32)h_sbox[(x >> 16) & 0xff] << 16 |
               (u32)h_sbox[x >> 24] << 24;
    };
    for (int j = nk; j < 4 * (nr + 1); ++j) {
        u32 t = w[j - 1];
        if (j % nk == 0) {
            t = sub((t >> 8) | (t << 24)) ^ rcon;
            rcon = ((rcon << 1) ^ (rcon & 0x80 ? 0x1b : 0)) & 0xff;
        } else if (nk > 6 && j % nk == 4) {
            t = sub(t);
        }
        w[j] = w[j - nk] ^ t;
    }
    for (int r = 0; r <= nr; ++r)
        for (int c = 0; c < 4; ++c)
            rk[r][c] = w[4 * r + c];
    return nr;
}

static u32 *d_rk, *d_kp;
static int g_nr;

extern "C" int aesctr_setup(const uint8_t *key, int key_size)
{
    init_sbox();
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_sbox), h_sbox, 256) != hipSuccess)
        return -1;
    u32 rk[15][4], kp[15 * 32];
    g_nr = expand(rk, key, key_size);
    for (int r = 0; r <= g_nr; ++r)
        bs::key_planes(kp + 32 * r, rk[r]);
    hipMalloc(&d_rk, sizeof(rk));
    hipMalloc(&d_kp, sizeof(kp));
    hipMemcpy(d_rk, rk, sizeof(rk), hipMemcpyHostToDevice);
    hipMemcpy(d_kp, kp, sizeof(kp), hipMemcpyHostToDevice);
    hipFuncSetAttribute((const void *)ctr_tt<10>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipFuncSetAttribute((const void *)ctr_tt<14>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    return 0;
}

// which: 0 = T-table, 1 = bitsliced. nblocks must be a multiple of 8.
extern "C" int aesctr_run(int which, const void *in, void *out, u64 nblocks, int grid, void *stream)
{
    const u32 n0 = 0x03020100u, n1 = 0x07060504u, n2 = 0x0b0a0908u;
    hipStream_t s = (hipStream_t)stream;
    if (which == 0) {
        if (g_nr == 10)
            ctr_tt<10><<<grid, 1024, 65536, s>>>(d_rk, (const uint8_t *)in, (uint8_t *)out, nblocks, n0, n1, n2);
        else
            ctr_tt<14><<<grid, 1024, 65536, s>>>(d_rk, (const uint8_t *)in, (uint8_t *)out, nblocks, n0, n1, n2);
    } else {
        if (g_nr == 10)
            ctr_bs<10><<<grid, 256, 0, s>>>(d_kp, (const uint8_t *)in, (uint8_t *)out, nblocks, n0, n1, n2);
        else
            ctr_bs<14><<<grid, 256, 0, s>>>(d_kp, (const uint8_t *)in, (uint8_t *)out, nblocks, n0, n1, n2);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
