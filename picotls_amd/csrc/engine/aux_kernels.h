// picotls_amd/csrc/engine/aux_kernels.h -- Key grouping, AES-ECB, QUIC header protection, QUIC-LB and TLS record checks.
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_AUX_KERNELS_H
#define PTLS_MI355X_ENGINE_AUX_KERNELS_H

// ------------------------------------------------------------------------------------------------ key grouping
// A many-key batch whose records are not grouped by connection would give the chunked kernel one-record key runs, each
// with its own table build and barrier (15 GiB/s on 4M records over 64K keys in random order against 724 grouped).
// Small kernels group it on the device first: the number of key changes between neighbours (regroup when runs would
// average under 8 records, or (round 5) under 32 with at least two runs per key of the keyset: connections in bursts
// of 9-10 records had run in 9-record runs at 510 GiB/s against 785 regrouped; a grouped batch stops here), key
// counts, their exclusive scan, and a scatter of record indices into key order. The chunked kernel then walks the permutation; descriptors, outputs and ok bytes stay
// at each record's own index, so the results are those of the batch order. ctl[0] = key changes, ctl[1] = regroup.
#define KEY_GROUP_MAX_KEYS (1u << 20)

// ctl[0]: key changes between neighbouring records, one atomic per workgroup. (Every wave adding its own sum put 8,192
// device-scope atomics on one word: 112 us per 4M-record batch; 2 workgroups per CU with four loads in flight per lane
// take 34 us, profiles/r5/aux_atomics_ab.txt.)
#define KEY_CHANGES_WG_PER_CU 2
__global__ __launch_bounds__(256) void key_changes_kernel(const ptls_mi355x_record_t *recs, u64 n, u32 *ctl)
{
    __shared__ u32 wsum[4];
    u32 changes = 0;
    const u64 stride = (u64)gridDim.x * blockDim.x;
#pragma unroll 4
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += stride)
        changes += recs[i - 1].key_idx != recs[i].key_idx;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
        changes += (u32)__shfl_xor((int)changes, off, 64);
    if ((threadIdx.x & 63) == 0)
        wsum[threadIdx.x >> 6] = changes;
    __syncthreads();
    if (threadIdx.x == 0) {
        const u32 total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (total != 0)
            atomicAdd(&ctl[0], total);
    }
}

// (the key count bounds the distinct keys of the batch from above: more runs than twice that means keys recur, with
// no per-key pass to find out; a batch over a few keys of a large keyset keeps its runs. The burst rule also wants
// enough runs for the table builds it saves, ~2.4 us a run, to repay the grouping passes: KEY_REGROUP_MIN_RUNS, about
// 32 runs per workgroup on 256 CUs)
#define KEY_REGROUP_MIN_RUNS 8192
__device__ __forceinline__ bool key_regroup(const u32 *ctl, u64 n, u32 nkeys)
{
    const u64 changes = ctl[0];
    return changes * 8 > n || (changes >= 2 * (u64)nkeys && changes * 32 > n && changes >= KEY_REGROUP_MIN_RUNS);
}

// key counts (only when regrouping): each thread counts a contiguous stretch of records and adds one count per key run
__global__ __launch_bounds__(256) void key_hist_kernel(const ptls_mi355x_record_t *recs, u64 n, u32 nkeys, u32 *cnt, const u32 *ctl)
{
    if (!key_regroup(ctl, n, nkeys))
        return;
    const u64 nthr = (u64)gridDim.x * blockDim.x, t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 per = (n + nthr - 1) / nthr, i0 = min(n, t * per), i1 = min(n, i0 + per);
    u32 run_key = 0xffffffffu, run_len = 0;
    for (u64 i = i0; i < i1; ++i) {
        u32 k = recs[i].key_idx;
        k = k < nkeys ? k : nkeys;  // out-of-range keys share the last bucket
        if (k != run_key) {
            if (run_len != 0)
                atomicAdd(&cnt[run_key], run_len);
            run_key = k, run_len = 0;
        }
        ++run_len;
    }
    if (run_len != 0)
        atomicAdd(&cnt[run_key], run_len);
}

// exclusive scan of the counts in place (one workgroup), then ctl[1] = regroup
__global__ __launch_bounds__(1024) void key_scan_kernel(u32 *cnt, u32 nb, u64 n, u32 *ctl)
{
    __shared__ u32 wsum[16];
    const bool regroup = key_regroup(ctl, n, nb - 1);
    if (threadIdx.x == 0)
        ctl[1] = regroup;
    if (!regroup)
        return;
    const u32 t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const u32 per = (nb + blockDim.x - 1) / blockDim.x, b0 = min(nb, t * per), b1 = min(nb, b0 + per);
    u32 sum = 0;
#pragma unroll 8
    for (u32 i = b0; i < b1; ++i)
        sum += cnt[i];
    u32 incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = (u32)__shfl_up((int)incl, off, 64);
        if (lane >= (u32)off)
            incl += y;
    }
    if (lane == 63)
        wsum[wave] = incl;
    __syncthreads();
    u32 run = incl - sum;
    for (u32 w = 0; w < wave; ++w)
        run += wsum[w];
#pragma unroll 8
    for (u32 i = b0; i < b1; ++i) {
        const u32 c = cnt[i];
        cnt[i] = run;
        run += c;
    }
}

__global__ __launch_bounds__(256) void key_scatter_kernel(const ptls_mi355x_record_t *recs, u64 n, u32 nkeys, u32 *cur, u32 *perm,
                                                          ptls_mi355x_record_t *grouped, const u32 *ctl)
{
    if (ctl[1] == 0)
        return;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_record_t r = recs[i];
        const u32 slot = atomicAdd(&cur[r.key_idx < nkeys ? r.key_idx : nkeys], 1u);
        perm[slot] = (u32)i;
        grouped[slot] = r;
    }
}

// ------------------------------------------------------------------------------------------------ byte balance
// A many-key batch of 256 or more records per workgroup is split among the chunked kernel's workgroups by work, not by
// record count: connections differ (a bulk download's 16 KiB records next to a chat's 100-byte ones), and a quarter
// of 64K connections being bulk left the busiest workgroup 26 % above the mean (max-over-workgroups is the launch
// time). Weight of a record = its GHASH stream steps (capped) + 1 for the per-record work; the sums of tiles of
// BALANCE_TILE records, then one workgroup cuts the batch at tile edges into grid ranges of equal weight (a tile is
// < 2 % of a workgroup's share at the sizes this runs at). Both walk the descriptor order the chunked kernel walks.
#define BALANCE_TILE 64

__device__ __forceinline__ u32 balance_weight(const ptls_mi355x_record_t &r, u32 frame)
{
    // (framed batches: flags carries the content type, the AAD is the record header)
    const u32 aad = frame != 0 ? TLS12_AAD_SIZE : (u32)r.aad_len | (u32)r.flags << 16;
    const u32 steps = (u32)(((u64)aad + 15) / 16 + ((u64)r.len + 15) / 16 + 1 + 7) / 8;
    return (steps < 65535u ? steps : 65535u) + 1;
}

// tiles[t] = weight of records [t * 64, t * 64 + 64): one wave per tile
__global__ __launch_bounds__(256) void balance_tiles_kernel(const ptls_mi355x_record_t *recs, const ptls_mi355x_record_t *grouped,
                                                            const u32 *perm_on, u64 n, u32 frame, u32 *tiles)
{
    static_assert(BALANCE_TILE == 64, "one lane per record of a tile");
    const ptls_mi355x_record_t *r = perm_on != nullptr && *perm_on ? grouped : recs;
    const u64 ntiles = (n + BALANCE_TILE - 1) / BALANCE_TILE, lane = threadIdx.x & 63;
    for (u64 t = ((u64)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < ntiles; t += ((u64)gridDim.x * blockDim.x) >> 6) {
        const u64 i = t * BALANCE_TILE + lane;
        u32 w = i < n ? balance_weight(r[i], frame) : 0u;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1)
            w += (u32)__shfl_xor((int)w, off, 64);
        if (lane == 0)
            tiles[t] = w;
    }
}

// bounds[0..grid]: the record ranges of the grid workgroups, cut at tile edges so that each holds about total / grid of
// the weight (one workgroup of 1024 threads: a scan of per-thread tile stretches, then each thread places the cuts that
// fall into its stretch)
__global__ __launch_bounds__(1024) void balance_bounds_kernel(const u32 *tiles, u64 n, u32 grid, u64 *bounds)
{
    __shared__ u64 s_off[1024];
    const u64 ntiles = (n + BALANCE_TILE - 1) / BALANCE_TILE;
    const u32 t = threadIdx.x;
    const u64 per = (ntiles + blockDim.x - 1) / blockDim.x, t0 = min(ntiles, t * per), t1 = min(ntiles, t0 + per);
    u64 sum = 0;
#pragma unroll 16
    for (u64 i = t0; i < t1; ++i)  // (unrolled: 16 loads in flight per lane, not one latency per tile)
        sum += tiles[i];
    s_off[t] = sum;
    __syncthreads();
    // inclusive scan of s_off (Hillis-Steele over 1024 entries; the batch's only serial step, a few microseconds)
    for (u32 off = 1; off < blockDim.x; off <<= 1) {
        const u64 v = t >= off ? s_off[t - off] : 0;
        __syncthreads();
        s_off[t] += v;
        __syncthreads();
    }
    const u64 total = s_off[blockDim.x - 1], lo = s_off[t] - sum, hi = s_off[t];
    if (t == 0) {
        bounds[0] = 0;
        bounds[grid] = n;
    }
    if (total == 0) {  // (no weight: an empty batch) contiguous ranges by count
        for (u32 b = 1 + t; b < grid; b += blockDim.x)
            bounds[b] = n * b / grid;
        return;
    }
    // cuts b (1 <= b < grid) with target total * b / grid in [lo, hi): walk this stretch's tiles to the first tile edge
    // at or past the target
    u64 b = (lo * grid + total - 1) / total;  // least b with total * b / grid >= lo (as exact integers: b * total >= lo * grid)
    b = b < 1 ? 1 : b;
    u64 acc = lo, i = t0;
    for (; b < grid; ++b) {
        const u64 tb = total * b;  // (weights are capped per record: total * grid stays far below 2^64)
        if (tb >= hi * grid)
            break;
        while (i < t1 && (acc + tiles[i]) * grid <= tb)
            acc += tiles[i++];
        bounds[b] = min(n, i * BALANCE_TILE);
    }
}

// AES-ECB of independent blocks (one block per thread, keys from the keyset). Blocks whose key index is out of range
// produce zeros.
template <int NR>
__global__ __launch_bounds__(256) void ecb_kernel(const KeyEntry *keys, u32 nkeys, const u32 *key_idx, const uint8_t *in,
                                                  uint8_t *out, u64 nblocks)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    build_aes_tables(lds);
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nblocks; i += (u64)gridDim.x * blockDim.x) {
        const u32 ki = key_idx != nullptr ? key_idx[i] : 0u;
        u32x4 o = {0, 0, 0, 0};
        if (ki < nkeys) {
            const KeyEntry *k = keys + ki;
            u32 rk[NR + 1][4];
            for (int r = 0; r <= NR; ++r)
                for (int c = 0; c < 4; ++c)
                    rk[r][c] = k->rk[r][c];
            const u32x4 v = *(const u32x4_u *)(in + 16 * i);
            u32 s0 = v[0] ^ rk[0][0], s1 = v[1] ^ rk[0][1], s2 = v[2] ^ rk[0][2], s3 = v[3] ^ rk[0][3];
            aes_encrypt_tt<NR>(lds, laneoff, rk, s0, s1, s2, s3);
            o = u32x4{s0, s1, s2, s3};
        }
        *(u32x4_u *)(out + 16 * i) = o;
    }
}

// QUIC header-protection masks (fusion's supp, lib/fusion.c:425-430,636-651): mask[i] = AES-ECB(hp key, the 16-byte
// sample at base + hp[i].sample_off). Runs after the seal kernel on the same stream, so the sample may cover the tag.
template <int NR>
__global__ __launch_bounds__(256) void hp_kernel(const KeyEntry *keys, u32 nkeys, const ptls_mi355x_hp_t *hp, const uint8_t *base,
                                                 uint8_t *masks, u64 n, u32 *done_flag, u32 done_token)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    build_aes_tables(lds);
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_hp_t h = hp[i];
        u32x4 o = {0, 0, 0, 0};
        if (h.key_idx < nkeys) {
            const KeyEntry *k = keys + h.key_idx;
            u32 rk[NR + 1][4];
            for (int r = 0; r <= NR; ++r)
                for (int c = 0; c < 4; ++c)
                    rk[r][c] = k->rk[r][c];
            const u32x4 v = *(const u32x4_u *)(base + h.sample_off);
            u32 s0 = v[0] ^ rk[0][0], s1 = v[1] ^ rk[0][1], s2 = v[2] ^ rk[0][2], s3 = v[3] ^ rk[0][3];
            aes_encrypt_tt<NR>(lds, laneoff, rk, s0, s1, s2, s3);
            o = u32x4{s0, s1, s2, s3};
        }
        *(u32x4_u *)(masks + 16 * i) = o;
    }
    publish_done(done_flag, done_token);  // (the per-record path: see gcm_chunked_kernel)
}

// QUIC-LB connection-ID cipher (lib/quiclb-impl.h:100-162, behind ptls_fusion_quiclb lib/fusion.c:2186-2233): a 4-round
// Feistel network over the two halves of a 7..19-byte CID, each round X ^ AES-ECB((Y & mask) | len_pass) with
// len_pass = {0 x 14, len, round} (:134-135, :47-70). One thread per CID; blocks are LE words (byte i of the block in
// word i/4). The middle byte of an odd-length CID belongs to both halves, split by nibble masks (:107-125).
template <int NR>
__device__ __forceinline__ u32x4 quiclb_f(const lds_u8 *lds, u32 laneoff, const u32 (*rk)[4], u32x4 y, u32x4 m, u32 len, u32 rnd)
{
    u32 s0 = (y[0] & m[0]) ^ rk[0][0], s1 = (y[1] & m[1]) ^ rk[0][1], s2 = (y[2] & m[2]) ^ rk[0][2];
    u32 s3 = ((y[3] & m[3]) | len << 16 | rnd << 24) ^ rk[0][3];
    aes_encrypt_tt<NR>(lds, laneoff, rk, s0, s1, s2, s3);
    return u32x4{s0, s1, s2, s3};
}

__device__ __forceinline__ void set_byte(u32x4 &v, u32 i, u32 b) { v[i >> 2] |= (b & 0xffu) << (8 * (i & 3)); }
__device__ __forceinline__ u32 get_byte(const u32x4 &v, u32 i) { return (v[i >> 2] >> (8 * (i & 3))) & 0xffu; }

template <int NR>
__global__ __launch_bounds__(256) void quiclb_kernel(const KeyEntry *keys, u32 nkeys, const ptls_mi355x_cid_t *cids,
                                                     const uint8_t *in, uint8_t *out, u64 n)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    build_aes_tables(lds);
    __syncthreads();
    const u32 laneoff = (threadIdx.x & 31) * 4;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_cid_t c = cids[i];
        const u32 L = c.len;
        if (c.key_idx >= nkeys || L < PTLS_MI355X_QUICLB_MIN_LEN || L > PTLS_MI355X_QUICLB_MAX_LEN)
            continue;  // invalid entries are not written
        const KeyEntry *k = keys + c.key_idx;
        u32 rk[NR + 1][4];
        for (int r = 0; r <= NR; ++r)
            for (int w = 0; w < 4; ++w)
                rk[r][w] = k->rk[r][w];
        const u32 half = L / 2, odd = L & 1, hl = half + odd;  // bytes per side: (L + 1) / 2
        // masks (:107-125): left keeps bytes [0, half) and the high nibble of the middle byte; right keeps its low nibble
        // (byte 0) and the bytes after it
        u32x4 ml = {0, 0, 0, 0}, mr = {0, 0, 0, 0};
        for (u32 b = 0; b < half; ++b)
            set_byte(ml, b, 0xff), set_byte(mr, b + odd, 0xff);
        if (odd)
            set_byte(ml, half, 0xf0), set_byte(mr, 0, 0x0f);
        // split (:72-84): l = in[0, hl), r = in[half, half + hl), zero padded
        const uint8_t *src = in + c.in_off;
        u32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
        for (u32 t = 0; t < hl; ++t)
            set_byte(a, t, src[t]), set_byte(b, t, src[half + t]);
        u32x4 l, r;
        if (c.encrypt) {  // (:149-154) l0 = a, r0 = b
            const u32x4 r1 = b ^ quiclb_f<NR>(lds, laneoff, rk, a, ml, L, 1);
            const u32x4 l1 = a ^ quiclb_f<NR>(lds, laneoff, rk, r1, mr, L, 2);
            r = r1 ^ quiclb_f<NR>(lds, laneoff, rk, l1, ml, L, 3);
            l = l1 ^ quiclb_f<NR>(lds, laneoff, rk, r, mr, L, 4);
        } else {  // (:155-161) l2 = a, r2 = b
            const u32x4 l1 = a ^ quiclb_f<NR>(lds, laneoff, rk, b, mr, L, 4);
            const u32x4 r1 = b ^ quiclb_f<NR>(lds, laneoff, rk, l1, ml, L, 3);
            l = l1 ^ quiclb_f<NR>(lds, laneoff, rk, r1, mr, L, 2);
            r = r1 ^ quiclb_f<NR>(lds, laneoff, rk, l, ml, L, 1);
        }
        // merge (:86-100)
        uint8_t *dst = out + c.out_off;
        for (u32 t = 0; t < half; ++t)
            dst[t] = (uint8_t)get_byte(l, t);
        if (odd)
            dst[half] = (uint8_t)((get_byte(l, half) & 0xf0u) | (get_byte(r, 0) & 0x0fu));
        for (u32 t = 0; t < half; ++t)
            dst[half + odd + t] = (uint8_t)get_byte(r, t + odd);
    }
}

// After opening framed TLS records: outer header check, then the receive-side padding strip of lib/picotls.c:5960-5968
// (the inner content type is the last non-zero plaintext byte; an all-zero plaintext, or an empty alert / handshake
// record, is an unexpected message). One thread per record; ok[i] becomes 1 only for status 0.
__global__ __launch_bounds__(256) void tls_unpad_kernel(const ptls_mi355x_record_t *recs, u64 n, const uint8_t *in,
                                                        const uint8_t *out, uint8_t *ok, ptls_mi355x_tls_result_t *res)
{
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_record_t r = recs[i];
        ptls_mi355x_tls_result_t o = {0, 0, 0, 0};
        const uint8_t *h = in + r.in_off;
        if (!ok[i]) {
            o.status = PTLS_MI355X_TLS_BAD_MAC;
        } else if (h[0] != 23 || h[1] != 3 || h[2] != 3 || ((u32)h[3] << 8 | h[4]) != r.len + 16) {
            o.status = PTLS_MI355X_TLS_BAD_HEADER;
        } else {
            const uint8_t *p = out + r.out_off;
            u32 len = r.len;
            while (len != 0 && p[len - 1] == 0)
                --len;
            if (len == 0) {
                o.status = PTLS_MI355X_TLS_UNEXPECTED_MESSAGE;
            } else {
                o.content_type = p[len - 1];
                o.plain_len = len - 1;
                if (o.plain_len == 0 && (o.content_type == 21 || o.content_type == 22))
                    o.status = PTLS_MI355X_TLS_UNEXPECTED_MESSAGE;
            }
        }
        ok[i] = o.status == 0;
        if (res != nullptr)
            res[i] = o;
    }
}

// After opening TLS 1.2 records: the record header must be {type, 3, 3, BE16(8 + len + 16)} (parse_record /
// handle_input_tls12, lib/picotls.c:6019-6045); TLS 1.2 has no inner content type or padding, so the content is the
// whole plaintext and the type is the (authenticated) outer one. ok[i] becomes 1 only for status 0.
__global__ __launch_bounds__(256) void tls12_check_kernel(const ptls_mi355x_record_t *recs, u64 n, const uint8_t *in, uint8_t *ok,
                                                          ptls_mi355x_tls_result_t *res)
{
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const ptls_mi355x_record_t r = recs[i];
        ptls_mi355x_tls_result_t o = {0, 0, 0, 0};
        const uint8_t *h = in + r.in_off;
        if (!ok[i])
            o.status = PTLS_MI355X_TLS_BAD_MAC;
        else if (h[1] != 3 || h[2] != 3 || ((u32)h[3] << 8 | h[4]) != r.len + TLS12_RECORD_IV_SIZE + 16)
            o.status = PTLS_MI355X_TLS_BAD_HEADER;
        o.content_type = h[0];
        o.plain_len = o.status == 0 ? r.len : 0;
        ok[i] = o.status == 0;
        if (res != nullptr)
            res[i] = o;
    }
}

// Measurement (ptls_mi355x_debug_clock_sample): one wave reads the shader-clock counter (s_memtime) and the constant-rate
// real-time counter (s_memrealtime) twice, SPIN_TICKS real-time ticks apart (20 us at 100 MHz), on the same CU, and
// writes both differences and the XCD: the shader clock of that XCD right then (s_memtime counters of different CUs or
// launches are not comparable: round 5 measured nonsense across launches). A bounded spin: at most 2^22 reads.
#define CLOCK_SPIN_TICKS 2000u
__global__ __launch_bounds__(64) void clock_probe_kernel(unsigned long long *out)
{
    if (threadIdx.x != 0)
        return;
    unsigned long long t0, r0, t1, r1;
    u32 xcc;
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_getreg_b32 %2, hwreg(HW_REG_XCC_ID)\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(t0), "=s"(r0), "=s"(xcc)::"memory");
    t1 = t0, r1 = r0;
    for (u32 k = 0; k < (1u << 22) && r1 - r0 < CLOCK_SPIN_TICKS; ++k)
        asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1)::"memory");
    out[0] = t1 - t0;
    out[1] = r1 - r0;
    out[2] = xcc;
}

#endif  // PTLS_MI355X_ENGINE_AUX_KERNELS_H
