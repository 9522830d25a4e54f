// picotls_amd/csrc/engine/gcm_kernels.h -- The batch kernels: lockstep (gcm_batch_kernel) and chunked (gcm_chunked_kernel).
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_GCM_KERNELS_H
#define PTLS_MI355X_ENGINE_GCM_KERNELS_H

// Unit length multiplier of a record of `steps` steps: 1, or for a record that would need more than CHUNK_MAX_UNITS units
// of 2^log2 steps the least factor that fits it in CHUNK_MAX_UNITS (its partials are then combined with the unit power
// applied mul times). Records up to PTLS_MI355X_MAX_RECORD_LEN thus always spread over the workgroup.
__device__ __forceinline__ u32 unit_mul(u32 steps, u32 log2)
{
    const u32 nc = (steps + (1u << log2) - 1) >> log2;
    return nc > CHUNK_MAX_UNITS ? (nc + CHUNK_MAX_UNITS - 1) / CHUNK_MAX_UNITS : 1u;
}

// Descriptors whose len exceeds PTLS_MI355X_MAX_RECORD_LEN or whose key_idx is not below the keyset size are rejected
// as a whole: nothing is written for them and an open reports ok = 0, so a corrupt length cannot make the kernel address
// memory far past the record's offsets. (Multi-key batches also reject invalid keys per key run, before any table build.)
__device__ __forceinline__ bool record_ok(const BatchArgs &args, const ptls_mi355x_record_t &r)
{
    return r.len <= PTLS_MI355X_MAX_RECORD_LEN && r.key_idx < args.nkeys;
}

// Seals / opens one whole record per G-lane group.
template <int NR, bool OPEN, int NB>
__device__ __forceinline__ void process_group(const BatchArgs &args, const lds_u8 *lds, const u32 (&rk)[NR + 1][4], u32 iv0,
                                              u32 iv1, u32 iv2, u64 rec, bool valid, u32 j, u32 laneoff, u32 tsel_horner,
                                              u32 tsel_last)
{
    constexpr int G = ENGINE_G;
    ptls_mi355x_record_t r = {};
    if (valid)
        r = args.recs[rec];
    if (valid && !record_ok(args, r)) {
        if (OPEN && j == 0)
            args.ok[rec] = 0;
        valid = false;
    }
    const u32 K = valid ? gcm_steps<OPEN, 0>(r) : 0;
    u32x4 acc, ek0;
    gcm_segment<NR, OPEN, NB>(args, lds, rk, iv0, iv1, iv2, r, valid, 0, K, j, laneoff, tsel_horner, tsel_last, acc, ek0,
                              true, rec);
}

// Persistent kernel: workgroup w owns the contiguous record range [n*w/grid, n*(w+1)/grid) and walks it in key runs
// (maximal stretches of equal key_idx, at most RUN_SCAN_CAP records); the GHASH tables in LDS are rebuilt only when
// the key changes, so a single-key batch builds them once and a key-sorted many-connection batch once per key.
// ENGINE_WG threads and 128+ KiB of LDS per workgroup: exactly one workgroup (ENGINE_WG/256 waves per SIMD) per CU, so
// the register allocator may use the whole per-wave budget instead of chasing an occupancy the LDS budget rules out.
template <int NR, bool OPEN>
__global__ __launch_bounds__(ENGINE_WG) __attribute__((amdgpu_waves_per_eu(ENGINE_WAVES_PER_SIMD, ENGINE_WAVES_PER_SIMD))) void gcm_batch_kernel(BatchArgs args)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    lds_u32 *s_run = (lds_u32 *)(lds + LDS_BYTES);  // scratch word after the tables
    check_lds_base(smem);
    constexpr int G = ENGINE_G;
    constexpr int RPW = 64 / G;  // records per wave-iteration

    build_aes_tables(lds);

    const u32 lane = threadIdx.x & 63;
    const u32 j = lane % G;
    const u32 slot = lane / G;
    const u32 laneoff = (lane & 31) * 4;
    const u32 wave = threadIdx.x >> 6;
    const u32 waves_per_wg = blockDim.x >> 6;
    const u32 tsel_horner = 0x10000u + (u32)(G - 1) * GHASH_TABLE_BYTES;
    const u32 tsel_last = 0x10000u + (u32)(G - 1 - j) * GHASH_TABLE_BYTES;

    const u64 n = args.nrecs;
    const u64 beg = n * blockIdx.x / gridDim.x, end = n * (blockIdx.x + 1) / gridDim.x;
    u32 loaded_key = 0xffffffffu;

    for (u64 pos = beg; pos < end;) {
        const u32 key_idx = args.multi_key ? args.recs[pos].key_idx : 0u;
        u64 run_end = end;
        if (args.multi_key) {
            const u64 lim = min(end, pos + RUN_SCAN_CAP);
            if (threadIdx.x == 0)
                *s_run = (u32)(lim - pos);
            __syncthreads();
            for (u64 t = pos + threadIdx.x; t < lim; t += blockDim.x)
                if (args.recs[t].key_idx != key_idx)
                    atomicMin((u32 *)s_run, (u32)(t - pos));
            __syncthreads();
            run_end = pos + *s_run;
            __syncthreads();
        }
        if (key_idx >= args.nkeys) {  // invalid key: nothing is written except a failed ok byte
            if (OPEN)
                for (u64 t = pos + threadIdx.x; t < run_end; t += blockDim.x)
                    args.ok[t] = 0;
            pos = run_end;
            continue;
        }
        if (key_idx != loaded_key) {
            __syncthreads();  // no wave still reads the previous key's tables
            build_ghash_tables(lds, args.keys + key_idx);
            __syncthreads();
            loaded_key = key_idx;
        }
        const KeyEntry *key = args.keys + key_idx;
        // round keys and IV are workgroup-uniform: pin them in SGPRs
        u32 rk[NR + 1][4];
#pragma unroll
        for (int r = 0; r <= NR; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                rk[r][c] = __builtin_amdgcn_readfirstlane(key->rk[r][c]);
        const u32 iv0 = __builtin_amdgcn_readfirstlane(key->iv[0]), iv1 = __builtin_amdgcn_readfirstlane(key->iv[1]),
                  iv2 = __builtin_amdgcn_readfirstlane(key->iv[2]);

        const u64 ngroups = (run_end - pos + RPW - 1) / RPW;
        for (u64 grp = wave; grp < ngroups; grp += waves_per_wg) {
            const u64 rec = pos + grp * RPW + slot;
            process_group<NR, OPEN, ENGINE_NB>(args, lds, rk, iv0, iv1, iv2, rec, rec < run_end, j, laneoff, tsel_horner, tsel_last);
        }
        pos = run_end;
    }
}

// Diagnostic build only (-DENGINE_PROFILE=1): s_memtime stamps of the chunked kernel's phases, summed over runs and
// workgroups: [0] run setup, [1] GHASH table build, [2] unit loop, [3] kernel prologue (AES tables), [4] wave idle at the unit-loop barrier,
// [5] units, [6] runs, [7] table builds.
#ifndef ENGINE_PROFILE
#define ENGINE_PROFILE 0
#endif
#if ENGINE_PROFILE
__device__ unsigned long long g_prof[16];
__device__ __forceinline__ unsigned long long stamp()
{
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define PROF_STAMP(v) const unsigned long long v = stamp()
#define PROF_ADD(i, x) atomicAdd(&g_prof[i], (unsigned long long)(x))
#else
#define PROF_STAMP(v)
#define PROF_ADD(i, x)
#endif

// Chunked schedule for many-key / mixed-length batches. The lockstep kernel above gives each G-lane group a whole
// record, so a wave runs as long as its longest record and a key run (~64 records of a connection) as long as its
// longest record too; with U[64 B, 16 KiB] lengths and a workgroup barrier per key that halves throughput twice.
// Here a run's records are cut into units of at most CHUNK_BLOCKS GHASH-stream blocks, counted from the END of the
// stream (so every unit but a record's first is exactly CHUNK_BLOCKS long), and waves pull units from a per-run LDS
// counter. A unit's group computes the partial P_k = sum over its blocks of X_i * H^(end_k - i) (k = units after it);
// GHASH = sum_k P_k * H^(k * CHUNK_BLOCKS). The group that completes a record's last outstanding unit (LDS counter per
// record) evaluates that sum by Horner with the H^CHUNK_BLOCKS table and finishes the tag, inside the unit loop.
// Single-unit records finish inside their unit as in the lockstep kernel.
template <int NR, bool OPEN, int FRAME>
__global__ __launch_bounds__(ENGINE_WG) __attribute__((amdgpu_waves_per_eu(ENGINE_WAVES_PER_SIMD, ENGINE_WAVES_PER_SIMD))) void gcm_chunked_kernel(BatchArgs args)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    PROF_STAMP(tk);
    // s_ctl: [1] next unit, [4..7] per-wave unit totals, [8..11] per-wave key boundary, [12..15] per-wave unit cut,
    // [16..19] / [20..23] per-wave min / max steps, [32 + 16 w + b] per-wave count of front-unit bucket b
    lds_u32 *s_front = (lds_u32 *)(lds + CLDS_FRONT);
    lds_u32 *s_ctl = (lds_u32 *)(lds + CLDS_CTL);
    lds_u32 *s_ubase = (lds_u32 *)(lds + CLDS_UBASE);
    lds_u32 *s_done = (lds_u32 *)(lds + CLDS_DONE);
    lds_u32x4 *s_ek0 = (lds_u32x4 *)(lds + CLDS_EK0);
    lds_u32x4 *s_part = (lds_u32x4 *)(lds + CLDS_PART);
    constexpr int G = ENGINE_G;
    constexpr int RPW = 64 / G;
    constexpr u32 SCAN_WAVES = CRUN_RECS / 64;

    const u32 lane = threadIdx.x & 63;
    const u32 j = lane % G;
    const u32 slot = lane / G;
    const u32 laneoff = (lane & 31) * 4;
    const u32 wave = threadIdx.x >> 6;
    const u32 tsel_horner = 0x10000u + (u32)(G - 1) * GHASH_TABLE_BYTES;
    const u32 tsel_last = 0x10000u + (u32)(G - 1 - j) * GHASH_TABLE_BYTES;
    const u32 tsel_chunk = 0x10000u + 8u * GHASH_TABLE_BYTES;
    // unit length in steps (a power of two <= CHUNK_STEPS) and the key element of its combine power H^(G * ustep)
    const u32 ustep = 1u << args.unit_log2;
    const u32 usrc = ustep == CHUNK_STEPS ? 8u : args.unit_log2 == 0 ? 7u : 8u + args.unit_log2;

    const u64 n = args.nrecs;
    const u64 beg = n * blockIdx.x / gridDim.x, end = n * (blockIdx.x + 1) / gridDim.x;
    u32 loaded_key = 0xffffffffu;
    // the descriptors in batch order, or (an ungrouped many-key batch) the key-grouped copy built on the device; ok
    // bytes go to the record's batch index either way
    const ptls_mi355x_record_t *recs = args.recs;
    const u32 *perm = nullptr;
    if (args.perm_on != nullptr && *args.perm_on)
        recs = args.grouped, perm = args.perm;
    auto ok_at = [&](u64 i) -> u64 { return perm != nullptr ? (u64)perm[i] : i; };

    build_aes_tables(lds);

    for (u64 pos = beg; pos < end;) {
        PROF_STAMP(t0);
        // ---- the run: records [pos, pos + run_n) with one key, at most CRUN_RECS records and CRUN_UNITS units.
        // Threads 0..CRUN_RECS-1 read one descriptor each: the key boundary and the unit counts come from one pass.
        const u32 key_idx = args.multi_key ? recs[pos].key_idx : 0u;
        const u32 lim = (u32)min(end - pos, (u64)CRUN_RECS);
        u32 nc = 0, incl = 0, bkt = 0;
        if (wave < SCAN_WAVES) {
            const u32 t = threadIdx.x;
            bool other_key = false;
            u32 smin = 0xffffffffu, smax = 0;
            if (t < lim) {
                ptls_mi355x_record_t r = recs[pos + t];
                if (!record_ok(args, r))  // rejected: one empty unit (see the unit loop)
                    r.len = 0, r.aad_len = 0;
                const u32 steps = gcm_steps<OPEN, FRAME>(r);
                // front-unit size bucket: 0 = a record too long for CHUNK_MAX_UNITS units (it takes units of a
                // multiple length, unit_mul), else ustep + 1 - size of the record's first unit (1 = a full unit, ustep =
                // one step)
                const u32 mul = unit_mul(steps, args.unit_log2);
                nc = (steps + ustep - 1) >> args.unit_log2;
                if (mul > 1)  // rare: the only division
                    nc = (steps + mul * ustep - 1) / (mul * ustep);
                bkt = mul > 1 ? 0u : ustep + 1 - (steps - (nc - 1) * ustep);
                other_key = args.multi_key && r.key_idx != key_idx;
                if (!other_key)
                    smin = smax = steps;
            }
            smin = wave_min(smin);
            smax = wave_max(smax);
            const u64 kb = __ballot(other_key || t >= lim);
            incl = wave_incl_sum(nc);
            if (lane == 63) {
                s_ctl[4 + wave] = incl;
                s_ctl[8 + wave] = kb ? 64 * wave + (u32)__builtin_ctzll(kb) : 0xffffffffu;
                s_ctl[16 + wave] = smin;
                s_ctl[20 + wave] = smax;
            }
            s_done[t] = 0;
            if (t == 0)
                s_ctl[1] = 0;
        }
        __syncthreads();
        PROF_STAMP(ts1);
        u32 run_n = lim, smin = 0xffffffffu, smax = 0;
#pragma unroll
        for (u32 w = 0; w < SCAN_WAVES; ++w) {
            run_n = min(run_n, s_ctl[8 + w]);
            smin = min(smin, s_ctl[16 + w]);
            smax = max(smax, s_ctl[20 + w]);
        }
        // uniform run: every record is one unit (no partials), and a one-key batch may take a much longer run. A
        // workgroup with fewer records left than it has groups cuts them into units instead, so that a small batch
        // (the per-record picotls path is a batch of one) spreads over the workgroup's waves.
        const bool whole = __builtin_amdgcn_readfirstlane(smax <= smin + UNIFORM_SLACK && end - pos >= WHOLE_MIN_RECS);
        if (whole && !args.multi_key)
            run_n = (u32)min(end - pos, (u64)WHOLE_RUN_RECS);
        if (!whole && wave < SCAN_WAVES) {
            for (u32 w = 0; w < wave; ++w)
                incl += s_ctl[4 + w];
            s_ubase[threadIdx.x + 1] = incl;
            if (threadIdx.x == 0)
                s_ubase[0] = 0;
            // the first record whose units overflow the run's partial slots ends the run (never the first record)
            const u64 cut = __ballot(incl > CRUN_UNITS);
            if (lane == 0)
                s_ctl[12 + wave] = cut ? 64 * wave + (u32)__builtin_ctzll(cut) : 0xffffffffu;
            if (lim == 1 && threadIdx.x == 0) {  // a lone record (a launch of one): its unit order needs no sort
                s_front[0] = 0;
                s_ctl[2] = bkt == 0;
            }
        }
        u32 nhuge = 0;
        PROF_STAMP(ts2);
        if (!whole) {
            __syncthreads();
#pragma unroll
            for (u32 w = 0; w < SCAN_WAVES; ++w)
                run_n = min(run_n, max(s_ctl[12 + w], 1u));
            if (lim == 1)
                nhuge = s_ctl[2];
            // Unit order: [front units of very long records][all full units, record-major][the other front units by
            // size, largest first]. Lockstep waves then draw units of equal or similar length, and the run ends on
            // its shortest units. Counting sort of the front units by bucket: per-wave counts, then positions.
            if (lim != 1) {  // (a lone record's order was set before the barrier above)
                u32 rank = 0;
                if (wave < SCAN_WAVES) {
                    const bool in = threadIdx.x < run_n;
#pragma unroll
                    for (u32 b = 0; b <= CHUNK_STEPS; ++b) {
                        const u64 m = __ballot(in && bkt == b);
                        if (lane == 0)
                            s_ctl[32 + BKT_STRIDE * wave + b] = (u32)__popcll(m);
                        if (in && bkt == b)
                            rank = (u32)__popcll(m & ((1ull << lane) - 1));
                    }
                }
                __syncthreads();
                PROF_STAMP(ts3);
                if (threadIdx.x == 0)
                    PROF_ADD(10, ts3 - ts2);
                if (wave < SCAN_WAVES) {
                    // lane b: first slot of this wave's bucket-b records = all records of earlier buckets (prefix over
                    // lanes) + bucket b of earlier waves; a record then takes lane bkt's value (no serial walk)
                    u32 tot = 0, mine = 0;
#pragma unroll
                    for (u32 w = 0; w < SCAN_WAVES; ++w) {
                        const u32 c = lane < BKT_STRIDE ? s_ctl[32 + BKT_STRIDE * w + lane] : 0u;
                        tot += c;
                        mine += w < wave ? c : 0u;
                    }
                    const u32 before = wave_incl_sum(tot);
                    const u32 first_slot = before - tot + mine;
                    const u32 base = (u32)__shfl((int)first_slot, (int)bkt, 64);
                    if (threadIdx.x < run_n)
                        s_front[base + rank] = threadIdx.x;
                }
#pragma unroll
                for (u32 w = 0; w < SCAN_WAVES; ++w)
                    nhuge += s_ctl[32 + BKT_STRIDE * w];
                __syncthreads();
            }
        }
        // run-level values are workgroup-uniform: keep them in SGPRs (they live across the unit loop, where VGPRs are
        // the scarce resource)
        run_n = __builtin_amdgcn_readfirstlane(run_n);
        nhuge = __builtin_amdgcn_readfirstlane(nhuge);
        const u32 total_units = __builtin_amdgcn_readfirstlane(whole ? run_n : s_ubase[run_n]);
        const u32 nfull = total_units - run_n;
        const u64 run_end = pos + run_n;
        PROF_STAMP(t1);

        if (key_idx >= args.nkeys) {  // invalid key: nothing is written except a failed ok byte
            if (OPEN)
                for (u64 t = pos + threadIdx.x; t < run_end; t += blockDim.x)
                    args.ok[ok_at(t)] = 0;
            __syncthreads();
            pos = run_end;
            continue;
        }
        if (key_idx != loaded_key) {
            build_ghash_tables(lds, args.keys + key_idx, 9, usrc);  // H^1..H^8 and the unit combine power
            __syncthreads();
            loaded_key = key_idx;
            if (threadIdx.x == 0)
                PROF_ADD(7, 1);
        }
        PROF_STAMP(t2);
        const KeyEntry *key = args.keys + key_idx;
        u32 rk[NR + 1][4];
#pragma unroll
        for (int r = 0; r <= NR; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                rk[r][c] = __builtin_amdgcn_readfirstlane(key->rk[r][c]);
        const u32 iv0 = __builtin_amdgcn_readfirstlane(key->iv[0]), iv1 = __builtin_amdgcn_readfirstlane(key->iv[1]),
                  iv2 = __builtin_amdgcn_readfirstlane(key->iv[2]);

        // ---- units: each wave takes RPW consecutive units (one per group) at a time
        for (;;) {
            u32 ub = 0;
            if (lane == 0)
                ub = atomicAdd((u32 *)&s_ctl[1], (u32)RPW);
            ub = __builtin_amdgcn_readfirstlane(ub);
            if (ub >= total_units)
                break;
            const u32 u = ub + slot;
            const bool valid = u < total_units;
            u32 lo = u, first = u, unc = 1, k_back = 0;
            if (!whole && valid) {
                if (u < nhuge || u >= nhuge + nfull) {  // a front unit
                    lo = s_front[u < nhuge ? u : u - nfull];
                    first = s_ubase[lo];
                    unc = s_ubase[lo + 1] - first;
                    k_back = unc - 1;
                } else {  // full unit f: record lo with s_ubase[lo] - lo <= f < s_ubase[lo + 1] - (lo + 1)
                    const u32 f = u - nhuge;
                    u32 hi = run_n;
                    lo = 0;
                    while (hi - lo > 1) {
                        const u32 mid = (lo + hi) >> 1;
                        if (s_ubase[mid] - mid <= f)
                            lo = mid;
                        else
                            hi = mid;
                    }
                    first = s_ubase[lo];
                    unc = s_ubase[lo + 1] - first;
                    k_back = f - (first - lo);
                }
            }
            const u32 ri = lo;
            ptls_mi355x_record_t r = {};
            if (valid)
                r = recs[pos + ri];
            const u64 rid = OPEN && valid ? ok_at(pos + ri) : pos + ri;  // the record's batch index (ok byte)
            const bool live = valid && record_ok(args, r);
            if (valid && !live) {  // rejected descriptor: the scan gave it one unit; nothing is written
                r.len = 0, r.aad_len = 0;
                if (OPEN && j == 0)
                    args.ok[rid] = 0;
            }
            const u32 steps = gcm_steps<OPEN, FRAME>(r);
            // unit [m_lo, m_hi) of the record's steps (whole mode: the record); huge records take longer units
            const u32 mul = whole ? 1u : unit_mul(steps, args.unit_log2);
            u32 m_hi = steps, m_lo = 0;
            if (!whole) {
                const u32 ulen = mul * ustep;
                m_hi = steps - k_back * ulen;
                m_lo = k_back + 1 == unc ? 0u : m_hi - ulen;
            }
            if (!live)
                m_lo = m_hi = 0;
            u32x4 acc, ek0;
            gcm_segment<NR, OPEN, 1, FRAME>(args, lds, rk, iv0, iv1, iv2, r, live, m_lo, m_hi, j, laneoff, tsel_horner,
                                     tsel_last, acc, ek0, unc == 1, rid);
            if (live && unc > 1) {  // uniform over the group
                u32 last = 0;
                if (j == G - 1) {
                    s_part[first + unc - 1 - k_back] = acc;  // stream order: the front unit first
                    if (k_back == 0)
                        s_ek0[ri] = ek0;
                    __threadfence_block();  // partial and E(K, J0) land before the count that publishes them
                    last = atomicAdd((u32 *)&s_done[ri], 1u) == unc - 1;
                }
                last = dpp_bcast7(last, lane);
                if (last) {
                    // last unit of the record: GHASH = Horner over the partials with H^(G * ulen) = (H^(G * ustep))^mul
                    // (whole group)
                    u32x4 g = s_part[first];
                    for (u32 i = 1; i < unc; ++i) {
                        g = gmul_group(lds, g, tsel_chunk, j);
                        for (u32 t = 1; t < mul; ++t)  // huge records only
                            g = gmul_group(lds, g, tsel_chunk, j);
                        g ^= s_part[first + i];
                    }
                    const u32x4 tag = g ^ s_ek0[ri];
                    if (j != G - 1) {
                    } else if (OPEN) {
                        const u32x4 rt = *(const u32x4_u *)(args.in + r.in_off + frame_in_skip<OPEN, FRAME>() +
                                                            gcm_text_len<OPEN, FRAME>(r));
                        const u32x4 d = rt ^ tag;
                        args.ok[rid] = (d[0] | d[1] | d[2] | d[3]) == 0;
                    } else {
                        *(u32x4_u *)(args.out + r.out_off + frame_out_skip<OPEN, FRAME>() + gcm_text_len<OPEN, FRAME>(r)) = tag;
                    }
                }
            }
        }
        PROF_STAMP(tw);
        __syncthreads();  // the run's tables, partials and counters are free again
        PROF_STAMP(t3);
#if ENGINE_PROFILE
        if (lane == 0)
            PROF_ADD(4, t3 - tw);
        if (threadIdx.x == 0) {
            PROF_ADD(0, t1 - t0);
            PROF_ADD(1, t2 - t1);
            PROF_ADD(2, t3 - t2);
            PROF_ADD(5, total_units);
            PROF_ADD(6, 1);
            PROF_ADD(8, ts1 - t0);
            PROF_ADD(9, ts2 - ts1);
            PROF_ADD(11, t1 - ts2);
            if (pos == beg)
                PROF_ADD(3, t0 - tk);
        }
#endif
        pos = run_end;
    }
}

#endif  // PTLS_MI355X_ENGINE_GCM_KERNELS_H
