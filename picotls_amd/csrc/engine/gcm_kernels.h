// picotls_amd/csrc/engine/gcm_kernels.h -- The batch kernels: lockstep (gcm_batch_kernel) and chunked (gcm_chunked_kernel).
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_GCM_KERNELS_H
#define PTLS_MI355X_ENGINE_GCM_KERNELS_H

// Unit length multiplier of a record of `steps` steps: 1, or for a record that would need more than `cap` units (the
// run's unit capacity: CHUNK_MAX_UNITS, or W8_RUN_UNITS in a launch pair) of 2^log2 steps the least factor that fits it
// in `cap` (its partials are then combined with the unit power applied mul times). Records up to
// PTLS_MI355X_MAX_RECORD_LEN thus always spread over the workgroup.
__device__ __forceinline__ u32 unit_mul(u32 steps, u32 log2, u32 cap)
{
    const u32 nc = (steps + (1u << log2) - 1) >> log2;
    return nc > cap ? (nc + cap - 1) / cap : 1u;
}
// the unit capacity of a launch's runs: the W8 kernels cut their runs at W8_RUN_UNITS (their partial region), the two
// of a pair identically, since each skips exactly the other's runs
__device__ __forceinline__ u32 run_unit_cap(const BatchArgs &args)
{
    return W8_HORNER && args.w8_split ? (u32)W8_RUN_UNITS : (u32)CRUN_UNITS;
}

// Descriptors whose len exceeds PTLS_MI355X_MAX_RECORD_LEN, whose AAD exceeds PTLS_MI355X_MAX_AAD_LEN or whose key_idx
// is not below the keyset size are rejected as a whole: nothing is written for them and an open reports ok = 0, so a
// corrupt length cannot make the kernel address memory far past the record's offsets. (Multi-key batches also reject
// invalid keys per key run, before any table build.)
template <int FRAME = 0>
__device__ __forceinline__ bool record_ok(const BatchArgs &args, const ptls_mi355x_record_t &r)
{
    return r.len <= PTLS_MI355X_MAX_RECORD_LEN && gcm_aad_len<false, FRAME>(r) <= PTLS_MI355X_MAX_AAD_LEN &&
           r.key_idx < args.nkeys;
}

// A small one-key batch's long records go to the spare workgroups (spread_pieces): from 512 KiB (a 256 KiB record cut
// into pieces paid more in the pieces' combine than it gained: 40 x 256 KiB 89 -> 124 us)
#ifndef SPREAD_MIN_BYTES
#define SPREAD_MIN_BYTES (512u << 10)
#endif
__device__ __forceinline__ bool spread_long(const BatchArgs &a, const ptls_mi355x_record_t &r)
{
    return r.len >= SPREAD_MIN_BYTES && record_ok<0>(a, r);
}

// Seals / opens one whole record per G-lane group.
template <int NR, bool OPEN, int NB>
__device__ __forceinline__ void process_group(const BatchArgs &args, const lds_u8 *lds, const u32 (&rk)[NR + 1][4], u32 iv0,
                                              u32 iv1, u32 iv2, u64 rec, bool valid, u32 j, u32 laneoff, u32 tsel_horner)
{
    ptls_mi355x_record_t r = {};
    if (valid)
        r = args.recs[rec];
    if (valid && !record_ok(args, r)) {
        if (OPEN && j == 0)
            args.ok[rec] = 0;
        valid = false;
    }
    const u32 K = valid ? gcm_steps<OPEN, 0>(r) : 0;
    u32x4 acc;
    u32 okw;
    gcm_segment<NR, OPEN, NB>(args, lds, rk, iv0, iv1, iv2, r, valid, 0, K, j, laneoff, tsel_horner, acc, true, okw,
                              true, LDS_EKSLOT + 16u * (threadIdx.x / ENGINE_G));
    if (OPEN && okw <= 1)
        args.ok[rec] = (uint8_t)okw;
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
            build_ghash_tables(lds, args.keys + key_idx, ENGINE_G, 8, 0, 0, 0, false, GHASH_WMASK(false));
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
            process_group<NR, OPEN, ENGINE_NB>(args, lds, rk, iv0, iv1, iv2, rec, rec < run_end, j, laneoff, tsel_horner);
        }
        pos = run_end;
    }
}


// Runs processed per chunked instantiation (EXT 0..4), one row per workgroup (blockIdx.x mod EXT_RUN_ROWS), summed on the
// host by ptls_mi355x_debug_counters: the evidence that a batch ran in the kernel a test means to exercise (one
// uncontended atomic per workgroup and launch, at its end). ENGINE_HOOKS=0 compiles these and the kernel clock out (the
// A/B of profiles/r6/hooks_ab.txt); the shipped build keeps them, as the GPU tests read them.
#ifndef ENGINE_HOOKS
#define ENGINE_HOOKS 1
#endif
#ifndef COMBINE_SCATTER
#define COMBINE_SCATTER 1  // round 5: a record's unit combine as a scattered chain of group products (ghash.h)
#endif
#define EXT_RUN_ROWS 256
__device__ unsigned long long g_ext_runs[EXT_RUN_ROWS][8];

#ifndef RUN_FILL_UNITS
#define RUN_FILL_UNITS (ENGINE_WG / ENGINE_G / 2)  // a cut run takes the longest units that still give this many
#endif
#ifndef RUN_MAX_CHAIN
#define RUN_MAX_CHAIN 36  // longest unit-combine chain a cut run's unit length may give a record (run_unit_log2)
#endif
#ifndef EARLY_GHASH
#define EARLY_GHASH 1
#endif
#ifndef MEAS_BUILD_ONCE
#define MEAS_BUILD_ONCE 0
#endif
#define EARLY_GHASH_WAVE 11  // waves 11..15 (320 threads: one per table window of 9 tables) build a one-key launch's tables

// Run-state control words (RUN_CTL_WORDS per buffer)
#define RC_KEY 0     // key index of the run
#define RC_NEXT 1    // next unit to hand out
#define RC_N 2       // records in the run
#define RC_WHOLE 3   // every record is one unit
#define RC_UNITS 4   // units in the run
#define RC_HUGE 5    // records whose front unit goes first (longer than CHUNK_MAX_UNITS units)
#define RC_CLAIM 6   // the first wave to find this run's queue empty scans the next run
#define RC_LOG2 7    // the run's unit length: 2^RC_LOG2 steps (run_unit_log2)
#define RC_HPNEXT 8  // seal_batch_hp: next header-protection mask of the previous run to hand out (hp_masks_pass)
#define RC_MK 9      // (round 6) an MK run's connections (scan_mk), 0 for any other run

// Scans the run that starts at record p into one run-state buffer, with ONE wave and no workgroup barrier, so that it
// runs while the other waves are still busy with the previous run (the end-of-run tail where they would otherwise
// wait). A run is records [p, p + n) with one key: at most CRUN_RECS records and CRUN_UNITS units, or (a uniform run of
// a one-key batch) up to WHOLE_RUN_RECS whole records. Each lane takes records q * 64 + lane, q < CRUN_RECS / 64.
// Outputs: ctl[RC_*], ubase[0..n] (prefix of unit counts), front[] (records ordered [very long][the others by
// front-unit size, largest first]; the kernel numbers units [their front units][all full units][the other front
// units]) and done[0..n) = 0. All lanes of the wave must be active. FIRST (a launch's first run, which the whole
// workgroup waits for: the critical path of a launch of one record) stops the loops at the run's last 64-record block,
// skips the sort for a lone record and ranks a run of at most 64 records directly; the scans in the run tails keep the plain loops, whose registers the unit loop
// shares (the guarded form adds VGPR spills to the open kernel).
// Unit length of a cut run (2^log2 steps, at most 2^cap) when the launch leaves it to the scan (args.unit_log2 ==
// CHUNK_LOG2): the longest that still gives at least 64 units (half the workgroup's 128 groups; shorter units would
// not shorten the run, only add per-unit work), but long enough that a record's unit combine chains at most 36
// partials (a chain is serial, ~0.15 us a link; 36 admits a 16 KiB TLS record, 129 steps, in 4-step units). Big
// batches keep 2 KiB units; a run of a few records -- a small batch -- is cut finer, so its records spread over the
// waves. (A launch of one record passes its own length rule, single() in aesgcm_engine.hip.)
__device__ __forceinline__ u32 run_unit_log2(u32 total_steps, u32 smax, u32 cap)
{
    u32 fill = 0, chain = 0;
    while (fill < cap && (total_steps >> (fill + 1)) >= (u32)RUN_FILL_UNITS)
        ++fill;
    while (chain < cap && ((smax + (1u << chain) - 1) >> chain) > (u32)RUN_MAX_CHAIN)
        ++chain;
    return fill > chain ? fill : chain;
}

// (round 6) an MK run's key entry of table slot `slot` (common.h: slot 0 at RUN_KEY_OFF as in any run, slots 1.. over the
// done / front words, which whole runs do not use)
typedef __attribute__((address_space(3))) const KeyEntry lds_key_ct;
__device__ __forceinline__ lds_key_ct *mk_key(lds_u32 *rs, u32 slot)
{
    return (lds_key_ct *)(slot == 0 ? rs + RUN_KEY_OFF : rs + RUN_DONE_OFF + (slot - 1) * (u32)(sizeof(KeyEntry) / 4));
}
static_assert(RUN_DONE_OFF + (MK_SLOTS - 1) * (int)(sizeof(KeyEntry) / 4) <= RUN_WORDS, "MK key entries in the run state");
static_assert(MK_SLOTS * ((WHOLE_MIN_RECS + 15) / 16) <= CRUN_RECS + 16 && MK_SLOTS * MK_SLOT_BYTES <= 65536,
              "MK claims in the ubase words, slots in [0, 64K)");

// (round 6) scan_mk (EXT 4, many-key batches; called by scan_run once it has found that the run at p is the short
// uniform records of one connection with fewer records than the workgroup has 8-lane groups, which it would otherwise
// cut into units): joins that connection and the next ones into one multi-key whole run (common.h MK_RUNS) while each
// is complete within the scan window (CRUN_RECS records; its last record followed by another key or the range end), has
// fewer than WHOLE_MIN_RECS records, all of them accepted descriptors of a valid key, and all the run's records stay
// within UNIFORM_SLACK steps of each other and under W8_MIN_STEPS steps -- so a W8 pair's EXT 3 kernel, which scans
// without MK runs, takes none of these records and walks past them to the same run boundary. At least two
// connections, else the run stays as scan_run makes it. One wave; writes the run state as scan_run does.
template <bool OPEN, int FRAME>
__device__ __forceinline__ bool scan_mk(const BatchArgs &args, u64 p, u64 end, lds_u32 *rs, const u32 (&kq)[CRUN_RECS / 64],
                                        const u32 (&sq)[CRUN_RECS / 64], u32 key_after)
{
    // (kq, sq: scan_run's descriptors of the window -- each record's key, and its steps if it may join, else ~0 -- so
    // that this adds no memory round trip but the key entries')
    constexpr u32 Q = CRUN_RECS / 64;
    const u32 lane = lane_here();
    const u32 lim = (u32)min(end - p, (u64)CRUN_RECS);
    u64 chg[Q];
#pragma unroll
    for (u32 q = 0; q < Q; ++q) {
        // the previous record's key: lane - 1, or lane 63 of the previous 64
        u32 prev = (u32)__builtin_amdgcn_ds_bpermute((int)((lane - 1) & 63) * 4, (int)kq[q]);
        if (lane == 0)
            prev = q == 0 ? kq[0] : (u32)__builtin_amdgcn_readlane((int)kq[q == 0 ? 0 : q - 1], 63);
        const u32 t = q * 64 + lane;
        chg[q] = __ballot(t < lim && t > 0 && kq[q] != prev);
    }
    u32 b[MK_SLOTS + 1];
    b[0] = 0;
    u32 k = 0, lo = 0xffffffffu, hi = 0;
#pragma unroll  // (b[] in registers: its indices constant)
    for (u32 s = 0; s < MK_SLOTS; ++s) {
        // the next connection's first record after b[s] (lim: none in the window)
        u32 nb = lim;
#pragma unroll
        for (int q = Q - 1; q >= 0; --q) {
            const u32 sh = b[s] + 1 > (u32)q * 64 ? b[s] + 1 - (u32)q * 64 : 0u;
            const u64 m = sh >= 64 ? 0ull : chg[q] & (~0ull << sh);
            if (m != 0)
                nb = (u32)q * 64 + (u32)__builtin_ctzll(m);
        }
        // complete: another key follows within the window, or the range ends there, or (a connection ending exactly at
        // a full window) the record after the window has another key
        const bool complete = nb < lim || p + lim == end ||
                              key_after != (u32)__builtin_amdgcn_readlane((int)kq[Q - 1], 63);
        if (!complete || nb - b[s] >= (u32)WHOLE_MIN_RECS)
            break;
        u32 mn = 0xffffffffu, mx = 0;
#pragma unroll
        for (u32 q = 0; q < Q; ++q) {
            const u32 t = q * 64 + lane;
            if (t >= b[s] && t < nb)
                mn = min(mn, sq[q]), mx = max(mx, sq[q]);
        }
        mn = wave_min(mn), mx = wave_max(mx);
        const u32 nlo = min(lo, mn), nhi = max(hi, mx);
        if (mx >= (u32)W8_MIN_STEPS || nhi > nlo + UNIFORM_SLACK)  // (an ineligible record: mx = ~0)
            break;
        lo = nlo, hi = nhi, b[s + 1] = nb, k = s + 1;
        if (nb >= lim)
            break;
    }
    if (k < 2)
        return false;
    // claims: a connection's records 16 at a time; slot s = the connection's table slot
    u32 nclaims = 0;
#pragma unroll
    for (u32 s = 0; s < MK_SLOTS; ++s) {
        if (s >= k)
            break;
        const u32 cnt = b[s + 1] - b[s], ncl = (cnt + 15) / 16;
        if (lane >= nclaims && lane < nclaims + ncl) {
            const u32 i = lane - nclaims;
            rs[RUN_UBASE_OFF + lane] = (b[s] + 16 * i) | min(16u, cnt - 16 * i) << 8 | s << 16;
        }
        nclaims += ncl;
        if (s > 0) {  // the connection's key entry beside the first connection's (staged by scan_run)
            const u32 qs = b[s] >> 6, kw = qs == 0 ? kq[0] : qs == 1 ? kq[1] : qs == 2 ? kq[2] : kq[3];
            static_assert(Q == 4, "the selects above");
            const u32 key = (u32)__builtin_amdgcn_readlane((int)kw, (int)(b[s] & 63));
            lds_u32 *dst = rs + RUN_DONE_OFF + (s - 1) * (u32)(sizeof(KeyEntry) / 4);
            dst[lane] = ((const u32 *)(args.keys + key))[lane];
            dst[lane + 64] = ((const u32 *)(args.keys + key))[lane + 64];
        }
    }
    if (lane == 0) {
        rs[RC_KEY] = kq[0];
        rs[RC_NEXT] = 0;
        rs[RC_N] = b[k];
        rs[RC_WHOLE] = 1;
        rs[RC_UNITS] = nclaims;
        rs[RC_HUGE] = 0;
        rs[RC_CLAIM] = 0;
        rs[RC_LOG2] = 0;
        rs[RC_HPNEXT] = 0;
        rs[RC_MK] = k;
    }
    return true;
}

// The only way a kernel instantiation (EXT) changes what scan_run returns: the spread kernel (EXT 1) scans its long
// records as empty units. A W8 pair relies on its two kernels scanning identically -- EXT 4 lists (start, chunk end) of
// the runs it leaves, and EXT 3 rebuilds exactly those runs from them -- so an EXT rule added here must keep EXT 3 and 4
// equal (or the list must carry the run's length and EXT 3 check it). (Round 6: EXT 5, the serial kernel of many-key
// batches, also joins connections of short records into MK runs, scan_mk; those hold no record of EXT 3's and end where
// EXT 3's own runs of them end.)
constexpr bool scan_rule_of_ext(int ext) { return ext == 1; }
static_assert(scan_rule_of_ext(3) == scan_rule_of_ext(4) && scan_rule_of_ext(3) == scan_rule_of_ext(5),
              "a W8 pair's kernels must scan runs identically");

template <bool OPEN, int FRAME, bool FIRST = false, int EXT = 0>
__device__ __forceinline__ void scan_run(const BatchArgs &args, const ptls_mi355x_record_t *__restrict__ recs, u64 p, u64 end,
                                      lds_u32 *rs)
{
    constexpr u32 Q = CRUN_RECS / 64;
    lds_u32 *ubase = rs + RUN_UBASE_OFF, *done = rs + RUN_DONE_OFF, *front = rs + RUN_FRONT_OFF;
    const u32 lane = lane_here();
    const u32 lim = (u32)min(end - p, (u64)CRUN_RECS);
    const u32 key = args.multi_key ? recs[p].key_idx : 0u;
    if (key < args.nkeys)  // the key entry (round keys, IV, H powers) moves to LDS now, off the next run's critical path
        ((lds_u32 *)(rs + RUN_KEY_OFF))[lane] = ((const u32 *)(args.keys + key))[lane],
        ((lds_u32 *)(rs + RUN_KEY_OFF))[lane + 64] = ((const u32 *)(args.keys + key))[lane + 64];
    u32 steps[Q], nc[Q], bkt[Q];
    constexpr bool MKS = MK_RUNS && EXT == 5;
    u32 mkk[MKS ? Q : 1], mks[MKS ? Q : 1];  // (MK: each record's key, and its steps if scan_mk may take it, else ~0)
    // (MK: the key of the record after a full window, so that a connection ending exactly there counts as complete)
    const u32 mk_after = MKS && args.multi_key && lim == (u32)CRUN_RECS && p + lim < end ? recs[p + lim].key_idx : 0xffffffffu;
    u32 n = lim;  // ends at the first record of another key
    // (round 6) the fields the scan reads -- len, key_idx, aad_len | flags << 16: 12 bytes at offset 28 -- loaded for all
    // Q record slots before any is used (a lane past the run's end re-reads the run's last record), so the window costs
    // one memory round trip; loaded whole and under the t < lim branch, the compiler issued the slots one trip each
    static_assert(offsetof(ptls_mi355x_record_t, len) == 28 && offsetof(ptls_mi355x_record_t, key_idx) == 32 &&
                      offsetof(ptls_mi355x_record_t, aad_len) == 36 && offsetof(ptls_mi355x_record_t, flags) == 38,
                  "descriptor layout");
    u32 dl[Q], dk[Q], da[Q];
#pragma unroll
    for (u32 q = 0; q < Q; ++q) {
        const u32 t = q * 64 + lane, tt = t < lim ? t : lim - 1;
        const u32 *w = (const u32 *)(recs + p + tt) + 7;
        dl[q] = w[0], dk[q] = w[1], da[q] = w[2];
    }
#pragma unroll
    for (u32 q = 0; q < Q; ++q) {
        const u32 t = q * 64 + lane;
        steps[q] = nc[q] = bkt[q] = 0;
        if constexpr (MKS)
            mkk[q] = mks[q] = 0xffffffffu;
        bool other = false;
        if (t < lim) {
            ptls_mi355x_record_t r = {};
            r.len = dl[q], r.key_idx = dk[q], r.aad_len = (uint16_t)da[q], r.flags = (uint16_t)(da[q] >> 16);
            other = args.multi_key && r.key_idx != key;
            if constexpr (MKS) {
                mkk[q] = r.key_idx;
                if (record_ok<FRAME>(args, r) && r.key_idx < args.nkeys)
                    mks[q] = gcm_steps<OPEN, FRAME>(r);
            }
            if (!record_ok<FRAME>(args, r) || (scan_rule_of_ext(EXT) && spread_long(args, r)))  // rejected or spread: one empty unit
                r.len = 0, r.aad_len = 0, r.flags = 0;
            steps[q] = gcm_steps<OPEN, FRAME>(r);
        }
        const u64 kb = __ballot(other);
        if (kb != 0)
            n = min(n, q * 64 + (u32)__builtin_ctzll(kb));
    }
    n = __builtin_amdgcn_readfirstlane(n);
    u32 smin = 0xffffffffu, smax = 0;
#pragma unroll
    for (u32 q = 0; q < Q; ++q)
        if (q * 64 + lane < n)
            smin = min(smin, steps[q]), smax = max(smax, steps[q]);
    smin = wave_min(smin);
    smax = wave_max(smax);
    if constexpr (MK_RUNS && EXT == 5) {
        // (round 6) a connection of short uniform records, fewer than the workgroup's groups: join the next
        // connections into one multi-key whole run (scan_mk) instead of cutting it into units
        if (args.multi_key && key < args.nkeys && n >= (u32)MK_MIN_FIRST && n < (u32)WHOLE_MIN_RECS && smax < (u32)W8_MIN_STEPS &&
            smax <= smin + UNIFORM_SLACK && scan_mk<OPEN, FRAME>(args, p, end, rs, mkk, mks, mk_after))
            return;
    }
    // uniform run: every record is one unit (no partials), and a one-key batch may take a much longer run. A workgroup
    // with fewer records left than it has groups cuts them into units instead, so that a small batch (the per-record
    // picotls path is a batch of one) spreads over the workgroup's waves; so does a many-key run of fewer records than
    // groups (round 5: the few records of a connection cut off at a workgroup's range edge were whole runs -- a few
    // groups busy, the rest waiting -- and, when long, a W8 pair's EXT 3 run, for which that workgroup's EXT 3 kernel
    // re-scanned all its runs: +2.7 ms per launch on 64K keys with uneven record counts)
    const bool whole = smax <= smin + UNIFORM_SLACK && (args.multi_key ? (u64)n : end - p) >= WHOLE_MIN_RECS;
    if (whole && !args.multi_key)
        n = (u32)min(end - p, (u64)WHOLE_RUN_RECS);
    u32 units = n, nhuge = 0, log2 = args.unit_log2;
    if (!whole) {
        u32 tot = 0;
#pragma unroll
        for (u32 q = 0; q < Q; ++q)
            tot += q * 64 + lane < n ? steps[q] : 0u;
        const u32 tot_incl = wave_incl_sum(tot);
        if (log2 == CHUNK_LOG2)
            log2 = run_unit_log2((u32)__builtin_amdgcn_readlane((int)tot_incl, 63), smax, CHUNK_LOG2);
        const u32 ustep = 1u << log2;
#pragma unroll
        for (u32 q = 0; q < Q; ++q) {
            // front-unit size bucket: 0 = a record too long for CHUNK_MAX_UNITS units (it takes units of a multiple
            // length, unit_mul), else ustep + 1 - size of the record's first unit (1 = a full unit, ustep = one step)
            const u32 mul = unit_mul(steps[q], log2, run_unit_cap(args));
            nc[q] = (steps[q] + ustep - 1) >> log2;
            if (mul > 1)  // rare: the only division
                nc[q] = (steps[q] + mul * ustep - 1) / (mul * ustep);
            bkt[q] = mul > 1 ? 0u : ustep + 1 - (steps[q] - (nc[q] - 1) * ustep);
        }
        // unit prefix in record order; the first record whose units overflow the run's partial slots ends the run
        // (never the first record)
        u32 carry = 0, cut = n;
#pragma unroll
        for (u32 q = 0; q < Q; ++q) {
            if (FIRST && q * 64 >= n)  // uniform: the rest of the lanes hold no record of this run
                break;
            const u32 t = q * 64 + lane;
            const u32 incl = carry + wave_incl_sum(t < n ? nc[q] : 0u);
            if (t < n)
                ubase[t + 1] = incl;
            const u64 c = __ballot(t < n && incl > run_unit_cap(args));
            if (c != 0)
                cut = min(cut, q * 64 + (u32)__builtin_ctzll(c));
            carry = (u32)__builtin_amdgcn_readlane((int)incl, 63);
        }
        if (lane == 0)
            ubase[0] = 0;
        n = __builtin_amdgcn_readfirstlane(min(n, max(cut, 1u)));
        if (FIRST && n == 1) {  // a lone record (the per-record picotls path): no sort
            nhuge = __builtin_amdgcn_readfirstlane(bkt[0]) == 0;
            if (lane == 0)
                front[0] = 0;
        } else if (FIRST && n <= 64) {
            // a small first run (a small batch, one record per lane): each lane ranks its record by (bucket, index)
            // against the others, n readlanes instead of the sort's 2 x (CHUNK_STEPS + 1) ballot passes
            const u32 mine = bkt[0];
            u32 rank = 0, huge = 0;
#pragma unroll 1
            for (u32 i = 0; i < n; ++i) {
                const u32 bi = (u32)__builtin_amdgcn_readlane((int)bkt[0], (int)i);
                rank += bi < mine || (bi == mine && i < lane) ? 1u : 0u;
                huge += bi == 0 ? 1u : 0u;
            }
            nhuge = __builtin_amdgcn_readfirstlane(huge);
            if (lane < n)
                front[rank] = lane;
        } else {
            // counting sort of the records by front-unit bucket: lane b counts bucket b, then an exclusive scan over
            // lanes
            u32 cnt = 0;
#pragma unroll
            for (u32 q = 0; q < Q; ++q) {
                if (FIRST && q * 64 >= n)
                    break;
#pragma unroll 1
                for (u32 b = 0; b <= CHUNK_STEPS; ++b) {
                    const u32 c = (u32)__popcll(__ballot(q * 64 + lane < n && bkt[q] == b));
                    cnt += lane == b ? c : 0u;
                }
            }
            u32 next = wave_incl_sum(cnt) - cnt;  // lane b: next free slot of bucket b
            nhuge = (u32)__builtin_amdgcn_readlane((int)cnt, 0);
#pragma unroll
            for (u32 q = 0; q < Q; ++q) {
                if (FIRST && q * 64 >= n)
                    break;
#pragma unroll 1
                for (u32 b = 0; b <= CHUNK_STEPS; ++b) {
                    const bool in = q * 64 + lane < n && bkt[q] == b;
                    const u64 m = __ballot(in);
                    if (m == 0)
                        continue;
                    if (in)
                        front[(u32)__builtin_amdgcn_readlane((int)next, (int)b) +
                              (u32)__popcll(m & ((1ull << lane) - 1))] = q * 64 + lane;
                    next += lane == b ? (u32)__popcll(m) : 0u;
                }
            }
        }
        units = (u32)__builtin_amdgcn_readfirstlane((int)ubase[n]);
    }
#pragma unroll
    for (u32 q = 0; q < Q; ++q)
        if (q * 64 + lane < n)
            done[q * 64 + lane] = 0;
    if (lane == 0) {
        rs[RC_KEY] = key;
        rs[RC_NEXT] = 0;
        rs[RC_N] = n;
        rs[RC_WHOLE] = whole;
        rs[RC_UNITS] = units;
        rs[RC_HUGE] = nhuge;
        rs[RC_CLAIM] = 0;
        rs[RC_LOG2] = log2;
        rs[RC_HPNEXT] = 0;
        if constexpr (MK_RUNS && EXT == 5)  // (only the MK kernel reads it)
            rs[RC_MK] = 0;
    }
}

// Chunked schedule for many-key / mixed-length batches (and the default for every batch). Workgroup w walks the chunks
// w, w + grid, ... of BatchArgs::chunk records (or one contiguous range), run by run. The lockstep kernel above gives each G-lane group a whole
// record, so a wave runs as long as its longest record and a key run (~64 records of a connection) as long as its
// longest record too; with U[64 B, 16 KiB] lengths and a workgroup barrier per key that halves throughput twice.
// Here a run's records are cut into units of at most CHUNK_BLOCKS GHASH-stream blocks, counted from the END of the
// stream (so every unit but a record's first is exactly CHUNK_BLOCKS long), and waves pull units from a per-run LDS
// counter. A unit's group computes the partial P_k = sum over its blocks of X_i * H^(end_k - i) (k = units after it);
// GHASH = sum_k P_k * H^(k * CHUNK_BLOCKS). The group that completes a record's last outstanding unit (LDS counter per
// record) evaluates that sum by Horner with the H^CHUNK_BLOCKS table and finishes the tag, inside the unit loop.
// Single-unit records finish inside their unit as in the lockstep kernel.
// QUIC header-protection masks (fusion's supp, lib/fusion.c:425-430,636-651) of sealed records [p, e) of a run, the
// thread tid of nthr taking records p + tid, p + tid + nthr, ...: AES-ECB of the 16-byte sample under the record's
// header-protection key, from the LDS T-tables. The records are complete (tags included: the sample may cover the tag),
// so this runs after the run's end-of-run barrier: a run's masks are work items of the NEXT run's unit loop, taken by
// waves whose units are done (they fill the tail where waves wait for the run's last units), and the workgroup's last
// run's masks are computed by all its threads after the last run. This replaces a second launch (hp_kernel), which
// re-read every sample, rebuilt the T-tables and ran after the whole seal. A thread takes up to HP_PASS_W records at
// once so their loads are in flight together; when the wave's records share one key (a batch grouped by connection, or
// one key) the round keys go to SGPRs and the HP_PASS_W AES chains interleave, otherwise each chain runs with its lanes'
// own round keys. Not inlined: inlined, its registers raised the unit loop's pressure (and the register allocator
// crashed on the constant-time kernel).
#define HP_PASS_W 4
#define HP_ITEM (64 * HP_PASS_W)  // records per work item of a wave
template <int HNR>
__device__ __attribute__((noinline)) void hp_masks_pass(const ptls_mi355x_hp_t *hp, const KeyEntry *hp_keys, u32 hp_nkeys,
                                                        const uint8_t *out, uint8_t *masks, u64 p, u64 e, const u32 *perm,
                                                        u32 tid, u32 nthr)
{
    const lds_u8 *lds = nullptr;  // (absolute LDS addressing: the T-tables are at address 0)
    const u32 laneoff = (lane_here() & 31) * 4;
    for (u64 t0 = p + tid; t0 < e; t0 += (u64)HP_PASS_W * nthr) {
        u64 i[HP_PASS_W];
        ptls_mi355x_hp_t h[HP_PASS_W];
        u32x4 v[HP_PASS_W];
#pragma unroll
        for (int k = 0; k < HP_PASS_W; ++k) {
            const u64 t = t0 + (u64)k * nthr;
            i[k] = t < e ? (perm != nullptr ? (u64)perm[t] : t) : ~(u64)0;  // batch index: the hp entry and mask slot
            h[k] = {0, 0xffffffffu, 0};
            if (t < e)
                h[k] = hp[i[k]];
        }
#pragma unroll
        for (int k = 0; k < HP_PASS_W; ++k) {
            v[k] = u32x4{0, 0, 0, 0};
            if (h[k].key_idx < hp_nkeys)  // (a gather from HBM: half of the masks' cost)
                v[k] = *(const u32x4_u *)(out + h[k].sample_off);
        }
        const u32 k0 = __builtin_amdgcn_readfirstlane(h[0].key_idx);
        bool same = true;
#pragma unroll
        for (int k = 0; k < HP_PASS_W; ++k)
            same = same && (i[k] == ~(u64)0 || h[k].key_idx == k0);
        if (k0 < hp_nkeys && __all(same)) {
            // (scalar loads through a constant-address-space pointer: readfirstlane of the loaded words crashed the
            // register allocator)
            typedef __attribute__((address_space(4))) const u32 const_u32;
            const_u32 *key = (const_u32 *)(const void *)(hp_keys + k0);
            u32 rk[HNR + 1][4];
#pragma unroll
            for (int r = 0; r <= HNR; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    rk[r][c] = key[4 * r + c];
            u32 st[HP_PASS_W][4];
#pragma unroll
            for (int k = 0; k < HP_PASS_W; ++k)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    st[k][c] = v[k][c] ^ rk[0][c];
            aes_rounds_n<HNR, 1, HP_PASS_W>(lds, laneoff, rk, st);
#pragma unroll
            for (int k = 0; k < HP_PASS_W; ++k)
                if (i[k] != ~(u64)0)
                    *(u32x4_u *)(masks + 16 * i[k]) = u32x4{st[k][0], st[k][1], st[k][2], st[k][3]};
            continue;
        }
#pragma unroll
        for (int k = 0; k < HP_PASS_W; ++k) {
            if (i[k] == ~(u64)0)
                continue;
            u32x4 o = {0, 0, 0, 0};
            if (h[k].key_idx < hp_nkeys) {  // (an out-of-range key: a zero mask)
                const u32(*rk)[4] = hp_keys[h[k].key_idx].rk;
                u32 s0 = v[k][0] ^ rk[0][0], s1 = v[k][1] ^ rk[0][1], s2 = v[k][2] ^ rk[0][2], s3 = v[k][3] ^ rk[0][3];
                aes_encrypt_tt<HNR>(lds, laneoff, rk, s0, s1, s2, s3);
                o = u32x4{s0, s1, s2, s3};
            }
            *(u32x4_u *)(masks + 16 * i[k]) = o;
        }
    }
}


// ---- small batches with long records (fusion takes records of any length at full speed,
// lib/fusion.c:1018-1041,1141-1145). The chunked kernel gives a record to one workgroup; in a batch of a few records a
// long one then runs on one CU (10 x 1 MiB: 10 CUs, 0.3 ms). For an unframed batch of fewer records than CUs (one key
// or many) the launch takes one workgroup per CU: workgroup w < nrecs seals or opens record w unless it is long (spread_long),
// and the other workgroups share the long records, each record cut into pieces of 2^e units of SPREAD_UNIT_STEPS steps
// counted from the stream's end (as the per-record path's span kernels cut a lone record, span_kernels.h). A workgroup
// seals its piece's units, one per 8-lane group, folds their partials into Q_s = sum_u P_(s 2^e + u) M_u^u (M_u =
// H^(8 SPREAD_UNIT_STEPS)), stores it, and the piece that completes a record evaluates GHASH = sum_s Q_s M^s, M = M_u^(2^e)
// (from the keyset's H^(2^m), squared further beyond H^1024, in a window table it builds), by Horner, and writes the tag
// or the ok byte.
#define SPREAD_PLAN_CTL 512  // plan words: [0, 256) first piece of record t, [256, 512) its e, [512] pieces in total
// The pieces' unit length in steps (a power of two from 2 to CHUNK_STEPS): a small batch leaves most of each CU's groups
// idle, so shorter units put more groups to work on fewer steps each, at more partials per piece (folded by eight
// groups at once, below). 10 x 1 MiB: 16 steps 102 us, 8 steps 93, 4 steps 92, 2 steps 97; 2 x 8 MiB: 141 / 134 / 136 /
// 146 us (profiles/r3_spread_unit_ab.txt)
#ifndef SPREAD_UNIT_STEPS
#define SPREAD_UNIT_STEPS 8
#endif
#define SPREAD_UNIT_LOG2 (__builtin_ctz(SPREAD_UNIT_STEPS))
static_assert(SPREAD_UNIT_STEPS >= 2 && SPREAD_UNIT_STEPS <= CHUNK_STEPS &&
              (SPREAD_UNIT_STEPS & (SPREAD_UNIT_STEPS - 1)) == 0, "spread unit length");
// key element index of H^(2^m), 3 <= m <= 10 (KeyEntry::h: [7] = H^8, [9..15] = H^16 .. H^1024)
__device__ __forceinline__ u32 key_pow2_idx(u32 m) { return m == 3 ? 7u : 5u + m; }

template <int NR, bool OPEN, bool CT>
__device__ __attribute__((noinline)) void spread_pieces(BatchArgs args, u32 w, u32 nspare)
{
    lds_u8 *lds = (lds_u8 *)nullptr;  // absolute LDS addressing (the kernel checked its base)
    lds_u32 *plan = (lds_u32 *)(lds + CLDS_RUN0);
    lds_u32x4 *s_part = (lds_u32x4 *)(lds + CLDS_PART);
    lds_u32 *s_flag = (lds_u32 *)(lds + CLDS_ONE);
    constexpr int G = ENGINE_G;
    const u32 wave = threadIdx.x >> 6;
    const u32 n = (u32)args.nrecs;  // < 256 (the host's condition)
    if (wave == 0) {
        // the plan, the same in every workgroup: the spare workgroups shared among the long records by their units
        const u32 lane = lane_here();
        u32 units[4], tot = 0;
#pragma unroll
        for (u32 q = 0; q < 4; ++q) {
            const u32 t = q * 64 + lane;
            units[q] = 0;
            if (t < n) {
                const ptls_mi355x_record_t r = args.recs[t];
                if (spread_long(args, r))
                    units[q] = (gcm_steps<OPEN, 0>(r) + SPREAD_UNIT_STEPS - 1) / SPREAD_UNIT_STEPS;
            }
            tot += units[q];
        }
        tot = (u32)__builtin_amdgcn_readlane((int)wave_incl_sum(tot), 63);
        u32 carry = 0;
#pragma unroll
        for (u32 q = 0; q < 4; ++q) {
            const u32 t = q * 64 + lane;
            u32 np = 0, e = 0;
            if (units[q] != 0) {
                const u64 share = (u64)nspare * units[q] / (tot != 0 ? tot : 1u);
                const u32 wr = share > 1 ? (u32)share : 1u;
                const u32 us = (units[q] + wr - 1) / wr;
                while ((1u << e) < us && (1u << e) < SPAN_MAX_UNITS)
                    ++e;
                np = (units[q] + (1u << e) - 1) >> e;
            }
            const u32 incl = carry + wave_incl_sum(np);
            if (t < 256) {
                plan[t] = incl - np;
                plan[256 + t] = e;
            }
            carry = (u32)__builtin_amdgcn_readlane((int)incl, 63);
        }
        if (lane == 0)
            plan[SPREAD_PLAN_CTL] = carry;
    }
    __syncthreads();
    const u32 P = __builtin_amdgcn_readfirstlane(plan[SPREAD_PLAN_CTL]);
    if (w >= P)
        return;  // nothing for this workgroup (a batch without long records: every spare one)
    // the piece's record: the last t with plan[t] <= p (records without pieces share the next one's start)
    auto piece_record = [&](u32 p) -> u32 {
        u32 lo = 0, hi = n;
        while (hi - lo > 1) {
            const u32 mid = (lo + hi) >> 1;
            if (plan[mid] <= p)
                lo = mid;
            else
                hi = mid;
        }
        return __builtin_amdgcn_readfirstlane(lo);
    };
    // H^1..H^8 and the unit power H^(8 SPREAD_UNIT_STEPS) of the first piece's key on waves EARLY_GHASH_WAVE.., the AES
    // tables on the other waves; a many-key batch rebuilds the GHASH tables when a later piece's key differs
    const u32 src8 = SPREAD_UNIT_STEPS == CHUNK_STEPS ? 8u : key_pow2_idx(3 + SPREAD_UNIT_LOG2);
    u32 loaded_key = args.multi_key ? args.recs[piece_record(w)].key_idx : 0u;
    if (wave >= EARLY_GHASH_WAVE)
        build_ghash_tables(lds, args.keys + loaded_key, 9, src8, 0, EARLY_GHASH_WAVE * 64, ENGINE_WG - EARLY_GHASH_WAVE * 64,
                           false, GHASH_WMASK(CT));
    else
        build_aes_tables(lds, 0, EARLY_GHASH_WAVE * 64);
    __syncthreads();
    const u32 tsel_horner = 0x10000u + (u32)(G - 1) * GHASH_TABLE_BYTES, tsel_chunk = 0x10000u + 8u * GHASH_TABLE_BYTES;
    for (u32 p = w; p < P; p += nspare) {
        const u32 t = piece_record(p), s = p - plan[t], e = plan[256 + t], pbase = plan[t];
        const u32 np_t = (t + 1 < n ? plan[t + 1] : P) - pbase;
        const ptls_mi355x_record_t r = args.recs[t];
        const u32 kidx = args.multi_key ? __builtin_amdgcn_readfirstlane(r.key_idx) : 0u;  // (< nkeys: spread_long)
        if (kidx != loaded_key) {
            build_ghash_tables(lds, args.keys + kidx, 9, src8, 0, 0, 0, false, GHASH_WMASK(CT));  // (freed by the last barrier)
            __syncthreads();
            loaded_key = kidx;
        }
        const KeyEntry *key = args.keys + kidx;
        u32 rk[NR + 1][4];
#pragma unroll
        for (int rr = 0; rr <= NR; ++rr)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                rk[rr][c] = __builtin_amdgcn_readfirstlane(key->rk[rr][c]);
        const u32 iv0 = __builtin_amdgcn_readfirstlane(key->iv[0]), iv1 = __builtin_amdgcn_readfirstlane(key->iv[1]),
                  iv2 = __builtin_amdgcn_readfirstlane(key->iv[2]);
        const u32 steps = gcm_steps<OPEN, 0>(r), U = (steps + SPREAD_UNIT_STEPS - 1) / SPREAD_UNIT_STEPS;
        const u32 k0 = s << e, nu = min(U - k0, 1u << e);
        for (u32 uu0 = wave * 8; uu0 < nu; uu0 += ENGINE_WG / G) {
            const u32 lane = lane_here(), j = lane % G, uu = uu0 + lane / G, laneoff = (lane & 31) * 4;
            const bool valid = uu < nu;
            const u32 k = k0 + uu;
            u32 m_hi = 0, m_lo = 0;
            if (valid) {
                m_hi = steps - k * SPREAD_UNIT_STEPS;
                m_lo = k + 1 == U ? 0u : m_hi - SPREAD_UNIT_STEPS;
            }
            u32x4 acc;
            u32 okw;
            gcm_segment<NR, OPEN, 1, 0, CT>(args, lds, rk, iv0, iv1, iv2, r, valid, m_lo, m_hi, j, laneoff, tsel_horner, acc,
                                            false, okw, false, CLDS_PART + 16u * uu);
            if (valid && j == G - 1)  // (the record's last unit includes E(K, J0), gcm_segment)
                s_part[uu] = acc;
        }
        __syncthreads();
        // Q_s = sum_u P_u M_u^u (M_u = H^(8 SPREAD_UNIT_STEPS), the table in slot 8). From 16 units, the eight groups of
        // wave 0 fold L = 2^(e-3) units each (Horner with M_u) while wave 1 builds the table of M_u^L (from the keyset)
        // after the partials, and the eight sums are then folded with it: L + 7 links instead of nu - 1.
        const u32 mL = SPREAD_UNIT_LOG2 + e;  // M_u^L = H^(2^mL)
        const bool split = e >= 4 && mL <= 10 && (16u << e) <= GHASH_TABLE_BYTES;
        lds_u32x4 *s_sum = (lds_u32x4 *)(lds + CLDS_RUN1);  // the eight groups' sums
        const u32 tsel_ml = CLDS_PART + GHASH_TABLE_BYTES;
        if (split) {
            if (wave == 1)
                build_elem_table(lds, tsel_ml, u32x4{key->h[key_pow2_idx(mL)][0], key->h[key_pow2_idx(mL)][1],
                                                     key->h[key_pow2_idx(mL)][2], key->h[key_pow2_idx(mL)][3]}, 64, SEG_COOP);
            if (wave == 0) {
                const u32 lane = lane_here(), c = lane / G, L = 1u << (e - 3), ulo = c * L, uhi = min(ulo + L, nu);
                u32x4 g = {0, 0, 0, 0};
                if (ulo < uhi) {
                    g = s_part[uhi - 1];
                    for (u32 i = uhi - 1; i-- > ulo;)
                        g = gmul_combine<CT>(lds, g, tsel_chunk, lane) ^ s_part[i];
                }
                if (lane % G == 0)
                    s_sum[c] = g;
            }
            __syncthreads();
        }
        if (wave == 0) {  // Q_s by Horner from the highest unit (or group sum) down (every lane of wave 0 holds it)
            const u32 lane = lane_here();
            u32x4 g;
            if (split) {
                g = s_sum[7];
                for (u32 c = 7; c-- > 0;)
                    g = gmul_combine<CT>(lds, g, tsel_ml, lane) ^ s_sum[c];
            } else {
                g = s_part[nu - 1];
                for (u32 i = nu - 1; i-- > 0;)
                    g = gmul_combine<CT>(lds, g, tsel_chunk, lane) ^ s_part[i];
            }
            if (lane == 0) {
                args.spread_part[pbase + s] = g;
                __threadfence();  // the partial is visible device-wide before the count that publishes it
                *s_flag = atomicAdd(args.spread_cnt + t, 1u) == np_t - 1;
            }
        }
        __syncthreads();
        if (*s_flag) {  // this piece completed the record: GHASH = sum_s Q_s M^s, M = H^(8 SPREAD_UNIT_STEPS 2^e)
            __threadfence();
            lds_u32x4 *s_m = (lds_u32x4 *)(lds + CLDS_PART + GHASH_TABLE_BYTES);  // M (after the element table)
            // M = H^(8 SPREAD_UNIT_STEPS 2^e) = H^(2^m) from the keyset for m <= 10, else by squaring H^1024
            const u32 m = 3 + SPREAD_UNIT_LOG2 + e, hi = m <= 10 ? key_pow2_idx(m) : 15u;
            if (threadIdx.x == 0)
                *s_m = u32x4{key->h[hi][0], key->h[hi][1], key->h[hi][2], key->h[hi][3]};
            __syncthreads();
            for (u32 i = 10; i < m; ++i) {
                build_elem_table(lds, CLDS_PART, *s_m);
                __syncthreads();
                const u32x4 sq = gmul_tab(lds, *s_m, CLDS_PART);
                __syncthreads();
                if (threadIdx.x == 0)
                    *s_m = sq;
                __syncthreads();
            }
            build_elem_table(lds, CLDS_PART, *s_m);
            __syncthreads();
            if (wave == 0) {
                const u32 lane = lane_here();
                const volatile u32x4 *vp = args.spread_part + pbase;  // (written by other workgroups: not cached reads)
                u32x4 g = vp[np_t - 1];
                for (u32 i = np_t - 1; i-- > 0;)
                    g = gmul_tab(lds, g, CLDS_PART) ^ u32x4(vp[i]);
                if (lane == 0) {
                    if (OPEN) {
                        const u32x4 rt = *(const u32x4_u *)(args.in + r.in_off + r.len);
                        const u32x4 d = rt ^ g;
                        args.ok[t] = (d[0] | d[1] | d[2] | d[3]) == 0;
                    } else {
                        *(u32x4_u *)(args.out + r.out_off + r.len) = g;
                    }
                    args.spread_cnt[t] = 0;  // zero for the next launch
                }
            }
        }
        __syncthreads();  // s_part, s_flag and the element table are free again
    }
}

// EXT (FRAME 0 only): 0 = plain; 1 = a spread launch (a small one-key batch, spread_pieces); 2 = seal with
// header-protection masks (seal_batch_hp). Separate instantiations: the calls these add (spread_pieces, hp_masks_pass)
// cost the plain kernels' loops registers (16 KiB seal -1.2 % with both compiled into one kernel).
// Constant-time combine of a record's unc unit partials p[0..unc) (GHASH = sum_i p_i M^(unc-1-i), M the unit power in
// table 8) by the G lanes of one group: blocks of 8 partials from the front (the first one short, right-aligned on the
// lanes), each summed by a butterfly in which level k pairs lane l (bit k clear) with lane l + k as v_l M^k + v_(l+k)
// (tables 8, 4, 5: M, M^2, M^4; every lane the same table), the blocks joined by Horner with M^8 (table 6). ceil(log2
// unc) products instead of unc - 1 chained ones for unc <= 8. Lane G - 1 holds the result.
__device__ __noinline__ u32x4 ct_combine_tree(const lds_u8 *lds, const lds_u32x4 *p, u32 unc, u32 j)
{
    const u32 nblk = (unc + 7) >> 3, c0 = unc - 8 * (nblk - 1);
    u32x4 g = {0, 0, 0, 0};
    for (u32 b = 0; b < nblk; ++b) {
        const int i = (int)j - 8 + (int)c0 + 8 * (int)b;
        u32x4 v = i >= 0 ? u32x4(p[i]) : u32x4{0, 0, 0, 0};
        const u32 lv = b != 0 || c0 > 4 ? 3u : c0 > 2 ? 2u : c0 > 1 ? 1u : 0u;
        for (u32 l = 0; l < lv; ++l) {
            const u32 k = 1u << l;
            const u32x4 y = gmul_tab(lds, v, 0x10000u + (l == 0 ? 8u : 3u + l) * GHASH_TABLE_BYTES);
            const bool hi = (j & k) != 0;
            const u32x4 send = hi ? v : y;
            u32x4 recv;
            // partner lane l ^ k: quad_perm [1,0,3,2], [2,3,0,1]; for k = 4 row_half_mirror (lane 7 - l), which holds
            // the same value as lane l ^ 4 once levels 1 and 2 made each quad uniform
#pragma unroll
            for (int c = 0; c < 4; ++c)
                recv[c] = k == 1   ? (u32)__builtin_amdgcn_update_dpp(0, (int)send[c], 0xB1, 0xF, 0xF, false)
                          : k == 2 ? (u32)__builtin_amdgcn_update_dpp(0, (int)send[c], 0x4E, 0xF, 0xF, false)
                                   : (u32)__builtin_amdgcn_update_dpp(0, (int)send[c], 0x141, 0xF, 0xF, false);
            v = hi ? (recv ^ v) : (y ^ recv);
        }
        g = b == 0 ? v : (gmul_tab(lds, g, 0x10000u + 6u * GHASH_TABLE_BYTES) ^ v);
    }
    return g;
}

// The W8 tables of the run's key (staged in LDS), by three waves at once: H^8's 4-bit nibble-major table into the
// partial region (free between runs) as the source of its 8-bit table over slots 0..7, H window-major into slot 8, and
// (a cut run: usrc = the key element of its unit combine power) that power window-major at W8_TAB_COMB; then the 8-bit
// table. Out of line: inlined into the run loop it cost the kernel's other runs registers (-4 % on 1200-byte records).
// tree (the EXT 3 kernel: long whole records): H and H^2 nibble-major at W8_TAB_H and W8_TAB_COMB instead (w8_tree_end).
__device__ __noinline__ void w8_build_tables(lds_u8 *lds, const lds_u8 *keyp, u32 usrc, bool tree, u32 hpow)
{
    typedef __attribute__((address_space(3))) const KeyEntry lds_key_t;
    lds_key_t *key = (lds_key_t *)keyp;
    auto el = [&](u32 i) { return u32x4{key->h[i][0], key->h[i][1], key->h[i][2], key->h[i][3]}; };
    build_elem_table(lds, CLDS_PART, el(hpow), 0, false);  // (the Horner power: H^8, or H^4 for 4-lane groups)
    build_elem_table(lds, W8_TAB_H, el(0), 64, !tree);
    if (tree)
        build_elem_table(lds, W8_TAB_COMB, el(1), 128, false);
    else if (usrc != 0xffffffffu)
        build_elem_table(lds, W8_TAB_COMB, el(usrc), 128, true);
    __syncthreads();
    build_h8_byte_table(lds, CLDS_PART);
    __syncthreads();
}

// (test and measurement hook, include/picotls/mi355x_debug.h: ptls_mi355x_debug_kernel_clock) when g_kclock_buf is set,
// workgroup 0 of every chunked launch that has work appends {s_memtime, s_memrealtime} at its start and at its end: the
// shader clock the chip holds over the launch itself, which a probe after the launch cannot see
__device__ unsigned long long *g_kclock_buf;
__device__ unsigned int g_kclock_cap;
__device__ unsigned int g_kclock_n;

template <int NR, bool OPEN, int FRAME, bool CT = false, int EXT = 0>
__global__ __launch_bounds__(ENGINE_WG) __attribute__((amdgpu_waves_per_eu(ENGINE_WAVES_PER_SIMD, ENGINE_WAVES_PER_SIMD))) void gcm_chunked_kernel(BatchArgs args)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *lds = (lds_u8 *)smem;
    check_lds_base(smem);
    PROF_STAMP(tk);
    lds_u32x4 *s_part = (lds_u32x4 *)(lds + CLDS_PART);
    constexpr int G = ENGINE_G;
    constexpr int RPW = 64 / G;

    // (the lane index and what derives from it are computed in the unit loop, lane_here())
    const u32 wave = threadIdx.x >> 6;
    const u32 tsel_horner = 0x10000u + (u32)(G - 1) * GHASH_TABLE_BYTES;
    constexpr bool W8K = W8_HORNER && (EXT == 3 || EXT == 4 || EXT == 5);  // a W8 kernel (launch_chunked)
    constexpr bool W8TREE = W8_HORNER && EXT == 3;                  // ... with the butterfly segment end
    // the unit combine table: slot 8, or in the W8 kernel's map W8_TAB_COMB
    const u32 tsel_chunk = W8K ? (u32)W8_TAB_COMB : 0x10000u + 8u * GHASH_TABLE_BYTES;

    const u64 n = args.nrecs, C = args.bounds != nullptr ? 0 : args.chunk;
    // the pair's second kernel (EXT 3): none of this workgroup's runs is its kind (the first kernel saw them all), or
    // (round 5) the runs it left are listed, and this kernel visits just those (`slist`, `scnt`)
    const u32 *slist = nullptr;
    u32 scnt = 0;
    if constexpr (W8TREE) {
        if (args.w8_split == 2 && args.w8_flags != nullptr) {
            scnt = args.w8_flags[(u64)blockIdx.x * W8_FLAG_WORDS];
            if (scnt == 0)
                return;
            if (scnt <= W8_SKIP_LIST)
                slist = args.w8_flags + (u64)blockIdx.x * W8_FLAG_WORDS + 1;
        }
    }
    unsigned long long *const kclock = ENGINE_HOOKS && blockIdx.x == 0 ? g_kclock_buf : nullptr;
    const u64 kc_t0 = kclock != nullptr ? __builtin_amdgcn_s_memtime() : 0ull;
    const u64 kc_r0 = kclock != nullptr ? __builtin_amdgcn_s_memrealtime() : 0ull;
    u32 skipped_w8 = 0;  // (the pair's first kernel: the runs this workgroup left to the second one)
    // (test hook, ptls_mi355x_debug_counters) the runs this workgroup processed, and those in 4-lane groups: counted in
    // SGPRs, added to g_ext_runs once at the end (round 6: was one device-scope atomic per run)
    u32 runs_here = 0, g4_here = 0, mk_here = 0;
    constexpr bool SPREAD = FRAME == 0 && EXT == 1;
    if constexpr (SPREAD) {  // a small one-key batch (spread_pieces): workgroup w < n takes record w unless it is long
        if (blockIdx.x >= n) {
            spread_pieces<NR, OPEN, CT>(args, blockIdx.x - (u32)n, gridDim.x - (u32)n);
            return;
        }
    }
    // this workgroup's records: the chunk [beg, end) (cstart: its first record), then the chunk grid * C further on
    // (C != 0), or one contiguous range (C == 0): balanced by weight (args.bounds) or by count (spread: record w)
    u64 beg = SPREAD ? (u64)blockIdx.x : args.bounds != nullptr ? args.bounds[blockIdx.x] : C != 0 ? min(n, (u64)blockIdx.x * C) : n * blockIdx.x / gridDim.x;
    u64 end = SPREAD ? (u64)blockIdx.x + 1 : args.bounds != nullptr ? args.bounds[blockIdx.x + 1] : C != 0 ? min(n, beg + C) : n * (blockIdx.x + 1) / gridDim.x;
    u64 cstart = beg;
    u32 sidx = 0;  // (EXT 3 with a run list) the listed run being processed
    if constexpr (W8TREE) {
        if (slist != nullptr)
            beg = slist[0], end = slist[1];
    }
    u32 loaded_key = 0xffffffffu, loaded_usrc = 0xffffffffu;
    u32 loaded_w8 = 0;  // the LDS holds the nine 4-bit tables (0) or the W8 map: serial segment ends (1), the tree (2)
    // the descriptors in batch order, or (an ungrouped many-key batch) the key-grouped copy built on the device; ok
    // bytes go to the record's batch index either way
    const ptls_mi355x_record_t *recs = args.recs;
    const u32 *perm = nullptr;
    if (args.perm_on != nullptr && *args.perm_on)
        recs = args.grouped, perm = args.perm;
    if (args.one_inline) {
        // a lone record's descriptor from the kernel arguments into LDS: the per-record path stages its inputs in
        // mapped host memory, where reading the descriptor would put a PCIe round trip ahead of everything else
        recs = (const ptls_mi355x_record_t *)(smem + CLDS_ONE);
        if (threadIdx.x < sizeof(ptls_mi355x_record_t) / 4)
            ((lds_u32 *)(lds + CLDS_ONE))[threadIdx.x] = ((const u32 *)&args.one)[threadIdx.x];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // wave 0 writes it and scans it; the other waves read it
        __builtin_amdgcn_wave_barrier();                          // after the prologue barrier
    }
    auto ok_at = [&](u64 i) -> u64 { return perm != nullptr ? (u64)perm[i] : i; };
    // seal_batch_hp: the header-protection masks of each run's records once the run is sealed (hp_masks_pass; a macro,
    // as a lambda called twice was outlined into a call, which put the kernel arguments on the stack). hp_pos / hp_n:
    // the previous run's records, whose masks the current run's waves take as work items (RC_HPNEXT)
    constexpr bool HPK = !OPEN && FRAME == 0 && EXT == 2;
    const bool with_hp = HPK && args.hp != nullptr;
    u64 hp_pos = 0;
    u32 hp_n = 0;
#define HP_PASS(p_, e_, tid_, nthr_)                                                                                    \
    do {                                                                                                                \
        if constexpr (HPK) {                                                                                            \
            if (args.hp_nr == 10)                                                                                       \
                hp_masks_pass<10>(args.hp, args.hp_keys, args.hp_nkeys, args.out, args.masks, (p_), (e_), perm, (tid_),  \
                                  (nthr_));                                                                             \
            else                                                                                                        \
                hp_masks_pass<14>(args.hp, args.hp_keys, args.hp_nkeys, args.out, args.masks, (p_), (e_), perm, (tid_),  \
                                  (nthr_));                                                                             \
        }                                                                                                               \
    } while (0)

    // the first run's state on wave 0 (later runs are scanned during the previous run's tail) while waves 1.. copy
    // the AES tables. A one-key launch knows its key before the scan: waves EARLY_GHASH_WAVE.. build its GHASH tables
    // H^1..H^8 meanwhile (and the unit combine table when the launch fixes the unit length: the per-record path),
    // instead of after the prologue barrier; the AES copy keeps the waves in between.
    const bool early = EARLY_GHASH && !args.multi_key && !W8K;
    const u32 fixed_usrc = args.unit_log2 == CHUNK_LOG2 ? 8u : args.unit_log2 == 0 ? 7u : 8u + args.unit_log2;
    const bool early_combine = early && args.unit_log2 < CHUNK_LOG2;
    if (early && wave >= EARLY_GHASH_WAVE) {
        build_ghash_tables(lds, args.keys, early_combine ? 9u : 8u, fixed_usrc, 0, EARLY_GHASH_WAVE * 64,
                           ENGINE_WG - EARLY_GHASH_WAVE * 64, CT && CT_COMB_TREE_ON, GHASH_WMASK(CT));
    } else if (wave == 0) {
        if (beg < end)
            scan_run<OPEN, FRAME, true, EXT>(args, recs, beg, end, (lds_u32 *)(lds + CLDS_RUN0));
#if ENGINE_PROFILE
        if (threadIdx.x == 0)
            PROF_ADD(9, stamp() - tk), PROF_ADD(10, 1);
#endif
    } else {
        build_aes_tables(lds, 64, early ? EARLY_GHASH_WAVE * 64 : 0, W8K ? W8_AES_BASE : 0u);
#if ENGINE_PROFILE
        if (threadIdx.x == 64)
            PROF_ADD(8, stamp() - tk);
#endif
    }
    __syncthreads();

    if (early)  // key 0's tables are in place (and the combine table of the fixed unit length)
        loaded_key = 0, loaded_usrc = early_combine ? fixed_usrc : 0xffffffffu;

    u32 rb = 0;  // run-state buffer of the current run
    for (u64 pos = beg; pos < end;) {
        PROF_STAMP(t0);
        lds_u32 *rs = (lds_u32 *)(lds + (rb ? CLDS_RUN1 : CLDS_RUN0));
        lds_u32 *rs_next = (lds_u32 *)(lds + (rb ? CLDS_RUN0 : CLDS_RUN1));
        lds_u32 *s_ubase = rs + RUN_UBASE_OFF, *s_done = rs + RUN_DONE_OFF, *s_front = rs + RUN_FRONT_OFF;
        // run-level values are workgroup-uniform: keep them in SGPRs (they live across the unit loop, where VGPRs are
        // the scarce resource)
        const u32 key_idx = __builtin_amdgcn_readfirstlane(rs[RC_KEY]);
        const u32 run_n = __builtin_amdgcn_readfirstlane(rs[RC_N]);
        const bool whole_run = __builtin_amdgcn_readfirstlane(rs[RC_WHOLE]);
        const u32 total_units = __builtin_amdgcn_readfirstlane(rs[RC_UNITS]);
        const u32 nhuge = __builtin_amdgcn_readfirstlane(rs[RC_HUGE]);
        // (round 6) a multi-key run (EXT 4, scan_mk): its connections, 0 for any other run
        const u32 mk_n = MK_RUNS && EXT == 5 ? __builtin_amdgcn_readfirstlane(rs[RC_MK]) : 0u;
        // the run's unit length in steps (a power of two <= CHUNK_STEPS) and the key element of its combine power
        // H^(G * ustep): [7] = H^8, [9..12] = H^16..H^128, [8] = H^CHUNK_BLOCKS
        const u32 ulog2 = __builtin_amdgcn_readfirstlane(rs[RC_LOG2]), ustep = 1u << ulog2;
        const u32 usrc = ustep == CHUNK_STEPS ? 8u : ulog2 == 0 ? 7u : 8u + ulog2;
        const u32 nfull = total_units - run_n;
        const u64 run_end = pos + run_n;
        // the next run: the rest of this chunk, or the workgroup's next chunk
        u64 nxt = run_end, nxt_end = end, nxt_cstart = cstart;
        if (C != 0 && run_end >= end) {
            nxt_cstart = cstart + (u64)gridDim.x * C;
            nxt = min(n, nxt_cstart);
            nxt_end = min(n, nxt_cstart + C);
        }
        if constexpr (W8TREE) {
            if (slist != nullptr) {  // the next listed run (none: the loop ends)
                if (sidx + 1 < scnt) {
                    nxt = slist[2 * sidx + 2];
                    nxt_end = slist[2 * sidx + 3];
                } else {
                    nxt = nxt_end = 0;
                }
                ++sidx;
            }
        }
        PROF_STAMP(t1);

        // a W8 pair (w8_split 2): runs of long whole records (at least W8_MIN_STEPS steps) belong to the EXT 3 kernel,
        // the others to the EXT 4 one; each scans past the other's runs
        if (W8K && args.w8_split == 2) {
            const bool tree = whole_run &&
                              __builtin_amdgcn_readfirstlane(gcm_steps<OPEN, FRAME>(recs[pos]) >= W8_MIN_STEPS ? 1u : 0u) != 0;
            if (tree != W8TREE) {
                if constexpr (!W8TREE) {  // (the pair's first kernel: the run's start into the list)
                    const bool fits = end <= 0xffffffffull;
                    if (args.w8_flags != nullptr && threadIdx.x == 0 && skipped_w8 < W8_SKIP_LIST && fits) {
                        u32 *f = args.w8_flags + (u64)blockIdx.x * W8_FLAG_WORDS + 1 + 2 * skipped_w8;
                        f[0] = (u32)pos, f[1] = (u32)end;
                    }
                    skipped_w8 = fits ? skipped_w8 + 1 : W8_SKIP_LIST + 1;
                }
                if (wave == 0 && nxt < nxt_end)
                    scan_run<OPEN, FRAME, false, EXT>(args, recs, nxt, nxt_end, rs_next);
                __syncthreads();
                pos = nxt, end = nxt_end, cstart = nxt_cstart;
                rb ^= 1;
                continue;
            }
        }
        // (EXT 3 is launched only as a pair's second kernel, w8_split 2: every run it keeps is whole, and its code for
        // cut runs goes; -13 VGPRs)
        const bool whole = W8TREE || whole_run;
        if (key_idx >= args.nkeys) {  // invalid key: nothing is written except a failed ok byte
            if (OPEN)
                for (u64 t = pos + threadIdx.x; t < run_end; t += blockDim.x)
                    args.ok[ok_at(t)] = 0;
            if (wave == 0 && nxt < nxt_end)
                scan_run<OPEN, FRAME, false, EXT>(args, recs, nxt, nxt_end, rs_next);
            __syncthreads();
            if (with_hp) {  // (no unit loop to take them: the previous run's masks and this run's, by every thread)
                if (hp_n != 0)
                    HP_PASS(hp_pos, hp_pos + hp_n, threadIdx.x, blockDim.x);
                HP_PASS(pos, run_end, threadIdx.x, blockDim.x);
                hp_n = 0;
            }
            pos = nxt, end = nxt_end, cstart = nxt_cstart;
            rb ^= 1;
            continue;
        }
        ++runs_here;  // (this instantiation processes the run: ptls_mi355x_debug_counters)
        typedef __attribute__((address_space(3))) const KeyEntry lds_key_t;
        lds_key_t *key = (lds_key_t *)(rs + RUN_KEY_OFF);  // staged by the scanner
        // the EXT 3 kernel's runs (all W8: the others were skipped above) take the 8-bit Horner table (ghash.h)
        constexpr bool w8run = W8K;
        // W8 segment ends: the serial chain (1), the tree (2), or a whole run of the serial kernel in 4-lane groups (3:
        // Horner with H^4)
        const bool g4run = W8K && !W8TREE && (whole ? W8_G4 : W8_G4_CUT);
        const u32 w8mode = !w8run ? 0u : W8TREE ? 2u : g4run ? 3u : 1u;
        // (MEAS_BUILD_ONCE, measurement builds only: a workgroup's later runs keep its first run's tables -- wrong tags
        // for other keys -- to price the per-run build, profiles/r5/table_build_cost.txt)
        const bool key_new = key_idx != loaded_key && !(MEAS_BUILD_ONCE && loaded_key != 0xffffffffu);
        if (mk_n != 0) {
            // (round 6) an MK run: each connection's H^4 and H as 4-bit window-major tables in its slot (ghash.h),
            // 128 threads a table; the next other run rebuilds its own tables (loaded_key none)
            static_assert(ENGINE_WG >= 2 * MK_SLOTS * 128, "a table per 128 threads");
            const u32 t = threadIdx.x >> 7, slot = t >> 1;
            if (slot < mk_n) {
                lds_key_t *kp = mk_key(rs, slot);
                const u32 el = (t & 1) ? 0u : 3u;  // H, H^4
                build_elem_table_w4(lds, slot * MK_SLOT_BYTES + (t & 1) * GHASH_TABLE_BYTES,
                                    u32x4{kp->h[el][0], kp->h[el][1], kp->h[el][2], kp->h[el][3]}, 128u * t);
            }
            __syncthreads();
            loaded_key = 0xffffffffu;
            loaded_usrc = 0xffffffffu;
            loaded_w8 = 4;
        } else if (w8run && (key_new || loaded_w8 != w8mode)) {
            // the 8-bit H^8 (H^4) table over slots 0..7, H in slot 8, and a cut run's combine power (or the tree's H^2)
            // at W8_TAB_COMB
            w8_build_tables(lds, (const lds_u8 *)key, whole ? 0xffffffffu : usrc, w8mode == 2, w8mode == 3 ? 3u : 7u);
            loaded_key = key_idx;
            loaded_usrc = whole ? 0xffffffffu : usrc;
            loaded_w8 = w8mode;
            if (threadIdx.x == 0)
                PROF_ADD(7, 1);
        } else if (w8run && !whole && usrc != loaded_usrc) {  // the same key, another unit length: its combine power
            build_elem_table(lds, W8_TAB_COMB, u32x4{key->h[usrc][0], key->h[usrc][1], key->h[usrc][2], key->h[usrc][3]}, 0, true);
            __syncthreads();
            loaded_usrc = usrc;
        } else if (!w8run && (key_idx != loaded_key || loaded_w8 || (!whole && usrc != loaded_usrc))) {
            // H^1..H^8 and the unit combine power (only the latter when just the unit length changed; constant-time
            // mode: its powers in tables 4..6 too)
            constexpr bool CTT = CT && CT_COMB_TREE_ON;
            build_ghash_tables(lds, key, 9, usrc, key_idx != loaded_key || loaded_w8 ? 0u : CTT ? 4u : 8u, 0, 0, CTT,
                               GHASH_WMASK(CT));
            __syncthreads();
            loaded_key = key_idx;
            loaded_usrc = usrc;
            loaded_w8 = 0;
            if (threadIdx.x == 0)
                PROF_ADD(7, 1);
        }
#if ENGINE_PROFILE
        unsigned long long t2 = stamp();
#endif
        if (MK_RUNS && EXT == 5 && mk_n != 0) {
            ++mk_here;  // (ptls_mi355x_debug_counters: MK runs)
#if MK_EARLY_SCAN
            // the workgroup's last wave scans the next run before it claims: the scan's memory round trips then wait
            // while the other waves work, instead of after the claims, when all of them would wait for it
            if (wave == ENGINE_WG / 64 - 1) {
                u32 claim = 0;
                if (lane_here() == 0)
                    claim = atomicAdd((u32 *)&rs[RC_CLAIM], 1u) == 0;
                PROF_STAMP(ts0);
                if (__builtin_amdgcn_readfirstlane(claim) && nxt < nxt_end)
                    scan_run<OPEN, FRAME, false, EXT>(args, recs, nxt, nxt_end, rs_next);
#if ENGINE_PROFILE
                if (lane_here() == 0)  // [15] the early scans' cycles
                    PROF_ADD(15, stamp() - ts0);
#endif
            }
#endif
            {
                // (round 6) an MK run: each wave claims one of the run's claims (up to 16 records of one connection,
                // scan_mk) and runs them as a whole run's 4-lane groups do, with the connection's round keys and IV in
                // SGPRs and its tables' slot (gmul4w, w8_lane_end4 on the slot's H)
                constexpr u32 G4 = 4;
                for (;;) {
                    u32 cb = 0;
                    if (lane_here() == 0)
                        cb = atomicAdd((u32 *)&rs[RC_NEXT], 1u);
                    cb = __builtin_amdgcn_readfirstlane(cb);
                    if (cb >= total_units)
                        break;
                    PROF_STAMP(tc0);
                    const u32 e = __builtin_amdgcn_readfirstlane(rs[RUN_UBASE_OFF + cb]);
                    const u32 mk_first = e & 0xffu, mk_cnt = (e >> 8) & 0xffu, slot = e >> 16;
                    lds_key_t *kp = mk_key(rs, slot);
                    u32 rkm[NR + 1][4];
#pragma unroll
                    for (int r = 0; r <= NR; ++r)
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            rkm[r][c] = __builtin_amdgcn_readfirstlane(kp->rk[r][c]);
                    const u32 mv0 = __builtin_amdgcn_readfirstlane(kp->iv[0]), mv1 = __builtin_amdgcn_readfirstlane(kp->iv[1]),
                              mv2 = __builtin_amdgcn_readfirstlane(kp->iv[2]);
                    u32x4 acc;
                    u32 okw;
                    {
                        const u32 lane = lane_here(), j = lane % G4, qd = lane / G4;
                        const u32 laneoff = (lane & 31) * 4 | W8_AES_BASE;
                        const bool valid = qd < mk_cnt;
                        ptls_mi355x_record_t r = {};
                        if (valid)
                            r = recs[pos + mk_first + qd];
                        const bool live = valid && record_ok<FRAME>(args, r);  // (scan_mk took accepted ones only)
                        if (!live)
                            r.len = 0, r.aad_len = 0, r.flags = 0;
                        const u32 ekslot = CLDS_PART + 16u * (threadIdx.x / G4);
                        gcm_segment<NR, OPEN, 1, FRAME, CT, true, (int)G4, true>(
                            args, lds, rkm, mv0, mv1, mv2, r, live, 0u, live ? 2u * gcm_steps<OPEN, FRAME>(r) : 0u, j, laneoff, 0u, acc,
                            true, okw, true, ekslot, false, mk_kslot(slot));
                    }
                    asm volatile("" ::: "memory");
                    const u32 qd = lane_here() / G4;
                    if (OPEN && okw <= 1 && qd < mk_cnt)  // the tag check (its length lane)
                        args.ok[ok_at(pos + mk_first + qd)] = (uint8_t)okw;
#if ENGINE_PROFILE
                    if (lane_here() == 0)  // [13] MK claims' cycles, [14] MK claims
                        PROF_ADD(13, stamp() - tc0), PROF_ADD(14, 1);
#endif
                }
            }
        } else {
#if ENGINE_PROFILE
        t2 = stamp();
#endif
        u32 rk[NR + 1][4];
#pragma unroll
        for (int r = 0; r <= NR; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                rk[r][c] = __builtin_amdgcn_readfirstlane(key->rk[r][c]);
        const u32 iv0 = __builtin_amdgcn_readfirstlane(key->iv[0]), iv1 = __builtin_amdgcn_readfirstlane(key->iv[1]),
                  iv2 = __builtin_amdgcn_readfirstlane(key->iv[2]);

        // ---- units: each wave takes RPW consecutive units (one per group) at a time
        // unit_of: the group's unit u -> its record (lo, in run order), the record's first unit, its unit count and
        // how many of its units follow this one (k_back), from the run state in LDS. It runs again after the segment
        // instead of keeping these values (and the descriptor, the ok index) live across it: kept, they were spilled to
        // scratch once per unit (the open kernels: 13 spill stores, which reached HBM as extra writes).
        auto unit_of = [&](u32 u, u32 &lo, u32 &first, u32 &unc, u32 &k_back) {
            lo = u, first = u, unc = 1, k_back = 0;
            if (whole)
                return;
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
        };
        bool g4done = false;
        if constexpr (W8K && !W8TREE && (W8_G4 || W8_G4_CUT)) {
            if (g4run) {
                // (round 5) the serial W8 kernel's whole runs (and with W8_G4_CUT its cut runs): 16 units a wave in
                // 4-lane groups (ghash.h). A whole run gives each group a record on 64-byte aligned steps; a cut run's
                // units keep their 8-lane-step bounds (the stream padded to a multiple of 8 positions, unit k of a
                // record ending 128 * k positions before its end), each taken in twice as many 4-lane steps, so the
                // partials, their slots and the combine power are the 8-lane kernel's
                constexpr u32 G4 = 4, RPW4 = 64 / G4;
                ++g4_here;  // (ptls_mi355x_debug_counters: runs in 4-lane groups)
                for (;;) {
                    u32 ub = 0;
                    if (lane_here() == 0)
                        ub = atomicAdd((u32 *)&rs[RC_NEXT], RPW4);
                    ub = __builtin_amdgcn_readfirstlane(ub);
                    if (ub >= total_units)
                        break;
                    u32x4 acc;
                    u32 okw;
                    {
                        const u32 lane = lane_here(), j = lane % G4, u = ub + lane / G4;
                        const u32 laneoff = (lane & 31) * 4 | W8_AES_BASE;
                        const bool valid = u < total_units;
                        u32 lo, first, unc, k_back;
                        unit_of(valid ? u : 0u, lo, first, unc, k_back);
                        ptls_mi355x_record_t r = {};
                        if (valid)
                            r = recs[pos + lo];
                        const bool live = valid && record_ok<FRAME>(args, r);
                        if (valid && !live) {  // rejected descriptor (one unit): nothing is written
                            r.len = 0, r.aad_len = 0, r.flags = 0;
                            if (OPEN && j == 0)
                                args.ok[ok_at(pos + lo)] = 0;
                        }
                        // the unit's 8-lane steps [m_lo, m_hi), as the 8-lane loop computes them
                        const u32 steps = gcm_steps<OPEN, FRAME>(r);
                        u32 m_hi = steps, m_lo = 0;
                        if (!whole) {
                            const u32 ulen = unit_mul(steps, ulog2, run_unit_cap(args)) * ustep;
                            m_hi = steps - k_back * ulen;
                            m_lo = k_back + 1 == unc ? 0u : m_hi - ulen;
                        }
                        if (!live)
                            m_lo = m_hi = 0;
                        const u32 ekslot = CLDS_PART + 16u * (whole ? threadIdx.x / G4 : first + unc - 1);
                        gcm_segment<NR, OPEN, 1, FRAME, CT, true, (int)G4>(args, lds, rk, iv0, iv1, iv2, r, live, 2u * m_lo,
                                                                         2u * m_hi, j, laneoff, tsel_horner, acc,
                                                                         unc == 1, okw, whole, ekslot, false);
                    }
                    asm volatile("" ::: "memory");
                    const u32 lane = lane_here(), j = lane % G4, u = ub + lane / G4;
                    if (u >= total_units)
                        continue;  // (uniform over the group)
                    u32 lo, first, unc, k_back;
                    unit_of(u, lo, first, unc, k_back);
                    if (OPEN && okw <= 1)  // a whole record's tag check (its length lane)
                        args.ok[ok_at(pos + lo)] = (uint8_t)okw;
                    if constexpr (W8_G4_CUT) {
                        if (unc > 1) {  // uniform over the group; a rejected descriptor is always one unit
                            u32 last = 0;
                            if (j == G4 - 1) {
                                s_part[first + unc - 1 - k_back] = acc;
                                __threadfence_block();  // the partial lands before the count that publishes it
                                last = atomicAdd((u32 *)&s_done[lo], 1u) == unc - 1;
                            }
                            last = (u32)__builtin_amdgcn_update_dpp(0, (int)last, 0xFF, 0xF, 0xF, false);  // quad lane 3
                            if (last) {
                                // the record's GHASH: Horner over its partials with the unit power (W8_TAB_COMB), a
                                // scattered chain over the quad (lane j carries dword j)
                                const ptls_mi355x_record_t r = recs[pos + lo];
                                const u32 mul = unit_mul(gcm_steps<OPEN, FRAME>(r), ulog2, run_unit_cap(args));
                                const Group4Ws k = group4_ws(tsel_chunk, lane);
                                const u32x4 z = {0, 0, 0, 0};
                                u32 gs = ((const lds_u32 *)(s_part + first))[j];
                                for (u32 i = 1; i < unc; ++i) {
                                    for (u32 t = 0; t < mul; ++t)  // (mul > 1: huge records only)
                                        gs = group4_scatter(group4_ws_terms(gs, k, z), lane);
                                    gs ^= ((const lds_u32 *)(s_part + first + i))[j];
                                }
                                const u32x4 tag = {(u32)__builtin_amdgcn_update_dpp(0, (int)gs, 0x00, 0xF, 0xF, false),
                                                   (u32)__builtin_amdgcn_update_dpp(0, (int)gs, 0x55, 0xF, 0xF, false),
                                                   (u32)__builtin_amdgcn_update_dpp(0, (int)gs, 0xAA, 0xF, 0xF, false),
                                                   (u32)__builtin_amdgcn_update_dpp(0, (int)gs, 0xFF, 0xF, 0xF, false)};
                                if (j != G4 - 1) {
                                } else if (OPEN) {
                                    const u32x4 rt = *(const u32x4_u *)(args.in + r.in_off + frame_in_skip<OPEN, FRAME>() +
                                                                        gcm_text_len<OPEN, FRAME>(r));
                                    const u32x4 d = rt ^ tag;
                                    args.ok[ok_at(pos + lo)] = (d[0] | d[1] | d[2] | d[3]) == 0;
                                } else {
                                    *(u32x4_u *)(args.out + r.out_off + frame_out_skip<OPEN, FRAME>() +
                                                 gcm_text_len<OPEN, FRAME>(r)) = tag;
                                }
                            }
                        }
                    }
                }
                g4done = true;
            }
        }
        if (!g4done)
        for (;;) {
            u32 ub = 0;
            if (lane_here() == 0)
                ub = atomicAdd((u32 *)&rs[RC_NEXT], (u32)RPW);
            ub = __builtin_amdgcn_readfirstlane(ub);
            if (ub >= total_units) {
                if (with_hp && hp_n != 0) {  // the run's units are all handed out: masks of the previous run
                    u32 m = 0;
                    if (lane_here() == 0)
                        m = atomicAdd((u32 *)&rs[RC_HPNEXT], (u32)HP_ITEM);
                    m = __builtin_amdgcn_readfirstlane(m);
                    if (m < hp_n) {
                        HP_PASS(hp_pos + m, hp_pos + min(hp_n, m + (u32)HP_ITEM), lane_here(), 64u);
                        continue;
                    }
                }
                break;
            }
            u32x4 acc;
            u32 okw;
            {
                const u32 lane = lane_here(), j = lane % G, slot = lane / G, laneoff = (lane & 31) * 4 | (W8K ? W8_AES_BASE : 0u);
                const u32 u = ub + slot;
                const bool valid = u < total_units;
                u32 lo, first, unc, k_back;
                unit_of(valid ? u : 0u, lo, first, unc, k_back);
                ptls_mi355x_record_t r = {};
                if (valid)
                    r = recs[pos + lo];
                // a long record of a spread launch is another workgroup's (spread_pieces): nothing here, not even ok
                const bool spread = SPREAD && valid && spread_long(args, r);
                const bool live = valid && !spread && record_ok<FRAME>(args, r);
                if (valid && !live) {  // rejected descriptor: the scan gave it one unit; nothing is written
                    r.len = 0, r.aad_len = 0, r.flags = 0;
                    if (OPEN && j == 0 && !spread)
                        args.ok[ok_at(pos + lo)] = 0;
                }
                const u32 steps = gcm_steps<OPEN, FRAME>(r);
                // unit [m_lo, m_hi) of the record's steps (whole mode: the record); huge records take longer units
                const u32 mul = whole ? 1u : unit_mul(steps, ulog2, run_unit_cap(args));
                u32 m_hi = steps, m_lo = 0;
                if (!whole) {
                    const u32 ulen = mul * ustep;
                    m_hi = steps - k_back * ulen;
                    m_lo = k_back + 1 == unc ? 0u : m_hi - ulen;
                }
                if (!live)
                    m_lo = m_hi = 0;
                // (constant-time mode: E(K, J0) waits in the slot of the record's last unit partial, or of the group
                // in a whole-record run, which has no partials)
                const u32 ekslot = CLDS_PART + 16u * (whole ? threadIdx.x / G : first + unc - 1);
                gcm_segment<NR, OPEN, 1, FRAME, CT, W8K>(args, lds, rk, iv0, iv1, iv2, r, live, m_lo, m_hi, j, laneoff,
                                                         tsel_horner, acc, unc == 1, okw, whole, ekslot, W8TREE);
            }
            // from here on everything is read again (run state, descriptor), not carried across the segment
            asm volatile("" ::: "memory");
            const u32 lane = lane_here(), j = lane % G, u = ub + lane / G;
            if (u >= total_units)
                continue;  // (uniform over the group)
            u32 lo, first, unc, k_back;
            unit_of(u, lo, first, unc, k_back);
            if (OPEN && okw <= 1)  // a whole record's tag check (its length lane)
                args.ok[ok_at(pos + lo)] = (uint8_t)okw;
#if ENGINE_PROFILE
            PROF_STAMP(tc0);
#endif
            if (unc > 1) {  // uniform over the group; a rejected descriptor is always one unit
                u32 last = 0;
                if (j == G - 1) {
                    // stream order, the front unit first; the last unit (k_back 0, multiplier H^0 in the combine)
                    // carries E(K, J0) (gcm_segment), so the combine ends on the tag
                    s_part[first + unc - 1 - k_back] = acc;
                    __threadfence_block();  // the partial lands before the count that publishes it
                    last = atomicAdd((u32 *)&s_done[lo], 1u) == unc - 1;
                }
                last = dpp_bcast7(last, lane);
                if (last) {
                    const ptls_mi355x_record_t r = recs[pos + lo];
                    const u32 mul = unit_mul(gcm_steps<OPEN, FRAME>(r), ulog2, run_unit_cap(args));
                    // last unit of the record: GHASH = Horner over the partials with H^(G * ulen) = (H^(G * ustep))^mul
                    // (whole group)
                    // (CT: each lane forms the whole product from the same table rows, instead of a share of it from
                    // its own window rows)
                    u32x4 g;
                    if (CT && CT_COMB_TREE_ON && mul == 1) {
                        g = ct_combine_tree(lds, s_part + first, unc, j);
                    } else if constexpr (SEG_COOP && COMBINE_SCATTER) {
                        // (round 5) a scattered chain (ghash.h): each lane carries its dword of the running sum
                        const GroupWs k = group_ws(tsel_chunk, lane);
                        const u32 q = j >> 1;
                        const u32x4 z = {0, 0, 0, 0};
                        u32 gs = ((const lds_u32 *)(s_part + first))[q];
                        for (u32 i = 1; i < unc; ++i) {
                            for (u32 t = 0; t < mul; ++t)  // (mul > 1: huge records only)
                                gs = gmul_group_ws(lds, gs, k, z, lane);
                            gs ^= ((const lds_u32 *)(s_part + first + i))[q];
                        }
                        g = group_gather(gs, lane);
                    } else {
                        g = s_part[first];
                        for (u32 i = 1; i < unc; ++i) {
                            g = gmul_combine<CT>(lds, g, tsel_chunk, lane);
                            for (u32 t = 1; t < mul; ++t)  // huge records only
                                g = gmul_combine<CT>(lds, g, tsel_chunk, lane);
                            g ^= s_part[first + i];
                        }
                    }
                    const u32x4 tag = g;
                    if (j != G - 1) {
                    } else if (OPEN) {
                        const u32x4 rt = *(const u32x4_u *)(args.in + r.in_off + frame_in_skip<OPEN, FRAME>() +
                                                            gcm_text_len<OPEN, FRAME>(r));
                        const u32x4 d = rt ^ tag;
                        args.ok[ok_at(pos + lo)] = (d[0] | d[1] | d[2] | d[3]) == 0;
                    } else {
                        *(u32x4_u *)(args.out + r.out_off + frame_out_skip<OPEN, FRAME>() + gcm_text_len<OPEN, FRAME>(r)) = tag;
                    }
                }
            }
#if ENGINE_PROFILE
            if (lane_here() == 0)  // [11] wave cycles in the unit's combine tail, [12] unit rounds of the wave
                PROF_ADD(11, stamp() - tc0), PROF_ADD(12, 1);
#endif
        }
        }  // (not an MK run)
        // the run's units are all handed out: the first wave to get here scans the next run into the other buffer
        // while the rest finish theirs
        u32 claim = 0;
        if (lane_here() == 0)
            claim = atomicAdd((u32 *)&rs[RC_CLAIM], 1u) == 0;
#if ENGINE_PROFILE
        PROF_STAMP(tsc);
#endif
        if (__builtin_amdgcn_readfirstlane(claim) && nxt < nxt_end)
            scan_run<OPEN, FRAME, false, EXT>(args, recs, nxt, nxt_end, rs_next);
        PROF_STAMP(tw);
        __syncthreads();  // the run's tables, partials and counters are free again
        if (with_hp)  // this run's records now await their masks (taken in the next run's unit loop)
            hp_pos = pos, hp_n = run_n;
        PROF_STAMP(t3);
#if ENGINE_PROFILE
        if (lane_here() == 0)
            PROF_ADD(4, t3 - tw);
        // (not an MK run) [13] the tail scan's cycles, [14] the scanning wave's wait at the barrier after it
        if (lane_here() == 0 && mk_n == 0 && __builtin_amdgcn_readfirstlane(claim) && nxt < nxt_end)
            PROF_ADD(13, tw - tsc), PROF_ADD(14, t3 - tw);
        if (threadIdx.x == 0) {
            PROF_ADD(0, t1 - t0);
            PROF_ADD(1, t2 - t1);
            PROF_ADD(2, t3 - t2);
            PROF_ADD(5, total_units);
            PROF_ADD(6, 1);
            if (pos == beg)
                PROF_ADD(3, t0 - tk);
        }
#endif
        pos = nxt, end = nxt_end, cstart = nxt_cstart;
        rb ^= 1;
    }
    if (with_hp && hp_n != 0)  // the last run's masks
        HP_PASS(hp_pos, hp_pos + hp_n, threadIdx.x, blockDim.x);
    if constexpr (W8K && !W8TREE) {  // the pair's first kernel, for the second (workgroup-uniform)
        if (args.w8_split == 2 && args.w8_flags != nullptr && threadIdx.x == 0)
            args.w8_flags[(u64)blockIdx.x * W8_FLAG_WORDS] = min(skipped_w8, (u32)W8_SKIP_LIST + 1);
    }
    if (ENGINE_HOOKS && threadIdx.x == 0) {
        if (runs_here != 0)
            atomicAdd(&g_ext_runs[blockIdx.x % EXT_RUN_ROWS][EXT == 5 ? 4 : EXT], (unsigned long long)runs_here);
        if (g4_here != 0)
            atomicAdd(&g_ext_runs[blockIdx.x % EXT_RUN_ROWS][7], (unsigned long long)g4_here);
        if (MK_RUNS && EXT == 5 && mk_here != 0)
            atomicAdd(&g_ext_runs[blockIdx.x % EXT_RUN_ROWS][6], (unsigned long long)mk_here);
    }
    if (kclock != nullptr && threadIdx.x == 0) {  // (vector stores and atomics only)
        const u64 t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        const u32 i = atomicAdd(&g_kclock_n, 1u);
        if (i < g_kclock_cap) {
            kclock[4 * i + 0] = kc_t0, kclock[4 * i + 1] = t1;
            kclock[4 * i + 2] = kc_r0, kclock[4 * i + 3] = r1;
        }
    }
    publish_done(args.done_flag, args.done_token);  // the per-record path polls these instead of waiting for the stream
#undef HP_PASS
}

#endif  // PTLS_MI355X_ENGINE_GCM_KERNELS_H
