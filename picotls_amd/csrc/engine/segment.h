// picotls_amd/csrc/engine/segment.h -- gcm_segment: AES-CTR + GHASH of a range of one record's stream by one 8-lane group.
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_SEGMENT_H
#define PTLS_MI355X_ENGINE_SEGMENT_H

// GHASH/CTR work of one G-lane group on steps [m_lo, m_hi) of record r's stream (see file header): lane j owns stream
// positions j + G*m and runs them NB at a time. The NB AES-CTR blocks of a step are independent (NB x 16 LDS lookups
// per round in flight); their GHASH folds stay sequential (Horner with H^G; each lane's last position in the segment
// with H^(end - position), from its own table). On return every lane of the group holds the segment's GHASH partial
// sum(X_i * H^(end - i)), plus E(K, J0) when the segment holds the record's length block: the length lane (lane
// (N - 1) mod G) encrypts J0 in that step and XORs it into its accumulator after its last multiply (the length block is
// the last stream position, H^0 in every later combine), so a finished record's GHASH sum is its tag, and E(K, J0)
// need not stay live through the loop (it was spilled to scratch once per segment); with CT only the length lane's
// partial includes it. Invalid groups pass m_lo == m_hi. With finish (a whole record), a seal writes the tag and an open
// returns the tag check in okw on the length lane (1 = verified, 0 = not; 2 on every other lane and without finish):
// the caller stores the ok byte, so the record's batch index need not stay live through the segment.
//
// Stream layout. Units of the chunked schedule end on step boundaries, so their stream [zero padding | AAD | text |
// length] is front-padded to a multiple of G positions (N = G * K). A whole record (ALIGNED: the lockstep kernel and the
// chunked kernel's whole-record runs) instead takes the front padding that puts its text blocks on 128-byte lines of the
// output: the group then stores one full line per step instead of parts of two (the parts of two cost 14.5 % more HBM
// writes and 2 % of seal time on 16 KiB records, profiles/r2_write_align.txt). Its stream ends where it ends (N any):
// lanes past the length block in the last step are idle, and each lane's last position p multiplies by H^(N - p), 1..G.
//
// Segment end (SEG_COOP, both modes, late round 3): a lane's last multiply by its own power H^e from its own
// nibble-major table read another table row than the lanes beside it, so its bank conflicts depended on the data
// (profiles/r2_ct_counters.txt). Now every lane keeps its last position unmultiplied, the wave's last step skips the
// Horner multiply, and coop_last_powers (ghash.h) applies the powers from window-major tables after the loop: 32
// conflict-free lookups per lane, E(K, J0) waiting in the caller's LDS slot (ekslot) and added on the length lane.
// Without SEG_COOP: CT (constant-time LDS access) with CT_TREE (round 3), every step multiplies by the uniform Horner table, a lane's last position stays unmultiplied, and
// after the loop a butterfly over the group's lanes applies the powers H^e (three levels with the tables H, H^2, H^4,
// then H once more: four uniform-table multiplies per segment). E(K, J0) then waits in an LDS slot of the caller's
// (ekslot) until the tree is done, and is added on the length lane only (lane jl: the lane the tag or the unit partial
// is taken from). The round-2 form (CT_TREE 0) ran four multiplies, H^8, H^4, H^2, H^1 kept on the bits of e, in every
// step in which some lane of the wave was at its last position (two or more steps per segment).
template <int NR, bool OPEN, int NB, int FRAME = 0, bool CT = false, bool W8 = false, int GG = ENGINE_G, bool MK4 = false>
__device__ __forceinline__ void gcm_segment(const BatchArgs &args, const lds_u8 *lds, const u32 (&rk)[NR + 1][4], u32 iv0,
                                            u32 iv1, u32 iv2, const ptls_mi355x_record_t &r, bool valid, u32 m_lo,
                                            u32 m_hi, u32 j, u32 laneoff, u32 tsel_horner, u32x4 &acc, bool finish,
                                            u32 &okw, bool aligned, u32 ekslot = 0, bool w8tree = false,
                                            u32 mk_kslot = MK_NONE)
{
    // G lanes per record: ENGINE_G, or 4 in the W8 serial kernel's whole runs (ghash.h, 4-lane groups), whose aligned
    // streams then put text blocks on 64-byte boundaries (a group stores 64 bytes a step)
    constexpr int G = GG;
    static_assert(G == 8 || (G == 4 && W8), "8-lane groups, or 4-lane groups in the W8 kernels");
#if ENGINE_PROFILE
    const unsigned long long tsg0 = stamp();
#endif
    constexpr int GS = G == 8 ? 3 : 2;  // log2 G
    // W8 (a W8 run of the pair's EXT 3 kernel, gcm_chunked_kernel): Horner on the 8-bit H^8 table (gmul8), the lanes'
    // last powers by a serial Horner over the group's ranks with the window-major H table (W8_TAB_H, w8_lane_end)
    constexpr bool COOP = SEG_COOP && !W8;  // the conflict-free segment end (coop_last_powers), both modes
    constexpr bool TREE = !W8 && !SEG_COOP && CT && CT_TREE;
    W8Lane w8 = {};
    if constexpr (W8)
        w8 = w8_lane(lane_here());
    // (round 6) MK4: a multi-key run's record (4-lane groups of the W8 serial kernel): the Horner on its connection's
    // 4-bit H^4 table (gmul4w) and the segment end on its H table, in the table slot mk_kslot names (ghash.h)
    static_assert(!MK4 || (W8 && G == 4), "MK runs are 4-lane W8 runs");
    MK4Lane mk4 = {};
    if constexpr (MK4)
        mk4 = mk4_lane(lane_here());
    auto horner = [&](u32x4 t) -> u32x4 {
        if constexpr (MK4)
            return gmul4w(lds, t, w8, mk4, mk_kslot);
        else
            return gmul8(lds, t, GMUL8_LANE(), w8);
    };
    constexpr bool SEAL_FRAME = FRAME == 1 && !OPEN, OPEN_FRAME = FRAME == 1 && OPEN, TLS12 = FRAME == 2;
    const u32 L = gcm_text_len<OPEN, FRAME>(r), A = gcm_aad_len<OPEN, FRAME>(r);
    // bytes of text readable at src (a framed seal reads len payload bytes; its last text byte is the content type)
    const u32 Lsrc = SEAL_FRAME ? L - 1 : L;
    const u32 na = (A + 15) >> 4, nb = (L + 15) >> 4;
    const u32 total = na + nb + 1;
    const uint8_t *src = args.in + r.in_off + frame_in_skip<OPEN, FRAME>();
    uint8_t *dst = args.out + r.out_off + frame_out_skip<OPEN, FRAME>();
    int P;
    u32 N;
    if (aligned) {  // text block b at position P + na + b, and (dst / 16 + b) mod G == that position mod G
        const u32 K0 = (total + G - 1) / G;
        P = (int)(((u32)((uintptr_t)dst >> 4) - na) & (G - 1));
        // (round 6) a 4-lane open puts text block 0 at a step's start instead: the steps before it need no keystream
        // (the seal's aligned output gives it the same padding), and the steady steps hold their blocks until a line is
        // whole (G4_LINE_HOLD)
        if constexpr (G4_OPEN_TEXT_STEPS && OPEN && G == 4)
            P = (int)((0u - na) & (G - 1));
        // ... unless that costs a record shorter than ALIGN_MIN_STEPS steps one more step (its wave would take it too:
        // -6 % on 1200-byte records), which keeps the padding of a multiple of G positions
        if ((u32)P + total > K0 * G && K0 < ALIGN_MIN_STEPS)
            P = (int)(K0 * G - total);
        N = (u32)P + total;
        if (valid)
            m_hi = (N + G - 1) / G;
    } else {  // (padded to a multiple of ENGINE_G positions for any G: 4-lane groups take the 8-lane units' bounds)
        const u32 K = (total + ENGINE_G - 1) / ENGINE_G;
        P = (int)(K * ENGINE_G) - (int)total;
        N = K * ENGINE_G;
    }
    // this lane's last step in the segment and its power there: at the record's end H^(N - p) for its last position p,
    // at a unit's end (a step boundary) H^(G - j)
    const bool at_end = aligned;
    const int m_last = !valid ? -1 : at_end ? ((int)N - 1 - (int)j) >> GS : (int)m_hi - 1;
    const u32 e_last = at_end ? N - ((u32)G * (u32)m_last + j) : (u32)G - j;  // 1..G
    const u32 tsel_last = 0x10000u + (e_last - 1) * GHASH_TABLE_BYTES;
    // the first step in which some lane of the group is at its last position (the steady range ends before it)
    const int m_first_last = at_end ? ((int)N - G) >> GS : (int)m_hi - 1;
    const u32 jl = (N - 1) & (G - 1);  // the length block's lane

    const u32 Smax = wave_max_perg<G>(m_hi - m_lo);  // m_lo, m_hi are uniform within a group

    // nonce = iv ^ (0^32 || BE64(seq)) (lib/picotls.c:6587-6601); TLS 1.2 takes the explicit nonce of the record in
    // place of seq, read as stored (big endian), so its two words need no swap
    u32 nw1 = bswap32((u32)(r.seq >> 32)), nw2 = bswap32((u32)r.seq);
    if (TLS12) {
        const uint8_t *e = args.in + r.in_off + (OPEN ? TLS_HEADER_SIZE : 0);
        nw1 = *(const u32_u *)e;
        nw2 = *(const u32_u *)(e + 4);
    }
    const u32 n0 = iv0 ^ rk[0][0];
    const u32 n1 = iv1 ^ nw1 ^ rk[0][1];
    const u32 n2 = iv2 ^ nw2 ^ rk[0][2];
    const uint8_t *aadp = OPEN_FRAME ? args.in + r.in_off : args.aad + r.aad_off;

    acc = u32x4{0, 0, 0, 0};

    static_assert(NB == 1, "the counter cache runs one block per lane and step");
    CtrCache1 cc1 = {};
    u32 cc1_key = 0xffffffffu;  // counter >> 8 of the cached window (none yet)

    // data block of lane j at step m: b = j + G*m - P - na; a full 16-byte input block is loaded one step ahead, so
    // its HBM latency hides under the AES of the current step
    auto full_block = [&](u32 m, int &b) -> bool {
        b = (int)(j + G * m) - P - (int)na;
        return m < m_hi && b >= 0 && b < (int)nb && Lsrc - 16u * (u32)b >= 16;
    };
    u32x4 nxt[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        int b;
        nxt[i] = u32x4{0, 0, 0, 0};
        if (full_block(m_lo + i, b))
            nxt[i] = *(const u32x4_u *)(src + 16u * (u32)b);
    }

    // step m, part 1: the next step's input prefetch and this step's counter block (refreshing the counter cache when
    // the lane enters a new 256-counter window)
    u32x4 cur;
    auto setup_step = [&](u32 m0, u32 (&st)[1][4], bool wave_ks) {
        cur = nxt[0];
        int bn;
        if (full_block(m0 + 1, bn))
            nxt[0] = *(const u32x4_u *)(src + 16u * (u32)bn);
        // AES-CTR input: data positions encrypt counter 2+b, all others J0 (kept by the length lane as E(K, J0))
        const int logical = (int)(j + G * m0) - P;
        const int b = logical - (int)na;
        const bool is_data = m0 < m_hi && logical >= (int)na && b < (int)nb;
        st[0][0] = n0, st[0][1] = n1, st[0][2] = n2;
        const u32 ctr = is_data ? (u32)(b + 2) : 1u;
        st[0][3] = bswap32(ctr) ^ rk[0][3];
        if (wave_ks && (ctr >> 8) != cc1_key) {  // entering a new 256-counter window (divergent; skipped when no lane does)
            cc1 = ctr_cache1_init<NR>(lds, laneoff, rk, n0, n1, n2, st[0][3]);
            cc1_key = ctr >> 8;
        }
    };
    // step m, part 2: with the keystream block ks, write the output and return the GHASH input block X of position
    // j + G*m
    auto finish_step = [&](u32 m, const u32x4 &ks, u32x4 &ek0) -> u32x4 {
        const bool act = m < m_hi;
        const int logical = (int)(j + G * m) - P;
        const int b = logical - (int)na;
        const bool is_data = act && logical >= (int)na && b < (int)nb;
        const bool is_aad = act && logical >= 0 && logical < (int)na;
        const bool is_len = act && logical == (int)(na + nb);
        u32x4 X = {0, 0, 0, 0};
#if ENGINE_FAST_STEP
        // steady state: every active lane of the wave holds a full 16-byte text block (one uniform branch, no
        // per-case dispatch)
        const bool full = is_data && Lsrc - 16u * (u32)b >= 16;
        if (__all(!act || full)) {
            const u32x4 o = cur ^ ks;
            if (act)
                *(u32x4_u *)(dst + 16u * (u32)b) = o;
            return OPEN ? cur : o;
        }
#endif
        if (is_data) {
            const u32 rem = L - 16u * (u32)b;
            uint8_t *op = dst + 16u * (u32)b;
            if (rem >= 16 && (!SEAL_FRAME || Lsrc - 16u * (u32)b >= 16)) {
                const u32x4 v = cur;
                const u32x4 o = v ^ ks;
                *(u32x4_u *)op = o;
                X = OPEN ? v : o;
            } else {
                const u32 srem = Lsrc - 16u * (u32)b;
                u32x4 v = load_partial(src + 16u * (u32)b, srem);
                if (SEAL_FRAME)  // the inner content type follows the payload
                    v[srem >> 2] |= (u32)(r.flags & 0xffu) << (8 * (srem & 3));
                const u32x4 o = rem >= 16 ? v ^ ks : mask_tail(v ^ ks, rem);
                if (rem >= 16)
                    *(u32x4_u *)op = o;
                else
                    store_partial(op, o, rem);
                X = OPEN ? v : o;
            }
        } else if (is_aad) {
            if (SEAL_FRAME) {  // the record header: built here, written to the wire, and authenticated
                const u32 wl = L + 16;
                X = u32x4{0x00030317u | ((wl >> 8) & 0xffu) << 24, wl & 0xffu, 0, 0};
                store_partial(args.out + r.out_off, X, TLS_HEADER_SIZE);
            } else if (TLS12) {  // AAD = BE64(seq) || type || 3 || 3 || BE16(len) (build_tls12_aad)
                const u32 type = OPEN ? (u32)args.in[r.in_off] : (r.flags & 0xffu);
                X = u32x4{bswap32((u32)(r.seq >> 32)), bswap32((u32)r.seq), type | 0x030300u | ((L >> 8) & 0xffu) << 24,
                          L & 0xffu};
                if (!OPEN) {  // the wire header and the explicit nonce
                    const u32 wl = TLS12_RECORD_IV_SIZE + L + 16;
                    const u32x4 h = {type | 0x030300u | ((wl >> 8) & 0xffu) << 24, (wl & 0xffu) | nw1 << 8,
                                     nw1 >> 24 | nw2 << 8, nw2 >> 24};
                    store_partial(args.out + r.out_off, h, TLS_HEADER_SIZE + TLS12_RECORD_IV_SIZE);
                }
            } else {
                const u32 rem = A - 16u * (u32)logical;
                const uint8_t *ap = aadp + 16u * (u32)logical;
                X = rem >= 16 ? *(const u32x4_u *)ap : load_partial(ap, rem);
            }
        } else if (is_len) {
            // (formed here, not hoisted: the loop-invariant length block was kept live through the loop and spilled)
            u32 Ah = A, Lh = L;
            asm volatile("" : "+v"(Ah), "+v"(Lh));
            const u64 abits = (u64)Ah * 8, cbits = (u64)Lh * 8;
            X[0] = bswap32((u32)(abits >> 32));
            X[1] = bswap32((u32)abits);
            X[2] = bswap32((u32)(cbits >> 32));
            X[3] = bswap32((u32)cbits);
            if (COOP || TREE || W8)  // (kept in LDS until after the loop: live through it, it was spilled)
                *(lds_u32x4 *)(const_cast<lds_u8 *>(lds) + ekslot) = ks;
            else
                ek0 = ks;
        }
        return X;
    };

    // Steady state: the steps [sa, sb) (relative to m_lo, wave-uniform) in which every lane of every group of the wave
    // holds a full text block, the next step's block is full too (the prefetch needs no check) and no group is at its
    // segment's last step (Horner with H^G throughout). They run without the per-lane position logic: the counter,
    // source and destination just advance by one step, about 30 VALU operations fewer per block.
    const int D0 = P + (int)na;         // stream position of text block 0
    const int nbf = (int)(Lsrc >> 4);   // full text blocks
    const int ms = (D0 + G - 1) / G;    // first step whose 8 positions are all >= D0
    const int me = nbf + D0 >= G ? (nbf + D0 - G) / G : -1;  // last step whose 8 positions are all full text
    int sa = max(ms, (int)m_lo) - (int)m_lo;
    int sb = min(me - 1, m_first_last - 1) + 1 - (int)m_lo;
    if (!valid || m_hi <= m_lo)
        sa = 1, sb = 0;
    sa = wave_smax_perg<G>(sa);
    sb = wave_smin_perg<G>(sb);

    // (round 6, PROGRESS_PRIO) the waves of a SIMD issue by the work they have left in the segment: the one furthest
    // behind first, so that equal claims end together instead of in the issue order's age skew (a run's last wave
    // otherwise finishes alone on its SIMD)
    auto progress_prio = [&](u32 left) {
        if constexpr (TREE_PRIO_BAND && W8) {
            if (w8tree) {
                const u32 q = left / TREE_PRIO_BAND;
                const u32 lvl = TREE_PRIO_INV ? (q >= 3 ? 0u : 3u - q) : (q >= 3 ? 3u : q);
                if (lvl == 3)
                    __builtin_amdgcn_s_setprio(3);
                else if (lvl == 2)
                    __builtin_amdgcn_s_setprio(2);
                else if (lvl == 1)
                    __builtin_amdgcn_s_setprio(1);
                else
                    __builtin_amdgcn_s_setprio(0);
                return;
            }
        }
        if constexpr (PROGRESS_PRIO && W8) {
            if (w8tree)  // (the tree kernel's long whole runs take TREE_PRIO_BAND above: bands of 4 measured -2.3 %)
                return;
            if (left > 3u * PROGRESS_PRIO)
                __builtin_amdgcn_s_setprio(3);
            else if (left > 2u * PROGRESS_PRIO)
                __builtin_amdgcn_s_setprio(2);
            else if (left > 1u * PROGRESS_PRIO)
                __builtin_amdgcn_s_setprio(1);
            else
                __builtin_amdgcn_s_setprio(0);
        }
    };
#if ENGINE_PROFILE
    const unsigned long long tsg1 = stamp();
    unsigned long long tsteady = 0;
#endif
    for (u32 s0 = 0; s0 < Smax; ++s0) {
        progress_prio(Smax - s0);
        if ((int)s0 == sa && sb > sa) {
#if ENGINE_PROFILE
            const unsigned long long tst0 = stamp();
#endif
            const int b0 = (int)(j + G * (m_lo + (u32)sa)) - D0;  // this lane's text block at step sa
            u32 off = 16u * (u32)b0;                               // its byte offset in the text
            u32 ctr = (u32)b0 + 2;
            // G4_PAIR_STORES: the block held from the previous step (the first half of its line), stored with this one
            constexpr bool LINE = G4_LINE_HOLD && G4_OPEN_TEXT_STEPS && OPEN && G == 4;
            constexpr bool PAIR = G4_PAIR_STORES && G == 4 && !LINE;
            u32x4 held = {0, 0, 0, 0};
            bool have = false;
            // G4_LINE_HOLD (a 4-lane open, its steps aligned to the text, not to the output): held = the lane's block
            // in a line's first half, held2 its block in the second half (the next step's). The line is whole at the
            // second half's step, or one step later for a lane past its first half's line offset ("late": j >
            // (dst + off) / 16 mod 4, the line's last block falls in the next step); then the lane stores both. Late
            // lanes store from dst - 64, so both kinds store at p - 64 and p
            u32x4 held2 = {0, 0, 0, 0};
            bool late = false;
            uint8_t *dst_l = dst;
            if constexpr (LINE) {
                late = j > (((u32)(uintptr_t)(dst + off) >> 4) & 3u);
                dst_l = dst - (late ? 64 : 0);
            }
            // G8_PAIR_STORES: a group whose steps straddle lines (a cut run's unit, counted from the stream's end) --
            // the lanes past the line boundary (the same lanes every step) hold their blocks one step, so each line is
            // stored by one step's instructions; uniform over the wave: no lane straddles in an aligned stream
            const bool holder = G == 8 && ((u32)(uintptr_t)(dst + off) & 127u) < 16u * j;
            // (unframed batches: the TLS-framed kernels measured slower with it, TLS 1.2 1200-byte seal -1.4 %)
            const bool pair8 = G8_PAIR_STORES && G == 8 && W8 && FRAME == 0 && !aligned && __any(holder);
            for (int s = sa; s < sb; ++s) {
                if ((s & 3) == 0)
                    progress_prio(Smax - (u32)s);
                cur = nxt[0];
                nxt[0] = *(const u32x4_u *)(src + off + 16 * G);
                u32 st[1][4] = {{n0, n1, n2, bswap32(ctr) ^ rk[0][3]}};
                if ((ctr >> 8) != cc1_key) {
                    cc1 = ctr_cache1_init<NR>(lds, laneoff, rk, n0, n1, n2, st[0][3]);
                    cc1_key = ctr >> 8;
                }
                aes_ctr_cached1<NR>(lds, laneoff, rk, cc1, st);
                __builtin_amdgcn_sched_barrier(0);
                const u32x4 o = cur ^ u32x4{st[0][0], st[0][1], st[0][2], st[0][3]};
                if constexpr (LINE) {
                    const bool first = (((u32)(uintptr_t)(dst + off)) & 64u) == 0;
                    if (!first)
                        held2 = o;
                    if (first == late) {  // the held line is whole at this step (held from inside the range only)
                        uint8_t *p = dst_l + off;
                        if (s >= sa + 1 + (int)late)
                            *(u32x4_u *)(p - 64) = held;
                        if (!late || s > sa)
                            *(u32x4_u *)p = held2;
                    }
                    if (first)
                        held = o;
                } else if constexpr (PAIR) {
                    if ((((uintptr_t)(dst + off)) & 64u) == 0 && s + 1 < sb) {
                        held = o;
                        have = true;
                    } else {
                        if (have)
                            *(u32x4_u *)(dst + off - 16 * G) = held;
                        *(u32x4_u *)(dst + off) = o;
                        have = false;
                    }
                } else if (pair8) {
                    if (have)
                        *(u32x4_u *)(dst + off - 16 * G) = held;
                    have = holder && s + 1 < sb;
                    if (have)
                        held = o;
                    else
                        *(u32x4_u *)(dst + off) = o;
                } else {
                    *(u32x4_u *)(dst + off) = o;
                }
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (W8)
                    acc = horner(acc ^ (OPEN ? cur : o));
                else
                    acc = gmul_tab(lds, acc ^ (OPEN ? cur : o), tsel_horner);
                __builtin_amdgcn_sched_barrier(0);
                ctr += G;
                off += 16 * G;
            }
            if constexpr (LINE) {  // the blocks still held after the range's last step
                uint8_t *p = dst + off - 16 * G;
                if ((((u32)(uintptr_t)p) & 64u) == 0) {
                    *(u32x4_u *)p = held;
                } else if (late) {
                    *(u32x4_u *)p = held2;
                    if (sb - 1 > sa)
                        *(u32x4_u *)(p - 64) = held;
                }
            }
            s0 = (u32)sb;  // (a block in the range's last step is stored at once: nothing is held past it)
#if ENGINE_PROFILE
            tsteady += stamp() - tst0;
#endif
        }
#if W8_LEAN_STEP
        if constexpr (W8 && FRAME == 0) {
            // (round 5) the W8 kernels' steps outside the steady range, unframed: every input that is not a full text
            // block (the AAD block, the record's partial last text block) is loaded before the AES, where its latency
            // hides, and the output cases are one chain of exec-masked branches instead of the per-case dispatch
            const u32 m0 = m_lo + s0;
            const bool act = m0 < m_hi;
            const int logical = (int)(j + G * m0) - P;
            const int b = logical - (int)na;
            const bool is_data = act && logical >= (int)na && b < (int)nb;
            const bool is_aad = act && logical >= 0 && logical < (int)na;
            const bool is_len = act && logical == (int)(na + nb);
            const u32 rem = L - 16u * (u32)b;  // (data positions)
            const bool full = is_data && rem >= 16;
            u32x4 xin = nxt[0];
            int bn;
            if (full_block(m0 + 1, bn))
                nxt[0] = *(const u32x4_u *)(src + 16u * (u32)bn);
            // (masked after the AES: a mask here would wait for the load before it)
            u32 nin = 16;
            if (is_aad) {
                const u32 arem = A - 16u * (u32)logical;
                const uint8_t *ap = aadp + 16u * (u32)logical;
                xin = arem >= 16 ? *(const u32x4_u *)ap : load_partial_raw(ap, arem);
                nin = min(arem, 16u);
            } else if (is_data && !full) {
                xin = load_partial_raw(src + 16u * (u32)b, rem);
                nin = rem;
            }
            // AES-CTR input: data positions encrypt counter 2 + b, all others J0 (the length lane keeps E(K, J0))
            const u32 ctr = is_data ? (u32)(b + 2) : 1u;
            u32 st[1][4] = {{n0, n1, n2, bswap32(ctr) ^ rk[0][3]}};
            if ((ctr >> 8) != cc1_key) {
                cc1 = ctr_cache1_init<NR>(lds, laneoff, rk, n0, n1, n2, st[0][3]);
                cc1_key = ctr >> 8;
            }
            aes_ctr_cached1<NR>(lds, laneoff, rk, cc1, st);
            __builtin_amdgcn_sched_barrier(0);
            const u32x4 ks = {st[0][0], st[0][1], st[0][2], st[0][3]};
            u32x4 X = {0, 0, 0, 0};
            if (full) {
                const u32x4 o = xin ^ ks;
                *(u32x4_u *)(dst + 16u * (u32)b) = o;
                X = OPEN ? xin : o;
            } else if (is_aad) {
                X = mask_tail(xin, nin);
            } else if (is_data) {
                const u32x4 v = mask_tail(xin, nin);
                const u32x4 o = mask_tail(v ^ ks, rem);
                store_partial(dst + 16u * (u32)b, o, rem);
                X = OPEN ? v : o;
            } else if (is_len) {
                u32 Ah = A, Lh = L;
                asm volatile("" : "+v"(Ah), "+v"(Lh));
                const u64 abits = (u64)Ah * 8, cbits = (u64)Lh * 8;
                X = u32x4{bswap32((u32)(abits >> 32)), bswap32((u32)abits), bswap32((u32)(cbits >> 32)),
                          bswap32((u32)cbits)};
                *(lds_u32x4 *)(const_cast<lds_u8 *>(lds) + ekslot) = ks;
            }
            __builtin_amdgcn_sched_barrier(0);
            // Horner with H^8 except at the lane's last position (its power comes in w8_lane_end); none in the wave's
            // last step
            const u32x4 t = acc ^ X;
            u32x4 prod = t;
            if (s0 + 1 < Smax) {
                prod = horner(t);
                if ((int)m0 == m_last)
                    prod = t;
            }
            if ((int)m0 <= m_last)
                acc = prod;
            __builtin_amdgcn_sched_barrier(0);
            continue;
        }
#endif
        const u32 m0 = m_lo + s0;
        // (round 5) a step in which no lane of the wave holds a text or length position (front padding and AAD only:
        // the first step of 4-lane groups on short records) needs no keystream and skips the AES; the lengths decide
        // it, not the data
        const int lg = (int)(j + G * m0) - P;
        // (4-lane groups only: in 8-lane kernels such a step is rare, and the test cost the TLS 1.3 open kernel spills)
        const bool wave_ks = !(SKIP_EMPTY_AES && G == 4) || __any(m0 < m_hi && lg >= (int)na && lg <= (int)(na + nb)) != 0;
        u32 st[1][4];
        setup_step(m0, st, wave_ks);
        if (wave_ks)
            aes_ctr_cached1<NR>(lds, laneoff, rk, cc1, st);
        __builtin_amdgcn_sched_barrier(0);
        u32x4 ek0 = {0, 0, 0, 0};
        const u32x4 X = finish_step(m0, u32x4{st[0][0], st[0][1], st[0][2], st[0][3]}, ek0);
        // scheduling fence: keeps the 32 table loads of this fold from being hoisted next to the other work (that
        // hoisting spills them to scratch)
        __builtin_amdgcn_sched_barrier(0);
        const bool last_here = (int)m0 == m_last;
        u32x4 prod;
        if (!W8 && !COOP && CT && CT_TREE) {
            // every lane multiplies by H^8, the uniform Horner table; a lane's last position stays unmultiplied and
            // takes its power H^e_last in the tree after the loop
            const u32x4 t = acc ^ X;
            prod = gmul_tab(lds, t, tsel_horner);
            if (last_here)
                prod = t;
        } else if (!W8 && !COOP && CT && __any(last_here)) {
            // H^8 (the Horner step, and a last power of 8), then H^4, H^2, H^1 kept on the bits of e_last; one
            // multiply site in a loop, so the branch costs no more registers than a plain step
            u32x4 t = acc ^ X;
            prod = t;
#pragma unroll 1
            for (u32 it = 0; it < 4; ++it) {
                const u32x4 q = gmul_tab(lds, t, 0x10000u + ((8u >> it) - 1u) * GHASH_TABLE_BYTES);
                if (it == 0)
                    prod = q;
                else if (e_last & (8u >> it))
                    t = q;
            }
            if (!last_here || e_last == (u32)G)
                t = prod;
            prod = t;
        } else if (COOP || W8) {
            // every lane multiplies by H^8, the uniform Horner table, except at its last position, which takes its
            // power H^e_last after the loop (coop_last_powers); in the wave's last step no lane needs the multiply
            const u32x4 t = acc ^ X;
            prod = t;
            if (s0 + 1 < Smax) {
                if constexpr (W8)
                    prod = horner(t);
                else
                    prod = gmul_tab(lds, t, tsel_horner);
                if (last_here)
                    prod = t;
            }
        } else {
            prod = gmul_tab(lds, acc ^ X, !CT && last_here ? tsel_last : tsel_horner);
        }
        if ((int)m0 <= m_last)
            acc = prod ^ ek0;
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PROGRESS_PRIO && W8)
        if (!w8tree || TREE_PRIO_BAND)
            __builtin_amdgcn_s_setprio(0);
#if ENGINE_PROFILE
    const unsigned long long tsg2 = stamp();
#endif

    static_assert(G == 8 || W8, "dpp_xor8 reduces groups of 8 lanes");
    // (round 5) an open's received tag is loaded before the segment end, whose lookups hide its latency (loaded after
    // it, the wave waited for it at every record's end: 2.3 % of the 1200-byte open)
    u32x4 rt = {0, 0, 0, 0};
    if (OPEN && finish && valid && j == jl)
        rt = *(const u32x4_u *)(src + L);
    if constexpr (W8) {
        // sum over the group of a_l H^(e_l) (rank r = 8 - e owes H^(8 - r)): ((v_0 H + v_1) H + ... + v_7) H by eight
        // group multiplies with the one window-major table H (4 conflict-free lookups per lane each: 32, as
        // coop_last_powers, with one table instead of seven)
        // (w8tree, the EXT 3 kernel's long whole records: the butterfly over the ranks with H and H^2 nibble-major)
        const u32 rank = valid ? (u32)G - e_last : j;
        if constexpr (G == 4)
            acc = w8_lane_end4(lds, acc, lane_here(), rank, MK4 ? mk_htab(mk_kslot) : (u32)W8_TAB_H);
        else if (w8tree)
            acc = w8_tree_end(lds, acc, lane_here(), rank);
        else
            acc = w8_lane_end(lds, acc, lane_here(), rank);
        if (valid && m_hi * G >= N && j == jl)  // the segment holds the length block: E(K, J0), on its lane
            acc ^= u32x4(*(const lds_u32x4 *)(lds + ekslot));
    } else if constexpr (TREE) {
        // sum over the group of a_l H^(e_l) (a_l: lane l's partial with its last position unmultiplied, e_l in 1..8 a
        // permutation over the lanes), as a butterfly over the ranks t = 8 - e: level k pairs rank t (bit k clear) with
        // rank t + k as v_t H^k + v_(t+k); every lane multiplies by the same table (H, H^2, H^4, then H once more) and
        // takes its partner's product or value through the crossbar. Lane l holds rank (l - rot) mod 8.
        const u32 lane = lane_here();
        const u32 rank = valid ? (u32)G - e_last : j;
        const u32 rot = (j - rank) & (G - 1);
        u32x4 v = acc;
#pragma unroll 1
        for (u32 lv = 0; lv < 3; ++lv) {
            const u32 k = 1u << lv;
            const u32x4 y = gmul_tab(lds, v, 0x10000u + (k - 1u) * GHASH_TABLE_BYTES);  // H^k
            const bool hi = (rank & k) != 0;
            const u32x4 send = hi ? v : y;
            const int src = (int)(((lane & ~(u32)(G - 1)) | (((rank ^ k) + rot) & (G - 1))) * 4);
            u32x4 recv;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                recv[c] = (u32)__builtin_amdgcn_ds_bpermute(src, (int)send[c]);
            v = hi ? (recv ^ v) : (y ^ recv);
        }
        acc = gmul_tab(lds, v, 0x10000u);  // * H
        if (valid && m_hi * G >= N && j == jl)  // the segment holds the length block: E(K, J0), on its lane
            acc ^= u32x4(*(const lds_u32x4 *)(lds + ekslot));
    } else {
        if constexpr (COOP) {  // the lanes' powers H^(e_last - 1), conflict-free (ghash.h); ranks rotated by N mod 8
            const u32 rank = valid ? (u32)G - e_last : j;
            acc = coop_last_powers(lds, acc, lane_here(), (j - rank) & (G - 1));
        }
        // XOR over the G lanes of the group
#pragma unroll
        for (int c = 0; c < 4; ++c)
            acc[c] = dpp_xor8(acc[c]);
        if constexpr (COOP)  // the group's sum times H (table 0, window-major)
            acc = gmul_group_w(lds, acc, LDS_AES_BYTES, lane_here());
        if (COOP && valid && m_hi * G >= N && j == jl)  // the segment holds the length block: E(K, J0), on its lane
            acc ^= u32x4(*(const lds_u32x4 *)(lds + ekslot));
    }
    // whole record (finish): tag = GHASH ^ E(K, J0), written after the ciphertext (seal) or compared with the
    // received one (open)
    okw = 2;
    if (finish && valid && j == jl) {
        const u32x4 tag = acc;
        if (OPEN) {
            const u32x4 d = rt ^ tag;
            okw = (d[0] | d[1] | d[2] | d[3]) == 0;
        } else {
            *(u32x4_u *)(dst + L) = tag;
        }
    }
#if ENGINE_PROFILE
    if (W8 && !w8tree && lane_here() == 0) {  // [16] setup, [17] steps, [18] end of the serial W8 kernels' segments, [19] segments
        const unsigned long long tsg3 = stamp();
        PROF_ADD(16, tsg1 - tsg0), PROF_ADD(17, tsg2 - tsg1), PROF_ADD(18, tsg3 - tsg2), PROF_ADD(19, 1);
        // [20] the wave's steps, [21] of them in the steady form
        PROF_ADD(20, Smax), PROF_ADD(21, sb > sa ? (u32)(sb - sa) : 0u), PROF_ADD(22, tsteady);
    }
#endif
}

#endif  // PTLS_MI355X_ENGINE_SEGMENT_H
