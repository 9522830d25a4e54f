// picotls_amd/csrc/engine/common.h -- Types, constants, the S-box, the keyset entry layout and small lane/GF helpers.
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_COMMON_H
#define PTLS_MI355X_ENGINE_COMMON_H

typedef uint32_t u32;
typedef uint64_t u64;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4_u;
typedef u32 __attribute__((aligned(1))) u32_u;

static_assert(sizeof(ptls_mi355x_record_t) == PTLS_MI355X_RECORD_SIZE, "record descriptor must be 40 bytes");
static_assert(sizeof(ptls_mi355x_cid_t) == 24, "CID descriptor must be 24 bytes");

// ------------------------------------------------------------------------------------------------ constants

namespace {

struct SboxTable {
    uint8_t v[256];
};

constexpr uint8_t xtime_c(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

// FIPS-197 S-box derived at compile time: multiplicative inverse via exp/log tables of generator 3, then the
// affine transform.
constexpr SboxTable make_sbox()
{
    uint8_t exp_t[256] = {}, log_t[256] = {};
    uint8_t x = 1;
    for (int i = 0; i < 255; ++i) {
        exp_t[i] = x;
        log_t[x] = (uint8_t)i;
        x = (uint8_t)(x ^ xtime_c(x));  // x * 3
    }
    SboxTable t = {};
    for (int v = 0; v < 256; ++v) {
        uint8_t inv = v == 0 ? 0 : exp_t[(255 - log_t[v]) % 255];
        uint8_t s = inv;
        for (int k = 1; k <= 4; ++k)
            s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
        t.v[v] = (uint8_t)(s ^ 0x63);
    }
    return t;
}

}  // namespace

__constant__ SboxTable c_sbox = make_sbox();

// one keyset entry in HBM (512 bytes, 16-byte aligned)
struct KeyEntry {
    u32 rk[15][4];  // round keys, LE column words; rounds 1..NR-1 stored rotated right by 8 bits (see aes_rounds_n)
    u32 iv[4];      // static IV as LE words (word 3 = 0)
    u32 h[16][4];   // GHASH elements (LE words): [0..7] = H^1..H^8, [8] = H^CHUNK_BLOCKS, [9..12] = H^16, H^32, H^64, H^128
                    // (the combine powers of smaller units), [13..15] = H^256, H^512, H^1024 (spread_pieces)
};
static_assert(sizeof(KeyEntry) == 512, "KeyEntry layout");

// The lane index, computed where it is used: the asm is volatile, so the compiler neither hoists it nor keeps a value
// derived from it live across the kernel's loops (such values were spilled to scratch and reloaded per unit and step).
__device__ __forceinline__ u32 lane_here()
{
    u32 x;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(x));
    return x;
}

// CT_PROBE_CONST=1 (a diagnosis build only, never shipped): every LDS lookup whose address comes from data (AES T-table
// bytes, GHASH operand bytes and nibbles) takes a constant operand instead, so the kernels' remaining LDS accesses are
// exactly those whose addresses come from lengths, indices and the work queue; its bank-conflict count against the
// product build's bounds what the data-dependent sites contribute (tools/gpu_r5.sh ct6)
#ifndef CT_PROBE_CONST
#define CT_PROBE_CONST 0
#endif

#ifndef ENGINE_FAST_STEP
#define ENGINE_FAST_STEP 1         // wave-uniform fast path for steps where every lane holds a full text block
#endif

#ifndef CT_TREE
#define CT_TREE 1                  // constant-time mode: the lanes' last powers by a uniform-table tree after the loop
#endif
#ifndef CT_COMBINE_TREE
#define CT_COMBINE_TREE 1          // constant-time mode: a record's unit partials combined by a uniform-table tree
#endif
#ifndef SEG_COOP
#define SEG_COOP 1                 // window-major power tables, the lanes' last powers by coop_last_powers (both modes)
#endif
// GHASH table layouts (build_ghash_tables `wmask`: bit t = table t window-major, ghash.h). With SEG_COOP the power
// tables H^1..H^7 (slots 0..6) and the unit combine power (slot 8, gmul_group_w) in both modes; H^8 (slot 7, the
// Horner table every lane reads at the same window) stays nibble-major.
#define GHASH_WMASK(ct) (SEG_COOP ? 0x17Fu : 0u)
// the constant-time mode's combine tree keeps combine powers in tables 4..6: only without SEG_COOP (H^5..H^7 there)
#define CT_COMB_TREE_ON (CT_COMBINE_TREE && !SEG_COOP)

#ifndef ALIGN_MIN_STEPS
#define ALIGN_MIN_STEPS 64         // whole records of this many steps may take one more step to align their stores
#endif

#define ENGINE_G 8                 // lanes per record
#ifndef ENGINE_NB
#define ENGINE_NB 1                // AES-CTR blocks per lane per step (independent chains in flight)
#endif
#ifndef ENGINE_WG
#define ENGINE_WG 1024             // threads per workgroup (one workgroup per CU)
#endif
#define ENGINE_WAVES_PER_SIMD (ENGINE_WG / 256)
#define LDS_AES_BYTES 65536        // Te0/Te2, 32-bank replicated
#define GHASH_TABLE_BYTES 8192     // 32 windows x 16 entries x 16 B
#define LDS_BYTES (LDS_AES_BYTES + ENGINE_G * GHASH_TABLE_BYTES)
#define LDS_EKSLOT (LDS_BYTES + 16)  // lockstep kernel: E(K, J0) slots, one per 8-lane group (gcm_segment's ekslot)
#define LDS_ALLOC (LDS_EKSLOT + 16 * (ENGINE_WG / ENGINE_G))  // + scratch word for the key-run scan, the E(K, J0) slots

// Chunked schedule (many-key batches): records are cut into units of at most CHUNK_BLOCKS GHASH-stream blocks, and
// the per-unit GHASH partials are recombined with H^CHUNK_BLOCKS (one more 8 KiB table, LDS table slot 8).
#ifndef CHUNK_BLOCKS
// 2 KiB units: 64K-key mixed +3 %, one-key mixed +7 % over 1 KiB units (interleaved A/B, round 1). 4 KiB units (256,
// round 2, profiles/r2_chunk_ab.txt): 64K-key mixed -2.3 %, random key order -1.5 %, one-key mixed +0.8 %
#define CHUNK_BLOCKS 128
#endif
#define CHUNK_STEPS (CHUNK_BLOCKS / ENGINE_G)
#define CHUNK_LOG2 (__builtin_ctz(CHUNK_STEPS))
#ifndef CHUNK_MAX_UNITS
#define CHUNK_MAX_UNITS CRUN_UNITS  // records longer than this many units (> ~2 MiB) use units of a multiple length
#endif
#define BKT_STRIDE (CHUNK_STEPS + 1)             // per-wave front-unit bucket counters in s_ctl (<= 32)
#define CRUN_RECS 256        // records per run (one key)
#ifndef CRUN_UNITS
#define CRUN_UNITS 1024      // units per run
#endif
#ifndef WHOLE_RUN_RECS
#define WHOLE_RUN_RECS 4096  // records per run when a one-key run is uniform (every record one unit)
#endif
#define UNIFORM_SLACK 2      // a run is uniform when its records' step counts differ by at most this
#define WHOLE_MIN_RECS (ENGINE_WG / ENGINE_G)  // whole-record mode needs at least one record per 8-lane group
// Per-run state, double-buffered so that one wave can scan run r+1 while the others finish run r (scan_run):
// ctl[16] | the run's KeyEntry | ubase u32[CRUN_RECS + 16] (first unit of each record) | done u32[CRUN_RECS] (finished units per record) |
// front u32[CRUN_RECS] (records by front-unit size). Then the unit partials (single: run r+1's units start after the
// end-of-run barrier).
#define RUN_CTL_WORDS 16
#define RUN_KEY_OFF RUN_CTL_WORDS                                 // the run's KeyEntry (512 B), staged by the scanner
#define RUN_UBASE_OFF (RUN_KEY_OFF + (int)(sizeof(KeyEntry) / 4))
#define RUN_DONE_OFF (RUN_UBASE_OFF + CRUN_RECS + 16)
#define RUN_FRONT_OFF (RUN_DONE_OFF + CRUN_RECS)
#define RUN_WORDS (RUN_FRONT_OFF + CRUN_RECS)
#define CLDS_RUN0 (LDS_BYTES + GHASH_TABLE_BYTES)
#define CLDS_RUN1 (CLDS_RUN0 + 4 * RUN_WORDS)
#define CLDS_PART (CLDS_RUN1 + 4 * RUN_WORDS)                    // 16 B per unit: GHASH partial
#define CLDS_ONE (CLDS_PART + 16 * CRUN_UNITS)                   // a lone record's descriptor (BatchArgs::one)
#define CLDS_ALLOC (CLDS_ONE + 48)
// W8 kernels (gcm_chunked_kernel EXT 3 and 4: the Horner step on an 8-bit H^8 table): every run of an unframed or
// TLS-framed batch, EXT 4 with the serial lane-Horner segment end, EXT 3 (long whole records, W8_MIN_STEPS steps and
// more) with the butterfly end. LDS map: AES [0, 64K), H^8 as an 8-bit window-major table over slots 0..7, H in slot 8
// (window-major for EXT 4, nibble-major for EXT 3), the unit partials of at most W8_RUN_UNITS units at CLDS_PART
// (their first 2 KiB the groups' E(K, J0) slots in whole runs; the table build's scratch before a run), at W8_TAB_COMB
// the unit combine power (window-major, EXT 4) or H^2 (nibble-major, EXT 3)
#ifndef W8_HORNER
#define W8_HORNER 1  // (round 4: on; profiles/r4/w8_ab.txt, w8all_ab.txt)
#endif
#ifndef W8_MIN_STEPS
#define W8_MIN_STEPS 64
#endif
#ifndef W8_TLS12
// TLS 1.2-framed batches in the W8 kernels too, although EXT 4's TLS 1.2 seal spills 96 B per lane: 131072 x 16 KiB
// records 1036.9 -> 1172.1 GiB/s seal+open, 1M x 1200 B 907.2 -> 979.1 (tools/ab_tls12.py, profiles/r4/tls12_w8_ab.txt)
#define W8_TLS12 1
#endif
#ifndef W8_MIN_RECS
// batches of fewer records keep the 4-bit kernel. Round 4 set 2048 (256 x 16 KiB -5 %, 1000 x 1200 B -4 %, 1000 x 16 KiB
// even, profiles/r4/w8all_ab.txt); with round 5's W8 kernels the 8-bit path is ahead from 256 records (256 x 16 KiB
// +1.8 %, 1000 x 16 KiB +3.2 %, 2000 x 16 KiB +2.3 %, 1000 x 1200 B +3.9 %) and even below (64 x 64 KiB, 100 x 16 KiB:
// ±0.3 % with 64), profiles/r5/w8_min_recs_ab.txt
#define W8_MIN_RECS 256
#endif
#ifndef W8_SWAP
// (round 5) the W8 kernels' LDS map puts the 8-bit H^8 table at [0, 64K) and the AES T-tables at [64K, 128K): the
// table's address bytes are then two (window, value), formed by one v_perm from registers that stay fixed through the
// loop, and the AES addresses take their 64 KiB slot from laneoff's byte 2 in the same v_perm (aes_tt.h TE_ADDR)
#define W8_SWAP 1
#endif
// (round 5) whole runs of the W8 serial kernel (EXT 4: uniform records under W8_MIN_STEPS steps) in 4-lane groups
// (ghash.h, gcm_chunked_kernel): quic1200 +3.3-3.9 % (profiles/r5/g4_ab.txt); 0 keeps 8-lane groups
#ifndef W8_G4
#define W8_G4 1
#endif
// (round 5) gmul8's selects by bit 3 of the lane from a constant lane mask (ghash.h)
// (round 5) steps without a text or length position skip the AES (segment.h)
#ifndef SKIP_EMPTY_AES
#define SKIP_EMPTY_AES 1
#endif
#ifndef GMUL8_CONST_MASK
#define GMUL8_CONST_MASK 1
#endif
#define GMUL8_LANE() (GMUL8_CONST_MASK && W8_SWAP ? 0u : lane_here())  // (lane_here is a volatile asm: not evaluated unless needed)
// ... and its cut runs too (the units keep their 8-lane-step bounds and combine power; gcm_chunked_kernel): measured
// -6 % on mixed (units twice as long in time, so the run tails wait twice as long; also with each run cut into at least
// 128 units), -18 % with units of half the length (twice the partials and combine links): off (profiles/r5/g4_ab.txt)
#ifndef W8_G4_CUT
#define W8_G4_CUT 0
#endif
// (round 5) the W8 kernels' unframed steps outside the steady range as one pass with the non-text inputs loaded ahead of
// the AES (segment.h): measured within +-0.5 % of the per-case setup_step / finish_step on quic1200 and mixed
// (profiles/r5/g4_ab.txt): off
#ifndef W8_LEAN_STEP
#define W8_LEAN_STEP 0
#endif
// (round 5) 4-lane groups store a line's two 64-byte halves together: a lane holds the first half's block one steady
// step and stores it beside the second (segment.h). Half lines stored a step apart leave the L2 as two write-backs of
// the line (tools/mb/wcal.hip: 1.07-1.08x the bytes; paired, 1.00x)
#ifndef G4_PAIR_STORES
#define G4_PAIR_STORES 1
#endif
// (round 6) a 4-lane group's open aligns its steps to the record's text, not to its output (segment.h): text block 0
// starts a step, so the AAD step needs no keystream, as in the seal (1200-byte open: 19 AES steps instead of 20)
#ifndef G4_OPEN_TEXT_STEPS
#define G4_OPEN_TEXT_STEPS 1
#endif
// ... and its steady steps, no longer aligned to the output's lines, still store every 128-byte line in one step: a lane
// holds up to two blocks (the line's halves) until the step that produces the line's last block (segment.h)
#ifndef G4_LINE_HOLD
#define G4_LINE_HOLD 1
#endif
// (round 6) the serial W8 kernels' waves issue by the steps left in their segment (s_setprio 3..0 in bands of this many
// steps, segment.h): the waves of a SIMD then end equal claims together instead of in the order of their age, which
// left a run's last wave alone on its SIMD. tls64k +4.3 %, quic64k +5.0 %, mixed +0.7 %, quic1200 +0.4 %; the tree
// kernel takes its own, wider bands (TREE_PRIO_BAND: with these, tls16k -2.3 %) (profiles/r6/progress_prio_ab.txt); 0: off
#ifndef PROGRESS_PRIO
#define PROGRESS_PRIO 4
#endif
// ... and the tree kernel's (EXT 3, long whole records) in bands of TREE_PRIO_BAND steps: 32 gave tls16k +0.4 / +0.7 %,
// AES-256 16 KiB +0.6 %, 256K x 16 KiB +2.2 % on two boxes, 16 a further +0.25 to +0.8 % on tls16k (bands of 4
// measured -2.3 %, of 64 -2 to -3 %; the waves nearest their segment's end first, TREE_PRIO_INV, -1 to -2 %)
// (profiles/r6/tree_prio_ab.txt, tree_prio_band_ab.txt); 0: the tree kernel keeps its issue order
#ifndef TREE_PRIO_BAND
#define TREE_PRIO_BAND 16
#endif
#ifndef TREE_PRIO_INV
#define TREE_PRIO_INV 0
#endif
// ... and 8-lane groups whose steps straddle lines (cut runs' units) store each line in one step (segment.h)
#ifndef G8_PAIR_STORES
#define G8_PAIR_STORES 1
#endif
// a W8 pair's flag block per workgroup (BatchArgs::w8_flags): [0] the runs EXT 4 left to EXT 3 (W8_SKIP_LIST + 1:
// more than the list holds, or records past 2^32), then per listed run (walk order) its first record and the end of
// the chunk that holds it
// (round 6) multi-key runs (MK runs, EXT 4): a many-key batch's connections of short uniform records (under
// W8_MIN_STEPS 8-lane steps, fewer than WHOLE_MIN_RECS records each: QUIC packets of many connections) share one
// whole-record run of up to MK_SLOTS connections and CRUN_RECS records, in 4-lane groups, each connection's 4-bit H^4 and
// H tables in a 16 KiB slot of [0, 64K) (ghash.h gmul4w). A connection's records are taken 16 at a time (a wave's
// "claim": one connection per wave, so its round keys stay in SGPRs). Run state: ctl[RC_MK] = connections (0: not an
// MK run), RC_UNITS = claims; the claims (first record | count << 8 | slot << 16) at RUN_UBASE_OFF, the key entries of
// slots 1.. at RUN_DONE_OFF (slot 0's at RUN_KEY_OFF, as any run's)
// (round 6) the scan tries an MK run only from a connection of MK_MIN_FIRST records: connections of one or two records
// stay cut into units, which spread over every wave where an MK run of such connections is one claim on one wave
// (64K connections of 2 packets +3.7 %, 100,000 mixed records over 64K keys +3.1 %, profiles/r6/mk_min_first_ab.txt)
#ifndef MK_MIN_FIRST
#define MK_MIN_FIRST 3
#endif
#ifndef MK_RUNS
#define MK_RUNS 1
#endif
#ifndef MK_EARLY_SCAN
#define MK_EARLY_SCAN 1
#endif
#define MK_SLOTS 4
#define MK_NONE 0xffffffffu
#define MK_SLOT_BYTES 16384
__host__ __device__ constexpr u32 mk_kslot(u32 slot) { return (slot << 6) * 0x01010101u; }  // slot bits in each byte
__host__ __device__ constexpr u32 mk_htab(u32 kslot) { return ((kslot & 0xc0u) << 8) + 8192u; }  // the slot's H table

#define W8_FLAG_WORDS 32
#define W8_SKIP_LIST ((W8_FLAG_WORDS - 1) / 2)
#define W8_H8_BASE (W8_SWAP ? 0u : (u32)LDS_AES_BYTES)   // the W8 kernels' 8-bit H^8 table
#define W8_AES_BASE (W8_SWAP ? (u32)LDS_AES_BYTES : 0u)  // ... and their AES T-tables
#define W8_RUN_UNITS 512  // units per run of a launch pair (both kernels: their runs must be the same)
#define W8_TAB_H (LDS_AES_BYTES + 8 * GHASH_TABLE_BYTES)
#define W8_TAB_COMB (CLDS_PART + 16 * W8_RUN_UNITS)
#define SPAN_MAX_UNITS CRUN_UNITS  // units per span of a long record (span_kernels.h, spread_pieces): the LDS partials
static_assert(CLDS_ALLOC <= 160 * 1024, "chunked schedule LDS budget");
static_assert(W8_TAB_COMB % 256 == 0 && W8_TAB_COMB + GHASH_TABLE_BYTES <= CLDS_ONE, "W8 combine table after the partials");
static_assert(16 * (ENGINE_WG / ENGINE_G) <= 16 * W8_RUN_UNITS && GHASH_TABLE_BYTES <= 16 * W8_RUN_UNITS,
              "E(K, J0) slots and the table build's scratch inside the W8 partial region");
static_assert(CHUNK_BLOCKS % ENGINE_G == 0, "units are whole steps");
static_assert((CHUNK_STEPS & (CHUNK_STEPS - 1)) == 0 && CHUNK_STEPS <= 32, "unit lengths are powers of two up to 32 steps");


// ------------------------------------------------------------------------------------------------ small helpers

__device__ __forceinline__ u32 bswap32(u32 x) { return __builtin_bswap32(x); }
__device__ __forceinline__ u32 rotl8(u32 x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ u32 rotr8(u32 x) { return __builtin_amdgcn_alignbit(x, x, 8); }
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// Cross-lane steps on the VALU (DPP) instead of the LDS crossbar (__shfl lowers to ds_bpermute, which competes with the
// table lookups for the LDS): XOR over each aligned group of 8 lanes (quad_perm [1,0,3,2], [2,3,0,1], then
// row_half_mirror pairs the two quads), result in all 8 lanes.
__device__ __forceinline__ u32 dpp_xor8(u32 v)
{
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    return v;
}
// lane 7 of each aligned 8-lane group, to all 8 lanes (quad_perm [3,3,3,3], then row_half_mirror for lanes 0-3)
__device__ __forceinline__ u32 dpp_bcast7(u32 v, u32 lane)
{
    const u32 t = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xFF, 0xF, 0xF, false);
    const u32 u = (u32)__builtin_amdgcn_update_dpp(0, (int)t, 0x141, 0xF, 0xF, false);
    return (lane & 4) ? t : u;
}
// Whole-wave inclusive scans on DPP (row_shr 1/2/4/8 inside each 16-lane row, then row_bcast 15 / 31 across rows):
// six dependent VALU ops instead of six ds_bpermute round trips. Lanes without a source take the identity.
template <typename Op>
__device__ __forceinline__ u32 dpp_scan(u32 v, u32 ident, Op op)
{
    v = op(v, (u32)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x111, 0xF, 0xF, false));
    v = op(v, (u32)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x112, 0xF, 0xF, false));
    v = op(v, (u32)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x114, 0xF, 0xF, false));
    v = op(v, (u32)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x118, 0xF, 0xF, false));
    v = op(v, (u32)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x142, 0xA, 0xF, false));
    v = op(v, (u32)__builtin_amdgcn_update_dpp((int)ident, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}
__device__ __forceinline__ u32 wave_incl_sum(u32 v) { return dpp_scan(v, 0u, [](u32 a, u32 b) { return a + b; }); }
__device__ __forceinline__ u32 wave_min(u32 v)
{
    return (u32)__builtin_amdgcn_readlane((int)dpp_scan(v, 0xffffffffu, [](u32 a, u32 b) { return min(a, b); }), 63);
}
__device__ __forceinline__ u32 wave_max(u32 v)
{
    return (u32)__builtin_amdgcn_readlane((int)dpp_scan(v, 0u, [](u32 a, u32 b) { return max(a, b); }), 63);
}

// maximum / signed maximum / signed minimum over the wave of a value that is uniform within each 8-lane group: the two
// groups of a 16-lane row meet through one DPP row rotation by 8, then four reads (one per row) instead of eight
__device__ __forceinline__ u32 row_ror8(u32 v)
{
    return (u32)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
}
__device__ __forceinline__ u32 wave_max_per8(u32 v)
{
    const u32 r = max(v, row_ror8(v));
    return max(max((u32)__builtin_amdgcn_readlane((int)r, 0), (u32)__builtin_amdgcn_readlane((int)r, 16)),
               max((u32)__builtin_amdgcn_readlane((int)r, 32), (u32)__builtin_amdgcn_readlane((int)r, 48)));
}
__device__ __forceinline__ int wave_smax_per8(int v)
{
    const int r = max(v, (int)row_ror8((u32)v));
    return max(max(__builtin_amdgcn_readlane(r, 0), __builtin_amdgcn_readlane(r, 16)),
               max(__builtin_amdgcn_readlane(r, 32), __builtin_amdgcn_readlane(r, 48)));
}
__device__ __forceinline__ int wave_smin_per8(int v)
{
    const int r = min(v, (int)row_ror8((u32)v));
    return min(min(__builtin_amdgcn_readlane(r, 0), __builtin_amdgcn_readlane(r, 16)),
               min(__builtin_amdgcn_readlane(r, 32), __builtin_amdgcn_readlane(r, 48)));
}
// the same over groups of G lanes (G = 8 above; G = 4: the 4-lane groups of a row meet through rotations by 4 and 8)
template <int G>
__device__ __forceinline__ u32 row_group_reduce_rot(u32 v, bool is_max, bool is_signed)
{
    auto op = [&](u32 a, u32 b) -> u32 {
        if (is_signed)
            return (u32)(is_max ? max((int)a, (int)b) : min((int)a, (int)b));
        return is_max ? max(a, b) : min(a, b);
    };
    if constexpr (G == 4)
        v = op(v, (u32)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x124, 0xf, 0xf, false));  // row_ror:4
    return op(v, row_ror8(v));
}
template <int G>
__device__ __forceinline__ u32 wave_max_perg(u32 v)
{
    if constexpr (G == 8)
        return wave_max_per8(v);
    const u32 r = row_group_reduce_rot<G>(v, true, false);
    return max(max((u32)__builtin_amdgcn_readlane((int)r, 0), (u32)__builtin_amdgcn_readlane((int)r, 16)),
               max((u32)__builtin_amdgcn_readlane((int)r, 32), (u32)__builtin_amdgcn_readlane((int)r, 48)));
}
template <int G>
__device__ __forceinline__ int wave_smax_perg(int v)
{
    if constexpr (G == 8)
        return wave_smax_per8(v);
    const int r = (int)row_group_reduce_rot<G>((u32)v, true, true);
    return max(max(__builtin_amdgcn_readlane(r, 0), __builtin_amdgcn_readlane(r, 16)),
               max(__builtin_amdgcn_readlane(r, 32), __builtin_amdgcn_readlane(r, 48)));
}
template <int G>
__device__ __forceinline__ int wave_smin_perg(int v)
{
    if constexpr (G == 8)
        return wave_smin_per8(v);
    const int r = (int)row_group_reduce_rot<G>((u32)v, false, true);
    return min(min(__builtin_amdgcn_readlane(r, 0), __builtin_amdgcn_readlane(r, 16)),
               min(__builtin_amdgcn_readlane(r, 32), __builtin_amdgcn_readlane(r, 48)));
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) u32 lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

// (b0..b3) *= x^s in GF(2^128), big-endian words (GCM bit order: the MSB of b0 is x^0), 1 <= s <= 32, in closed form:
// bit i of the s bits shifted out of b3 is x^(127 - i) and comes back as x^(s - 1 - i) * (1 + x + x^2 + x^7), i.e. the
// shifted-out bits land at the top of b0 ("1") and again 1, 2 and 7 bits further down, the last spilling into b1
__device__ __forceinline__ void gf_mulxs_be(u32 &b0, u32 &b1, u32 &b2, u32 &b3, u32 s)
{
    const u32 top = s == 32 ? b3 : b3 << (32 - s);
    if (s == 32) {
        b3 = b2, b2 = b1, b1 = b0, b0 = 0;
    } else {
        b3 = __builtin_amdgcn_alignbit(b2, b3, s);
        b2 = __builtin_amdgcn_alignbit(b1, b2, s);
        b1 = __builtin_amdgcn_alignbit(b0, b1, s);
        b0 >>= s;
    }
    const u64 v = (u64)top << 32;
    const u64 r = v ^ (v >> 1) ^ (v >> 2) ^ (v >> 7);
    b0 ^= (u32)(r >> 32);
    b1 ^= (u32)r;
}

// GF(2^128) * x on a GHASH element held as big-endian words (b0 most significant; bit 127 of the integer is x^0)
__device__ __forceinline__ void gf_mulx_be(u32 &b0, u32 &b1, u32 &b2, u32 &b3)
{
    u32 lsb = b3 & 1;
    b3 = (b3 >> 1) | (b2 << 31);
    b2 = (b2 >> 1) | (b1 << 31);
    b1 = (b1 >> 1) | (b0 << 31);
    b0 = (b0 >> 1) ^ (lsb ? 0xe1000000u : 0u);
}

// The per-record path's completion words (BatchArgs::done_flag, hp_kernel): every wave's stores of the workgroup complete
// at system scope, then one store per workgroup tells the host thread polling the mapped staging buffer. The word is
// the call's token (BatchArgs::done_token, never 0), not a constant: a word left set by an earlier call on the same
// staging buffer cannot pass for this call's completion.
__device__ __forceinline__ void publish_done(u32 *flags, u32 token)
{
    if (flags == nullptr)
        return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(flags + blockIdx.x, token, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Diagnostic build only (-DENGINE_PROFILE=1): s_memtime stamps of the chunked kernel's phases, summed over runs and
// workgroups: [0] run setup, [1] GHASH table build, [2] unit loop, [3] kernel prologue (AES tables, first scan), [4] wave idle at the unit-loop barrier,
// [5] units, [6] runs, [7] table builds.
#ifndef ENGINE_PROFILE
#define ENGINE_PROFILE 0
#endif
#if ENGINE_PROFILE
// one row of counters per workgroup (blockIdx.x mod PROF_ROWS): the rows are summed on the host, so the counter
// atomics of 256 workgroups do not queue on one address inside the phases they measure
#define PROF_ROWS 1024
#define PROF_SLOTS 24
__device__ unsigned long long g_prof[PROF_ROWS][PROF_SLOTS];
__device__ __forceinline__ unsigned long long stamp()
{
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define PROF_STAMP(v) const unsigned long long v = stamp()
#define PROF_ADD(i, v) atomicAdd(&g_prof[blockIdx.x % PROF_ROWS][i], (unsigned long long)(v))
#else
#define PROF_STAMP(v)
#define PROF_ADD(i, x)
#endif

#endif  // PTLS_MI355X_ENGINE_COMMON_H
