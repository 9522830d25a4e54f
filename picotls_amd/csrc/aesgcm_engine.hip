// picotls_amd/csrc/aesgcm_engine.hip -- MI355X (gfx950 / CDNA4) AES-GCM record engine: HIP kernels + the C ABI
// declared in include/picotls/mi355x.h.
//
// What it replaces: picotls' fusion AES-GCM engine (lib/fusion.c:401-845 seal/open, :847-929 AES core and key
// schedule, :114-321 + :934-1011 GHASH and H-power tables), re-designed for a GPU: one launch seals or opens a
// whole batch of independent records.
//
// Design (DESIGN.md has the numbers):
//   * one persistent 1024-thread workgroup per CU; G = 8 lanes of a wavefront work on one record, so a wave holds 8
//     records and lane j of a record handles GHASH stream positions j, j+G, j+2G, ... (the stream is
//     [zero padding | AAD blocks | ciphertext blocks | length block], front-padded to a multiple of G, which leaves
//     GHASH unchanged). A record's ciphertext block b sits at one stream position, so the lane that runs AES-CTR
//     on counter 2+b is the lane that folds that block into its GHASH accumulator: no data exchange.
//   * AES: T-table rounds from LDS. Te0 and Te2 (= rotl16 Te0) are replicated into all 32 banks
//     (entry n at n*256 + bank*4, Te2 at +128): lane l always reads bank l%32, so every ds_read_b32 is
//     conflict-free; Te1/Te3 are one v_alignbit away. The byte -> LDS address step is a single v_perm_b32.
//   * GHASH: 4-bit-window tables in LDS. For each H power one table = 32 windows x 16 entries x 16 B (8 KiB);
//     the 16 entries of a window fill exactly one 256-byte LDS bank row, so a ds_read_b128 of 16 lanes never
//     conflicts (equal entries broadcast). A product X*H^k is the XOR of 32 table entries; the reduction is baked
//     into the tables. Horner with stride H^G on every step except the last, where lane j multiplies by H^(G-j)
//     instead; an XOR over the G lanes then gives GHASH. Tables for H^1..H^G (64 KiB) are built on chip from the
//     keyset's H powers at kernel start.
//   * Data path: 16-byte unaligned-capable global loads/stores (unaligned access mode is on for gfx950), G lanes
//     of a record touch G*16 contiguous bytes per step. Partial first/last blocks use byte accesses so nothing
//     outside [in_off, in_off+len) / [out_off, out_off+len+16) is touched.
//
// All word-level state is kept in "LE column" form: a 16-byte block is 4 little-endian u32 words, word c = bytes
// 4c..4c+3 = AES state column c. GHASH elements use the same byte order (byte 0 holds x^0..x^7, MSB first).

#include <hip/hip_runtime.h>
#include <type_traits>
#include <vector>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#include "picotls/mi355x.h"

// Device code, in dependency order (one translation unit: the kernels are templates instantiated by the host side)
#include "engine/common.h"
#include "engine/keyset_setup.h"
#include "engine/lds_tables.h"
#include "engine/aes_tt.h"
#include "engine/ghash.h"
#include "engine/record.h"
#include "engine/segment.h"
#include "engine/gcm_kernels.h"
#include "engine/aux_kernels.h"

// ------------------------------------------------------------------------------------------------ host side

static thread_local char g_err[256];

static int fail(const char *fmt, const char *detail)
{
    snprintf(g_err, sizeof(g_err), fmt, detail);
    return -1;
}

#define HIP_TRY(expr)                                                                                                         \
    do {                                                                                                                      \
        hipError_t e_ = (expr);                                                                                               \
        if (e_ != hipSuccess)                                                                                                 \
            return fail(#expr ": %s", hipGetErrorString(e_));                                                                 \
    } while (0)

struct st_ptls_mi355x_keyset_t {
    int device;
    size_t nkeys, key_size;
    int nr;
    KeyEntry *d_keys;
    int ncu;
    int schedule;
    // staging for the synchronous host-buffer helpers (the per-record picotls path): one pinned host buffer and one
    // device buffer, grown on demand, and a stream of their own, so a call is one H2D copy, one launch, one D2H copy
    uint8_t *d_stage, *h_stage;
    uint8_t *h_stage_dev;  // device address of h_stage (NULL: not mapped, every round trip copies)
    size_t stage_cap;
    hipStream_t stream;
    // key grouping of ungrouped many-key batches (key_group_*): scratch for key counts and the record permutation,
    // grown on demand; group_ev orders its users when batches on several streams share the keyset
    u32 *d_group;
    size_t group_cap;
    hipEvent_t group_ev;
};

static int stage_reserve(ptls_mi355x_keyset_t *ks, size_t bytes)
{
    if (bytes <= ks->stage_cap)
        return 0;
    size_t cap = ks->stage_cap * 2 > bytes ? ks->stage_cap * 2 : bytes;
    cap = cap < 4096 ? 4096 : (cap + 4095) & ~(size_t)4095;
    if (ks->stream == NULL)
        HIP_TRY(hipStreamCreateWithFlags(&ks->stream, hipStreamNonBlocking));
    if (ks->d_stage != NULL) {
        HIP_TRY(hipStreamSynchronize(ks->stream));
        (void)hipFree(ks->d_stage);
        (void)hipHostFree(ks->h_stage);
        ks->d_stage = ks->h_stage = ks->h_stage_dev = NULL;
        ks->stage_cap = 0;
    }
    HIP_TRY(hipMalloc((void **)&ks->d_stage, cap));
    if (hipHostMalloc((void **)&ks->h_stage, cap, hipHostMallocDefault) != hipSuccess) {
        (void)hipFree(ks->d_stage);
        ks->d_stage = NULL;
        return fail("%s", "stage: pinned host allocation failed");
    }
    if (hipHostGetDevicePointer((void **)&ks->h_stage_dev, ks->h_stage, 0) != hipSuccess)
        ks->h_stage_dev = NULL;
    ks->stage_cap = cap;
    return 0;
}

// Round trips run on the pinned host buffer itself when it is mapped into the device's address space: the kernel reads
// its input and writes its output over PCIe, and the call saves the two copy launches. Measured against copying
// (tools/latency.py, interleaved): 16 B 29 -> 26 us, 1200 B 31 -> 29, 16 KiB 52 -> 38, 4 MiB 1.70 -> 1.58 ms.
static uint8_t *stage_dev(const ptls_mi355x_keyset_t *ks)
{
    return ks->h_stage_dev != NULL ? ks->h_stage_dev : ks->d_stage;
}

// the synchronous round trip of the host-buffer helpers, on the buffer stage_dev returned (d): unless that is the
// pinned buffer itself, H2D of the first `up` staged bytes before the launch (run by the caller's lambda) and D2H of
// [down_off, down_off + down) after it; then wait
template <typename Launch>
static int stage_roundtrip(ptls_mi355x_keyset_t *ks, const uint8_t *d, size_t up, size_t down_off, size_t down, Launch launch)
{
    const bool copy = d == ks->d_stage;
    if (copy)
        HIP_TRY(hipMemcpyAsync(ks->d_stage, ks->h_stage, up, hipMemcpyHostToDevice, ks->stream));
    if (launch() != 0)
        return -1;
    if (copy)
        HIP_TRY(hipMemcpyAsync(ks->h_stage + down_off, ks->d_stage + down_off, down, hipMemcpyDeviceToHost, ks->stream));
    HIP_TRY(hipStreamSynchronize(ks->stream));
    return 0;
}

static int engine_init_attrs(void)
{
    static int done = 0;
    if (done)
        return 0;
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<10, false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<10, true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<14, false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<14, true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
#define CHUNKED_ATTR(nr, open, frame)                                                                                  \
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_chunked_kernel<nr, open, frame>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                CLDS_ALLOC))
    CHUNKED_ATTR(10, false, 0);
    CHUNKED_ATTR(10, true, 0);
    CHUNKED_ATTR(14, false, 0);
    CHUNKED_ATTR(14, true, 0);
    CHUNKED_ATTR(10, false, 1);
    CHUNKED_ATTR(10, true, 1);
    CHUNKED_ATTR(14, false, 1);
    CHUNKED_ATTR(14, true, 1);
    CHUNKED_ATTR(10, false, 2);
    CHUNKED_ATTR(10, true, 2);
    CHUNKED_ATTR(14, false, 2);
    CHUNKED_ATTR(14, true, 2);
#undef CHUNKED_ATTR
    HIP_TRY(hipFuncSetAttribute((const void *)ecb_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)ecb_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)hp_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)hp_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)quiclb_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    done = 1;
    return 0;
}

extern "C" {

const char *ptls_mi355x_last_error(void) { return g_err; }

int ptls_mi355x_is_supported(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return 0;
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return 0;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

ptls_mi355x_keyset_t *ptls_mi355x_keyset_new(const void *keys, const void *ivs, size_t nkeys, size_t key_size)
{
    if (keys == NULL || ivs == NULL || nkeys == 0 || (key_size != 16 && key_size != 32) || nkeys > (1u << 30)) {
        fail("%s", "ptls_mi355x_keyset_new: invalid arguments");
        return NULL;
    }
    if (engine_init_attrs() != 0)
        return NULL;
    ptls_mi355x_keyset_t *ks = (ptls_mi355x_keyset_t *)calloc(1, sizeof(*ks));
    uint8_t *d_raw = NULL;
    if (ks == NULL)
        return NULL;
    ks->nkeys = nkeys, ks->key_size = key_size, ks->nr = key_size == 16 ? 10 : 14;
    if (hipGetDevice(&ks->device) != hipSuccess || hipDeviceGetAttribute(&ks->ncu, hipDeviceAttributeMultiprocessorCount, ks->device) != hipSuccess)
        goto Fail;
    if (hipMalloc((void **)&ks->d_keys, nkeys * sizeof(KeyEntry)) != hipSuccess)
        goto Fail;
    if (hipMalloc((void **)&d_raw, nkeys * (key_size + 12)) != hipSuccess)
        goto Fail;
    if (hipMemcpy(d_raw, keys, nkeys * key_size, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_raw + nkeys * key_size, ivs, nkeys * 12, hipMemcpyHostToDevice) != hipSuccess)
        goto Fail;
    keyset_setup_kernel<<<(unsigned)((nkeys + 127) / 128), 128>>>(d_raw, d_raw + nkeys * key_size, ks->d_keys, (u32)nkeys, (u32)key_size);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        goto Fail;
    (void)hipMemset(d_raw, 0, nkeys * (key_size + 12));
    (void)hipFree(d_raw);
    return ks;
Fail:
    fail("%s", "ptls_mi355x_keyset_new: device setup failed");
    if (d_raw != NULL)
        (void)hipFree(d_raw);
    if (ks->d_keys != NULL)
        (void)hipFree(ks->d_keys);
    free(ks);
    return NULL;
}

int ptls_mi355x_keyset_update(ptls_mi355x_keyset_t *ks, const uint32_t *key_idx, const void *keys, const void *ivs, size_t n)
{
    if (ks == NULL || (n != 0 && (key_idx == NULL || keys == NULL || ivs == NULL)))
        return fail("%s", "keyset_update: invalid arguments");
    std::vector<bool> seen(n != 0 ? ks->nkeys : 0);
    for (size_t i = 0; i < n; ++i) {
        if (key_idx[i] >= ks->nkeys)
            return fail("%s", "keyset_update: key index out of range");
        if (seen[key_idx[i]])
            return fail("%s", "keyset_update: key index listed twice");
        seen[key_idx[i]] = true;
    }
    if (n == 0)
        return 0;
    uint8_t *d = NULL;
    const size_t kb = n * ks->key_size, ib = n * 12, sb = n * 4;
    HIP_TRY(hipMalloc((void **)&d, kb + ib + sb));
    int ret = -1;
    if (hipDeviceSynchronize() == hipSuccess &&  // no launch in flight still reads the old entries
        hipMemcpy(d, keys, kb, hipMemcpyHostToDevice) == hipSuccess && hipMemcpy(d + kb, ivs, ib, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(d + kb + ib, key_idx, sb, hipMemcpyHostToDevice) == hipSuccess) {
        keyset_setup_kernel<<<(unsigned)((n + 127) / 128), 128>>>(d, d + kb, ks->d_keys, (u32)n, (u32)ks->key_size,
                                                                 (const u32 *)(d + kb + ib));
        if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess)
            ret = 0;
    }
    (void)hipMemset(d, 0, kb + ib);
    (void)hipDeviceSynchronize();
    (void)hipFree(d);
    if (ret != 0)
        fail("%s", "keyset_update: device setup failed");
    return ret;
}

void ptls_mi355x_keyset_free(ptls_mi355x_keyset_t *ks)
{
    if (ks == NULL)
        return;
    (void)hipMemset(ks->d_keys, 0, ks->nkeys * sizeof(KeyEntry));
    (void)hipDeviceSynchronize();
    (void)hipFree(ks->d_keys);
    if (ks->d_stage != NULL) {
        (void)hipMemset(ks->d_stage, 0, ks->stage_cap);
        memset(ks->h_stage, 0, ks->stage_cap);  // staged plaintext and keystream-derived bytes
        (void)hipDeviceSynchronize();
        (void)hipFree(ks->d_stage);
        (void)hipHostFree(ks->h_stage);
    }
    if (ks->stream != NULL)
        (void)hipStreamDestroy(ks->stream);
    if (ks->group_ev != NULL) {
        (void)hipEventSynchronize(ks->group_ev);
        (void)hipEventDestroy(ks->group_ev);
    }
    (void)hipFree(ks->d_group);
    free(ks);
}

#if ENGINE_PROFILE
int ptls_mi355x_debug_profile(unsigned long long *out, int reset)
{
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(g_prof)));
    if (reset) {
        static const unsigned long long z[16] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)));
    }
    return 0;
}
#endif

int ptls_mi355x_keyset_set_schedule(ptls_mi355x_keyset_t *ks, int schedule)
{
    if (ks == NULL || schedule < PTLS_MI355X_SCHEDULE_AUTO || schedule > PTLS_MI355X_SCHEDULE_CHUNKED)
        return fail("%s", "set_schedule: invalid arguments");
    ks->schedule = schedule;
    return 0;
}

size_t ptls_mi355x_keyset_size(const ptls_mi355x_keyset_t *ks) { return ks->nkeys; }
size_t ptls_mi355x_keyset_key_size(const ptls_mi355x_keyset_t *ks) { return ks->key_size; }

int ptls_mi355x_keyset_get_iv(ptls_mi355x_keyset_t *ks, size_t key_idx, void *iv)
{
    if (ks == NULL || key_idx >= ks->nkeys)
        return fail("%s", "get_iv: bad key index");
    u32 w[3];
    HIP_TRY(hipMemcpy(w, ks->d_keys[key_idx].iv, 12, hipMemcpyDeviceToHost));
    memcpy(iv, w, 12);
    return 0;
}

int ptls_mi355x_keyset_set_iv(ptls_mi355x_keyset_t *ks, size_t key_idx, const void *iv)
{
    if (ks == NULL || key_idx >= ks->nkeys)
        return fail("%s", "set_iv: bad key index");
    u32 w[3];
    memcpy(w, iv, 12);
    HIP_TRY(hipMemcpy(ks->d_keys[key_idx].iv, w, 12, hipMemcpyHostToDevice));
    return 0;
}

// Schedule choice (ptls_mi355x_keyset_set_schedule): AUTO = chunked. Its uniform runs take the whole-record path,
// which measured at or above the lockstep kernel on one-key uniform batches (929 vs 841 GiB/s on 16 KiB records,
// 784 vs 751 on 1200 B), and its chunked runs balance mixed lengths and short key runs.
static bool use_chunked(const ptls_mi355x_keyset_t *ks) { return ks->schedule != PTLS_MI355X_SCHEDULE_LOCKSTEP; }

static int launch_batch(ptls_mi355x_keyset_t *ks, bool open, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                        const void *aad, void *out, uint8_t *ok, void *stream, int frame = 0, u32 unit_log2 = CHUNK_LOG2)
{
    if (ks == NULL || (nrecs != 0 && (recs == NULL || in == NULL || out == NULL || (open && ok == NULL))))
        return fail("%s", "batch: invalid arguments");
    if (nrecs == 0)
        return 0;
    BatchArgs a = {ks->d_keys, recs, (u64)nrecs, (const uint8_t *)in, (const uint8_t *)aad, (uint8_t *)out, ok,
                   ks->nkeys > 1 ? 1u : 0u, (u32)ks->nkeys, unit_log2, nullptr, nullptr, nullptr};
    if (a.aad == NULL)
        a.aad = a.in;
    const u64 groups = (nrecs + (64 / ENGINE_G) - 1) / (64 / ENGINE_G);
    // one persistent workgroup per CU; small batches use fewer workgroups so each still gets >= 4 record groups
    u64 grid = (u64)ks->ncu;
    if (grid > (groups + 3) / 4)
        grid = (groups + 3) / 4;
    if (grid < 1)
        grid = 1;
    hipStream_t s = (hipStream_t)stream;
    // ungrouped many-key batches: group the records by key on the device first (see key_hist_kernel)
#ifndef KEY_GROUP_DISABLE
    const bool group = use_chunked(ks) && ks->nkeys > 1 && ks->nkeys <= KEY_GROUP_MAX_KEYS && nrecs > 1 &&
                       nrecs <= 0xffffffffu;
#else
    const bool group = false;
#endif
    if (group) {
        // scratch: ctl[2] | counts[nkeys + 1] | perm[n] | (8-byte aligned) grouped descriptors[n]
        const size_t nb = ks->nkeys + 1, words = ((2 + nb + nrecs + 1) & ~(size_t)1) + nrecs * (sizeof(ptls_mi355x_record_t) / 4);
        if (ks->group_ev == NULL)
            HIP_TRY(hipEventCreateWithFlags(&ks->group_ev, hipEventDisableTiming));
        if (words > ks->group_cap) {
            HIP_TRY(hipEventSynchronize(ks->group_ev));
            (void)hipFree(ks->d_group);
            ks->d_group = NULL;
            ks->group_cap = 0;
            HIP_TRY(hipMalloc((void **)&ks->d_group, words * 4));
            ks->group_cap = words;
        }
        HIP_TRY(hipStreamWaitEvent(s, ks->group_ev, 0));  // a batch on another stream may still use the scratch
        u32 *ctl = ks->d_group, *cnt = ctl + 2, *perm = cnt + nb;
        HIP_TRY(hipMemsetAsync(ctl, 0, (2 + nb) * 4, s));
        const unsigned gh = (unsigned)min((nrecs + 255) / 256, (size_t)ks->ncu * 8);
        key_changes_kernel<<<gh, 256, 0, s>>>(recs, nrecs, ctl);
        key_hist_kernel<<<gh, 256, 0, s>>>(recs, nrecs, (u32)ks->nkeys, cnt, ctl);
        key_scan_kernel<<<1, 1024, 0, s>>>(cnt, (u32)nb, nrecs, ctl);
        ptls_mi355x_record_t *grouped = (ptls_mi355x_record_t *)(ctl + ((2 + nb + nrecs + 1) & ~(size_t)1));
        key_scatter_kernel<<<gh, 256, 0, s>>>(recs, nrecs, (u32)ks->nkeys, cnt, perm, grouped, ctl);
        a.grouped = grouped;
        a.perm = perm;
        a.perm_on = ctl + 1;
    }
#define CHUNKED_LAUNCH(nr, op, frame) gcm_chunked_kernel<nr, op, frame><<<(unsigned)grid, ENGINE_WG, CLDS_ALLOC, s>>>(a)
    if (frame == 1) {
        if (ks->nr == 10) {
            if (open)
                CHUNKED_LAUNCH(10, true, 1);
            else
                CHUNKED_LAUNCH(10, false, 1);
        } else {
            if (open)
                CHUNKED_LAUNCH(14, true, 1);
            else
                CHUNKED_LAUNCH(14, false, 1);
        }
    } else if (frame == 2) {
        if (ks->nr == 10) {
            if (open)
                CHUNKED_LAUNCH(10, true, 2);
            else
                CHUNKED_LAUNCH(10, false, 2);
        } else {
            if (open)
                CHUNKED_LAUNCH(14, true, 2);
            else
                CHUNKED_LAUNCH(14, false, 2);
        }
    } else if (use_chunked(ks)) {
        if (ks->nr == 10) {
            if (open)
                CHUNKED_LAUNCH(10, true, 0);
            else
                CHUNKED_LAUNCH(10, false, 0);
        } else {
            if (open)
                CHUNKED_LAUNCH(14, true, 0);
            else
                CHUNKED_LAUNCH(14, false, 0);
        }
    } else if (ks->nr == 10) {
        if (open)
            gcm_batch_kernel<10, true><<<(unsigned)grid, ENGINE_WG, LDS_ALLOC, s>>>(a);
        else
            gcm_batch_kernel<10, false><<<(unsigned)grid, ENGINE_WG, LDS_ALLOC, s>>>(a);
    } else {
        if (open)
            gcm_batch_kernel<14, true><<<(unsigned)grid, ENGINE_WG, LDS_ALLOC, s>>>(a);
        else
            gcm_batch_kernel<14, false><<<(unsigned)grid, ENGINE_WG, LDS_ALLOC, s>>>(a);
    }
    HIP_TRY(hipGetLastError());
    if (group)
        HIP_TRY(hipEventRecord(ks->group_ev, s));
    return 0;
}

int ptls_mi355x_seal_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                           const void *aad, void *out, void *stream)
{
    return launch_batch(ks, false, recs, nrecs, in, aad, out, NULL, stream);
}

int ptls_mi355x_open_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                           const void *aad, void *out, uint8_t *ok, void *stream)
{
    return launch_batch(ks, true, recs, nrecs, in, aad, out, ok, stream);
}

int ptls_mi355x_ecb_batch(ptls_mi355x_keyset_t *ks, const uint32_t *key_idx, const void *in, void *out, size_t nblocks,
                          void *stream)
{
    if (ks == NULL || (nblocks != 0 && (in == NULL || out == NULL)))
        return fail("%s", "ecb: invalid arguments");
    if (nblocks == 0)
        return 0;
    u64 grid = (nblocks + 255) / 256;
    if (grid > (u64)ks->ncu * 4)
        grid = (u64)ks->ncu * 4;
    hipStream_t s = (hipStream_t)stream;
    if (ks->nr == 10)
        ecb_kernel<10><<<(unsigned)grid, 256, LDS_AES_BYTES, s>>>(ks->d_keys, (u32)ks->nkeys, key_idx, (const uint8_t *)in,
                                                                  (uint8_t *)out, nblocks);
    else
        ecb_kernel<14><<<(unsigned)grid, 256, LDS_AES_BYTES, s>>>(ks->d_keys, (u32)ks->nkeys, key_idx, (const uint8_t *)in,
                                                                  (uint8_t *)out, nblocks);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_seal_tls_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                 void *out, void *stream)
{
    return launch_batch(ks, false, recs, nrecs, in, NULL, out, NULL, stream, 1);
}

int ptls_mi355x_open_tls_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                 void *out, uint8_t *ok, ptls_mi355x_tls_result_t *results, void *stream)
{
    if (launch_batch(ks, true, recs, nrecs, in, NULL, out, ok, stream, 1) != 0)
        return -1;
    if (nrecs == 0)
        return 0;
    u64 grid = (nrecs + 255) / 256;
    if (grid > (u64)ks->ncu * 4)
        grid = (u64)ks->ncu * 4;
    tls_unpad_kernel<<<(unsigned)grid, 256, 0, (hipStream_t)stream>>>(recs, nrecs, (const uint8_t *)in, (const uint8_t *)out,
                                                                       ok, results);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_seal_tls12_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                   void *out, void *stream)
{
    return launch_batch(ks, false, recs, nrecs, in, NULL, out, NULL, stream, 2);
}

int ptls_mi355x_open_tls12_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                   void *out, uint8_t *ok, ptls_mi355x_tls_result_t *results, void *stream)
{
    if (launch_batch(ks, true, recs, nrecs, in, NULL, out, ok, stream, 2) != 0)
        return -1;
    if (nrecs == 0)
        return 0;
    u64 grid = (nrecs + 255) / 256;
    if (grid > (u64)ks->ncu * 4)
        grid = (u64)ks->ncu * 4;
    tls12_check_kernel<<<(unsigned)grid, 256, 0, (hipStream_t)stream>>>(recs, nrecs, (const uint8_t *)in, ok, results);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_hp_mask_batch(ptls_mi355x_keyset_t *hp_ks, const ptls_mi355x_hp_t *hp, size_t n, const void *base,
                              void *masks, void *stream)
{
    if (hp_ks == NULL || (n != 0 && (hp == NULL || base == NULL || masks == NULL)))
        return fail("%s", "hp_mask: invalid arguments");
    if (n == 0)
        return 0;
    u64 grid = (n + 255) / 256;
    if (grid > (u64)hp_ks->ncu * 4)
        grid = (u64)hp_ks->ncu * 4;
    hipStream_t s = (hipStream_t)stream;
    if (hp_ks->nr == 10)
        hp_kernel<10><<<(unsigned)grid, 256, LDS_AES_BYTES, s>>>(hp_ks->d_keys, (u32)hp_ks->nkeys, hp, (const uint8_t *)base,
                                                                 (uint8_t *)masks, n);
    else
        hp_kernel<14><<<(unsigned)grid, 256, LDS_AES_BYTES, s>>>(hp_ks->d_keys, (u32)hp_ks->nkeys, hp, (const uint8_t *)base,
                                                                 (uint8_t *)masks, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_seal_batch_hp(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                              const void *aad, void *out, ptls_mi355x_keyset_t *hp_ks, const ptls_mi355x_hp_t *hp,
                              void *masks, void *stream)
{
    if (hp_ks == NULL || (nrecs != 0 && (hp == NULL || masks == NULL)))
        return fail("%s", "seal_batch_hp: invalid arguments");
    if (launch_batch(ks, false, recs, nrecs, in, aad, out, NULL, stream) != 0)
        return -1;
    return ptls_mi355x_hp_mask_batch(hp_ks, hp, nrecs, out, masks, stream);
}

int ptls_mi355x_quiclb_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_cid_t *cids, size_t n, const void *in, void *out,
                             void *stream)
{
    if (ks == NULL || (n != 0 && (cids == NULL || in == NULL || out == NULL)))
        return fail("%s", "quiclb: invalid arguments");
    if (ks->key_size != 16)
        return fail("%s", "quiclb: the QUIC-LB cipher is keyed with AES-128 (PTLS_QUICLB_KEY_SIZE)");
    if (n == 0)
        return 0;
    u64 grid = (n + 255) / 256;
    if (grid > (u64)ks->ncu * 4)
        grid = (u64)ks->ncu * 4;
    quiclb_kernel<10><<<(unsigned)grid, 256, LDS_AES_BYTES, (hipStream_t)stream>>>(ks->d_keys, (u32)ks->nkeys, cids,
                                                                                    (const uint8_t *)in, (uint8_t *)out, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_quiclb_transform(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t len, int encrypt)
{
    if (ks == NULL || key_idx >= ks->nkeys || output == NULL || input == NULL || len < PTLS_MI355X_QUICLB_MIN_LEN ||
        len > PTLS_MI355X_QUICLB_MAX_LEN)
        return fail("%s", "quiclb_transform: invalid arguments");
    if (stage_reserve(ks, 96) != 0)
        return -1;
    // staging: [0, 32) CID in, [32, 56) descriptor | [64, 96) CID out
    const ptls_mi355x_cid_t c = {0, 64, (uint32_t)key_idx, (uint8_t)len, (uint8_t)(encrypt != 0), 0};
    memcpy(ks->h_stage, input, len);
    memcpy(ks->h_stage + 32, &c, sizeof(c));
    uint8_t *d = stage_dev(ks);
    if (stage_roundtrip(ks, d, 64, 64, 32, [&] {
            return ptls_mi355x_quiclb_batch(ks, (const ptls_mi355x_cid_t *)(d + 32), 1, d, d, ks->stream);
        }) != 0)
        return -1;
    memcpy(output, ks->h_stage + 64, len);
    return 0;
}

int ptls_mi355x_encrypt_block(ptls_mi355x_keyset_t *ks, size_t key_idx, void *out, const void *in)
{
    if (ks == NULL || key_idx >= ks->nkeys || out == NULL || in == NULL)
        return fail("%s", "encrypt_block: invalid arguments");
    if (stage_reserve(ks, 64) != 0)
        return -1;
    // staging: [0, 16) block in, [16, 20) key index | [32, 48) block out
    const u32 idx = (u32)key_idx;
    memcpy(ks->h_stage, in, 16);
    memcpy(ks->h_stage + 16, &idx, 4);
    uint8_t *d = stage_dev(ks);
    if (stage_roundtrip(ks, d, 32, 32, 16, [&] {
            return ptls_mi355x_ecb_batch(ks, (const uint32_t *)(d + 16), d, d + 32, 1, ks->stream);
        }) != 0)
        return -1;
    memcpy(out, ks->h_stage + 32, 16);
    return 0;
}

// single record on host buffers: a batch of one through the keyset's staging buffers
static int single(ptls_mi355x_keyset_t *ks, size_t key_idx, bool open, void *output, const void *input, size_t len, uint64_t seq,
                  const void *aad, size_t aadlen, int *verified)
{
    if (ks == NULL || key_idx >= ks->nkeys || aadlen > 0xffff || len > PTLS_MI355X_MAX_RECORD_LEN)
        return fail("%s", "single: invalid arguments");
    const size_t inbytes = len + (open ? 16 : 0), outbytes = len + (open ? 0 : 16);
    // staging: [in | aad | descriptor] goes up, [out | ok] comes back
    const size_t off_in = 0, off_aad = (inbytes + 15) & ~(size_t)15, off_rec = off_aad + ((aadlen + 15) & ~(size_t)15),
                 off_out = off_rec + 64, off_ok = off_out + ((outbytes + 15) & ~(size_t)15), total = off_ok + 16;
    if (stage_reserve(ks, total) != 0)
        return -1;
    const ptls_mi355x_record_t r = {0, 0, seq, 0, (u32)len, 0, (uint16_t)aadlen, 0};  // offsets relative to the arenas below
    ptls_mi355x_keyset_t view = *ks;
    view.d_keys = ks->d_keys + key_idx;
    view.nkeys = 1;
    uint8_t *h = ks->h_stage, *d = stage_dev(ks);
    if (inbytes != 0)
        memcpy(h + off_in, input, inbytes);
    if (aadlen != 0)
        memcpy(h + off_aad, aad, aadlen);
    memcpy(h + off_rec, &r, sizeof(r));
    // one record on one workgroup: shorter units put more of its waves to work (a unit step costs a lone wave ~2 us of
    // latency, a unit combine ~0.15 us); steps / 2^k units balance the two
    const size_t steps = ((aadlen + 15) / 16 + (len + 15) / 16 + 1 + ENGINE_G - 1) / ENGINE_G;
    const u32 unit_log2 = steps <= 24 ? 0 : steps <= 96 ? 1 : steps <= 400 ? 2 : steps <= 1600 ? 3 : CHUNK_LOG2;
    if (stage_roundtrip(ks, d, off_out, off_out, total - off_out, [&] {
            return launch_batch(&view, open, (const ptls_mi355x_record_t *)(d + off_rec), 1, d + off_in, d + off_aad,
                                d + off_out, d + off_ok, ks->stream, 0, unit_log2 < CHUNK_LOG2 ? unit_log2 : CHUNK_LOG2);
        }) != 0)
        return -1;
    if (outbytes != 0)
        memcpy(output, h + off_out, outbytes);
    if (open)
        *verified = h[off_ok];
    return 0;
}

int ptls_mi355x_encrypt(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                        const void *aad, size_t aadlen)
{
    return single(ks, key_idx, false, output, input, inlen, seq, aad, aadlen, NULL);
}

size_t ptls_mi355x_decrypt(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                           const void *aad, size_t aadlen)
{
    if (inlen < 16)
        return SIZE_MAX;
    int verified = 0;
    if (single(ks, key_idx, true, output, input, inlen - 16, seq, aad, aadlen, &verified) != 0)
        return SIZE_MAX;
    return verified ? inlen - 16 : SIZE_MAX;
}

}  // extern "C"
