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
#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <new>
#include <type_traits>
#include <vector>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <sched.h>

#include "picotls/mi355x.h"
#include "picotls/mi355x_debug.h"

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
#include "engine/span_kernels.h"

// ------------------------------------------------------------------------------------------------ host side

static thread_local char g_err[256];

static int fail(const char *fmt, const char *detail)
{
    snprintf(g_err, sizeof(g_err), fmt, detail);
    return -1;
}

// Kernel launches are checked with hipGetLastError, which also returns the error of any earlier call of this thread
// whose failure was handled (a failed hipHostGetDevicePointer, for one: tools/mb/lasterr.hip showed that error reported
// after a good launch). LAUNCH_CLEAR() before a launch makes the check after it about that launch only.
// (-DLAUNCH_CLEAR_NOOP=1: a tools/ variant without it, which the regression test of tests/c/test_vtable.c `lasterr`
// must fail on; never the shipped build)
#if LAUNCH_CLEAR_NOOP
#define LAUNCH_CLEAR() ((void)0)
#else
#define LAUNCH_CLEAR() ((void)hipGetLastError())
#endif

// Test and measurement counters (include/picotls/mi355x_debug.h): chunked-kernel launches per EXT instantiation (0..4),
// lockstep launches (5), span launches (6) -- host side, counted where the launch is made
static std::atomic<uint64_t> g_launches[8];
#define COUNT_LAUNCH(i) (ENGINE_HOOKS ? g_launches[(i)].fetch_add(1, std::memory_order_relaxed) : 0)

#define HIP_TRY(expr)                                                                                                         \
    do {                                                                                                                      \
        hipError_t e_ = (expr);                                                                                               \
        if (e_ != hipSuccess)                                                                                                 \
            return fail(#expr ": %s", hipGetErrorString(e_));                                                                 \
    } while (0)

static void clear_memory(void *p, size_t n)  // ptls_clear_memory: a memset the compiler may not drop
{
    volatile uint8_t *v = (volatile uint8_t *)p;
    while (n-- != 0)
        *v++ = 0;
}

// ---- per-device state
//
// picotls contexts are independent (lib/picotls.c:6553-6568: a context is malloc'd, set up and freed by its owner,
// fusion's setup touches nothing shared; SURVEY 8(b) Threading), and a QUIC or TLS server creates and frees them per
// connection and epoch. So nothing here waits for the whole device (no hipDeviceSynchronize, no hipFree, whose implicit
// device-wide synchronisation would stall every batch in flight):
//   * one-key keysets (a picotls context) take a 512-byte entry from a per-device slab and are set up by one launch whose
//     key travels in the kernel arguments, on the device's setup stream, with an event their first use waits for;
//   * teardown, rekey and IV changes run on the device's maintenance stream, ordered after the keyset's own launches
//     (an event per stream it was used on), and a freed slab entry returns to the pool only once it has been cleared;
//   * the synchronous host-buffer helpers (the per-record picotls path) take a staging buffer and its stream from a
//     per-device pool for the duration of one call, so concurrent contexts on different threads never share one.

#define MAX_DEVICES 64
#define STAGE_CLASSES 26   // pinned staging buffers of 4 KiB << class
#define SLAB_ENTRIES 1024  // one-key keyset entries per slab (512 KiB)
// Bounds of the staging pool (fusion's context owns one allocation and frees it, lib/fusion.c:1043-1049; here the pinned
// buffers outlive calls so that the next call of a thread skips hipHostMalloc, but not without limit):
#define STAGE_POOL_BYTES ((size_t)64 << 20)  // idle pinned bytes kept per device (PTLS_MI355X_STAGE_POOL_BYTES)
#define STAGE_KEEP_MAX ((size_t)16 << 20)     // a buffer above this (a call of a record > ~8 MiB) is freed after its call
#define STAGE_STREAMS 16                      // stager streams per device, shared round-robin beyond that

struct Stager {
    hipStream_t stream;  // one of the device's stager streams (DeviceState::stage_streams), not owned
    uint8_t *h;      // pinned host buffer
    uint8_t *h_dev;  // its device address (NULL: not mapped, or PTLS_MI355X_STAGE_COPY=1: round trips copy through d)
    uint8_t *d;      // device buffer of the copy path
    size_t cap;
    int cls;
    Stager *next;
};

struct PendingSlot {
    KeyEntry *e;
    KeyEntry *slab;
    hipEvent_t cleared;
};

struct OneCall;
struct Combiner {  // per-record calls of one kind waiting for a launch (submit)
    std::mutex mu;
    std::vector<OneCall *> q;
    int inflight = 0;
    size_t expect = 1;  // calls in the last batch: a caller that could lead waits briefly until as many have queued
};

struct DeviceState {
    int device = 0, ncu = 0;
    hipStream_t setup = nullptr;  // one-key and many-key setup launches (never waits on anything)
    hipStream_t maint = nullptr;  // teardown, rekey, set_iv: ordered after the keyset's launches
    int priority = 0;             // the device's greatest stream priority: the engine's own streams (setup, teardown,
                                  // per-record round trips) are dispatched ahead of bulk batches on ordinary streams
    bool force_copy = false;      // PTLS_MI355X_STAGE_COPY=1: the staging round trip copies instead of mapping
    bool stage_coherent = true;   // staging buffers fine-grained (hipHostMallocCoherent); PTLS_MI355X_STAGE_COHERENT=0: the
                                  // HIP default (coarse-grained), kept only to reproduce the round-3 race
    size_t stage_limit = 0;       // PTLS_MI355X_MAX_STAGE_BYTES: the largest staging buffer one call may use
    bool ct_default = true;       // new keysets are constant-time (PTLS_MI355X_CONSTANT_TIME=0: not, for an A/B)
    bool fault_order = false;     // PTLS_MI355X_FAULT_ORDER=1 (tests only): keyset teardown cannot order itself on the device
    bool diag = false;            // PTLS_MI355X_DIAG=1 (diagnosis only): per-record calls re-read their results after a stream
                                  // synchronisation and report bytes that changed after the completion words were seen
    std::mutex mu;                // the pools below
    Stager *stagers[STAGE_CLASSES] = {};
    size_t stage_idle = 0;        // pinned bytes of the idle stagers above
    size_t stage_busy = 0;        // ... and of the stagers in use by calls
    size_t stage_pool_cap = STAGE_POOL_BYTES;
    std::vector<hipStream_t> stage_streams;  // at most STAGE_STREAMS
    unsigned stage_rr = 0;
    std::vector<std::pair<KeyEntry *, KeyEntry *>> slots;  // free one-key entries and the slab each lies in
    std::vector<PendingSlot> pending;
    std::vector<hipEvent_t> events;
    int combine = 0;              // PTLS_MI355X_COMBINE: combined per-record launches in flight per kind (0: none)
    Combiner comb[32];
};

static std::atomic<DeviceState *> g_devs[MAX_DEVICES];
static std::mutex g_devs_mu;

static int set_kernel_attrs(void)
{
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<10, false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<10, true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<14, false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_batch_kernel<14, true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC));
#if SEG_COOP  // (one instantiation for both settings, launch_chunked_x)
#define CHUNKED_ATTR_X(nr, open, frame, ext)                                                                           \
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_chunked_kernel<nr, open, frame, true, ext>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                CLDS_ALLOC))
#else
#define CHUNKED_ATTR_X(nr, open, frame, ext)                                                                           \
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_chunked_kernel<nr, open, frame, false, ext>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                CLDS_ALLOC));                                                                              \
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_chunked_kernel<nr, open, frame, true, ext>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                CLDS_ALLOC))
#endif
#define CHUNKED_ATTR(nr, open, frame) CHUNKED_ATTR_X(nr, open, frame, 0)
    CHUNKED_ATTR_X(10, false, 0, 1);
    CHUNKED_ATTR_X(10, true, 0, 1);
    CHUNKED_ATTR_X(14, false, 0, 1);
    CHUNKED_ATTR_X(14, true, 0, 1);
    CHUNKED_ATTR_X(10, false, 0, 2);
    CHUNKED_ATTR_X(14, false, 0, 2);
#if MK_RUNS  // (round 6) the serial W8 kernel of many-key batches, with multi-key runs (EXT 5)
#define CHUNKED_ATTR_MK(frame)                                                                                         \
    CHUNKED_ATTR_X(10, false, frame, 5);                                                                               \
    CHUNKED_ATTR_X(10, true, frame, 5);                                                                                \
    CHUNKED_ATTR_X(14, false, frame, 5);                                                                               \
    CHUNKED_ATTR_X(14, true, frame, 5)
#else
#define CHUNKED_ATTR_MK(frame) (void)0
#endif
#define CHUNKED_ATTR_W8(frame)                                                                                         \
    CHUNKED_ATTR_X(10, false, frame, 3);                                                                               \
    CHUNKED_ATTR_X(10, true, frame, 3);                                                                                \
    CHUNKED_ATTR_X(14, false, frame, 3);                                                                               \
    CHUNKED_ATTR_X(14, true, frame, 3);                                                                                \
    CHUNKED_ATTR_X(10, false, frame, 4);                                                                               \
    CHUNKED_ATTR_X(10, true, frame, 4);                                                                                \
    CHUNKED_ATTR_X(14, false, frame, 4);                                                                               \
    CHUNKED_ATTR_X(14, true, frame, 4);                                                                                \
    CHUNKED_ATTR_MK(frame)
#if W8_HORNER
    CHUNKED_ATTR_W8(0);
    CHUNKED_ATTR_W8(1);
#if W8_TLS12
    CHUNKED_ATTR_W8(2);
#endif
#endif
#undef CHUNKED_ATTR_W8
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
#undef CHUNKED_ATTR_X
    HIP_TRY(hipFuncSetAttribute((const void *)ecb_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)ecb_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)hp_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)hp_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
    HIP_TRY(hipFuncSetAttribute((const void *)quiclb_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_AES_BYTES));
#if SEG_COOP
#define SPAN_ATTR(nr, open)                                                                                            \
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_span_kernel<nr, open, true>, hipFuncAttributeMaxDynamicSharedMemorySize, SPAN_LDS))
#else
#define SPAN_ATTR(nr, open)                                                                                            \
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_span_kernel<nr, open, false>, hipFuncAttributeMaxDynamicSharedMemorySize, SPAN_LDS)); \
    HIP_TRY(hipFuncSetAttribute((const void *)gcm_span_kernel<nr, open, true>, hipFuncAttributeMaxDynamicSharedMemorySize, SPAN_LDS))
#endif
    SPAN_ATTR(10, false);
    SPAN_ATTR(10, true);
    SPAN_ATTR(14, false);
    SPAN_ATTR(14, true);
#undef SPAN_ATTR
    return 0;
}

// The state of HIP device `dev` (the current device of the calling thread), created on first use under a lock; it
// lives as long as the process (it holds the pools).
static DeviceState *device_state(int dev)
{
    if (dev < 0 || dev >= MAX_DEVICES) {
        fail("%s", "device index out of range");
        return nullptr;
    }
    DeviceState *ds = g_devs[dev].load(std::memory_order_acquire);
    if (ds != nullptr)
        return ds;
    std::lock_guard<std::mutex> lk(g_devs_mu);
    if ((ds = g_devs[dev].load(std::memory_order_relaxed)) != nullptr)
        return ds;
    ds = new (std::nothrow) DeviceState();
    if (ds == nullptr) {
        fail("%s", "out of memory");
        return nullptr;
    }
    ds->device = dev;
    const char *copy = getenv("PTLS_MI355X_STAGE_COPY"), *limit = getenv("PTLS_MI355X_MAX_STAGE_BYTES");
    ds->force_copy = copy != nullptr && strcmp(copy, "1") == 0;
    const char *coh = getenv("PTLS_MI355X_STAGE_COHERENT");
    ds->stage_coherent = !(coh != nullptr && strcmp(coh, "0") == 0);
    const char *ct = getenv("PTLS_MI355X_CONSTANT_TIME");
    // (round 4) every keyset constant-time unless PTLS_MI355X_CONSTANT_TIME=0: since the window-major segment ends
    // (SEG_COOP) both modes run the same code, whose LDS accesses have data-independent bank patterns, at the same
    // rate; the flag only keeps such keysets off the lockstep schedule
    ds->ct_default = !(ct != nullptr && strcmp(ct, "0") == 0);
    const char *comb = getenv("PTLS_MI355X_COMBINE");
    if (comb != nullptr)
        ds->combine = atoi(comb) < 0 ? 0 : atoi(comb);
    const char *pool = getenv("PTLS_MI355X_STAGE_POOL_BYTES"), *fo = getenv("PTLS_MI355X_FAULT_ORDER");
    if (pool != nullptr)
        ds->stage_pool_cap = (size_t)strtoull(pool, nullptr, 0);
    ds->fault_order = fo != nullptr && strcmp(fo, "1") == 0;
    const char *dg = getenv("PTLS_MI355X_DIAG");
    ds->diag = dg != nullptr && strcmp(dg, "1") == 0;
    ds->stage_limit = limit != nullptr ? (size_t)strtoull(limit, nullptr, 0) : (size_t)4096 << (STAGE_CLASSES - 1);
    int least = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &ds->priority) != hipSuccess)
        ds->priority = 0;
    if (hipDeviceGetAttribute(&ds->ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || set_kernel_attrs() != 0 ||
        hipStreamCreateWithPriority(&ds->setup, hipStreamNonBlocking, ds->priority) != hipSuccess ||
        hipStreamCreateWithPriority(&ds->maint, hipStreamNonBlocking, ds->priority) != hipSuccess) {
        if (ds->setup != nullptr)
            (void)hipStreamDestroy(ds->setup);
        delete ds;
        fail("%s", "device initialisation failed");
        return nullptr;
    }
    g_devs[dev].store(ds, std::memory_order_release);
    return ds;
}

static DeviceState *current_device_state(void)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        fail("%s", "hipGetDevice failed");
        return nullptr;
    }
    return device_state(dev);
}

// makes `dev` the calling thread's current device for the scope of a call (a context may be used from a thread whose
// current device is another one), restoring the previous one after
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev)
    {
        int cur = 0;
        if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess)
            prev = cur;
    }
    ~DeviceScope()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

static hipEvent_t event_get(DeviceState *ds)
{
    {
        std::lock_guard<std::mutex> lk(ds->mu);
        if (!ds->events.empty()) {
            hipEvent_t e = ds->events.back();
            ds->events.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
        return nullptr;
    return e;
}

static void event_put(DeviceState *ds, hipEvent_t e)
{
    if (e == nullptr)
        return;
    std::lock_guard<std::mutex> lk(ds->mu);
    ds->events.push_back(e);
}

// one cleared keyset entry from the slab: a free one, else one whose clearing (keyset_free) has completed, else a new
// slab; *slab is the slab the entry lies in (entries of one slab may be addressed relative to each other)
static KeyEntry *slot_get(DeviceState *ds, KeyEntry **slab_of)
{
    {
        std::lock_guard<std::mutex> lk(ds->mu);
        if (ds->slots.empty()) {
            for (size_t i = 0; i < ds->pending.size();) {
                if (hipEventQuery(ds->pending[i].cleared) == hipSuccess) {
                    ds->slots.emplace_back(ds->pending[i].e, ds->pending[i].slab);
                    ds->events.push_back(ds->pending[i].cleared);
                    ds->pending[i] = ds->pending.back();
                    ds->pending.pop_back();
                } else {
                    (void)hipGetLastError();  // (not ready: not an error for the launches that follow)
                    ++i;
                }
            }
        }
        if (!ds->slots.empty()) {
            const auto e = ds->slots.back();
            ds->slots.pop_back();
            *slab_of = e.second;
            return e.first;
        }
    }
    KeyEntry *slab = nullptr;
    if (hipMalloc((void **)&slab, SLAB_ENTRIES * sizeof(KeyEntry)) != hipSuccess) {
        fail("%s", "keyset slab allocation failed");
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(ds->mu);
    for (int i = SLAB_ENTRIES - 1; i >= 1; --i)
        ds->slots.emplace_back(slab + i, slab);
    *slab_of = slab;
    return slab;
}

static void stager_destroy(Stager *s)
{
    if (s->d != nullptr)
        (void)hipFree(s->d);
    (void)hipHostFree(s->h);  // (an implicit device synchronisation: only buffers beyond the pool's bounds get here)
    delete s;
}

// frees the idle staging buffers of one device (hipHostFree waits for that device)
static void release_idle_stagers(DeviceState *ds)
{
    std::vector<Stager *> idle;
    {
        std::lock_guard<std::mutex> lk(ds->mu);
        for (int c = 0; c < STAGE_CLASSES; ++c) {
            for (Stager *s = ds->stagers[c]; s != nullptr; s = s->next)
                idle.push_back(s);
            ds->stagers[c] = nullptr;
        }
        ds->stage_idle = 0;
    }
    for (Stager *s : idle)
        stager_destroy(s);
}

static Stager *stager_get(DeviceState *ds, size_t bytes)
{
    if (bytes > ds->stage_limit) {
        fail("%s", "staging: the call needs more than PTLS_MI355X_MAX_STAGE_BYTES");
        return nullptr;
    }
    int cls = 0;
    while (cls < STAGE_CLASSES && ((size_t)4096 << cls) < bytes)
        ++cls;
    if (cls == STAGE_CLASSES) {
        fail("%s", "staging: record too large");
        return nullptr;
    }
    hipStream_t stream = nullptr;
    {
        std::lock_guard<std::mutex> lk(ds->mu);
        Stager *s = ds->stagers[cls];
        if (s != nullptr) {
            ds->stagers[cls] = s->next;
            ds->stage_idle -= s->cap;
            ds->stage_busy += s->cap;
            return s;
        }
        // the device's stager streams: created up to STAGE_STREAMS, then shared (a call then may wait for another
        // call's launch on the same stream; calls beyond that many at once would share the few hardware queues anyway)
        if (ds->stage_streams.size() >= STAGE_STREAMS)
            stream = ds->stage_streams[ds->stage_rr++ % STAGE_STREAMS];
    }
    if (stream == nullptr) {
        if (hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, ds->priority) != hipSuccess) {
            // (round 4) a stream that cannot be created now is no reason to fail the call: share an existing one
            (void)hipGetLastError();
            std::lock_guard<std::mutex> lk(ds->mu);
            if (ds->stage_streams.empty()) {
                fail("%s", "staging: stream creation failed");
                return nullptr;
            }
            stream = ds->stage_streams[ds->stage_rr++ % ds->stage_streams.size()];
        } else {
            std::lock_guard<std::mutex> lk(ds->mu);
            ds->stage_streams.push_back(stream);
        }
    }
    Stager *s = new (std::nothrow) Stager();
    if (s == nullptr) {
        fail("%s", "out of memory");
        return nullptr;
    }
    s->stream = stream;
    s->cap = (size_t)4096 << cls;
    s->cls = cls;
    // Fine-grained (coherent) pinned memory: kernels read the staged input and write the results in place over PCIe,
    // and the host rewrites the same bytes for the next call right after it sees the completion words. Coarse-grained
    // host memory (hipHostMallocDefault under HIP_HOST_COHERENT=0) may be cached in the GPU's L2, where a later
    // kernel on this buffer can read lines of the previous call's input.
    const unsigned hflags = ds->stage_coherent ? hipHostMallocCoherent : hipHostMallocDefault;
    if (hipHostMalloc((void **)&s->h, s->cap, hflags) != hipSuccess) {
        // (round 4) the pinned memory of idle buffers of other sizes is what this one may need: free this device's
        // (not every device's -- hipHostFree synchronises the device it frees for), try again
        (void)hipGetLastError();
        release_idle_stagers(ds);
        if (hipHostMalloc((void **)&s->h, s->cap, hflags) != hipSuccess) {
            (void)hipGetLastError();
            delete s;
            fail("%s", "staging: pinned host allocation failed");
            return nullptr;
        }
    }
    if (ds->force_copy || hipHostGetDevicePointer((void **)&s->h_dev, s->h, 0) != hipSuccess) {
        (void)hipGetLastError();  // (handled: the copy path)
        s->h_dev = nullptr;
    }
    if (s->h_dev == nullptr && hipMalloc((void **)&s->d, s->cap) != hipSuccess) {
        (void)hipHostFree(s->h);
        delete s;
        fail("%s", "staging: device allocation failed");
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(ds->mu);
    ds->stage_busy += s->cap;
    return s;
}

// back to the pool after its call (nothing of the call is still queued on its stream); a buffer beyond the pool's bounds
// (above STAGE_KEEP_MAX, or with the idle pool full) is freed instead
static void stager_put(DeviceState *ds, Stager *s)
{
    {
        std::lock_guard<std::mutex> lk(ds->mu);
        ds->stage_busy -= s->cap;
        if (s->cap <= STAGE_KEEP_MAX && ds->stage_idle + s->cap <= ds->stage_pool_cap) {
            s->next = ds->stagers[s->cls];
            ds->stagers[s->cls] = s;
            ds->stage_idle += s->cap;
            return;
        }
    }
    stager_destroy(s);
}

struct st_ptls_mi355x_keyset_t {
    DeviceState *ds;
    int device;
    size_t nkeys, key_size;
    int nr;
    KeyEntry *d_keys;
    bool slot;  // d_keys is one entry of the device's slab (one-key keysets)
    KeyEntry *slab;  // ... that slab
    int schedule;
    bool ct;                           // constant-time GHASH (ptls_mi355x_keyset_set_constant_time)
    hipEvent_t ready;                  // the last setup / update / set_iv of the entries
    std::atomic<bool> ready_seen;      // ... known to be complete: launches need not wait for it
    // a one-key keyset's setup waits for its first use and runs on that use's stream (no cross-stream wait for the
    // first seal of a context); until then the raw key stays here (cleared once launched)
    std::atomic<bool> pending;
    RawKey raw;
    std::vector<uint8_t> ivs;          // the static IVs (do_get_iv reads these; the device copy is what seals use)
    std::mutex mu;                     // launches from several threads: uses, group scratch
    std::vector<std::pair<hipStream_t, hipEvent_t>> uses;  // per stream: after this keyset's last launch on it
    // key grouping of ungrouped many-key batches (key_group_*): scratch for key counts and the record permutation,
    // grown on demand (stream-ordered); group_ev orders its users when batches on several streams share the keyset
    u32 *d_group;
    size_t group_cap;
    hipEvent_t group_ev;
    // small batches with long records (spread_pieces): the pieces' partials and per-record counters (zero
    // between launches), allocated on first use; spread_stream: the stream of the last launch that used them (a launch
    // on another stream waits for that one's use event, note_use)
    uint8_t *d_spread;
    size_t spread_cap;  // its bytes (sized for the batches seen so far, spread_bytes)
    hipStream_t spread_stream;
    bool spread_used;
    // W8 launch pairs (launch_chunked, W8_HORNER): one word per workgroup from the pair's first kernel to its second,
    // one buffer per stream (allocated on the stream's first pair; a stream orders its own pairs), so that pairs on
    // several streams run concurrently; at most W8_FLAG_STREAMS, the oldest taken over by a new stream in stream order
    std::vector<std::pair<hipStream_t, u32 *>> w8flags;
};

static int mark_ready(ptls_mi355x_keyset_t *ks, hipStream_t s);

// launches a pending one-key setup on `s` (the stream of the keyset's first use, or the maintenance stream); returns 1
// when it did (work on `s` is then ordered after it), 0 when there was none, -1 on failure
static int setup_now(ptls_mi355x_keyset_t *ks, hipStream_t s)
{
    if (!ks->pending.load(std::memory_order_acquire))
        return 0;
    std::lock_guard<std::mutex> lk(ks->mu);
    if (!ks->pending.load(std::memory_order_relaxed))
        return 0;
    LAUNCH_CLEAR();
    keyset_setup_one_kernel<<<1, 64, 0, s>>>(ks->raw, ks->d_keys);
    if (hipGetLastError() != hipSuccess)
        return fail("%s", "keyset setup launch failed");
    clear_memory(&ks->raw, sizeof(ks->raw));
    if (mark_ready(ks, s) != 0)
        return -1;
    ks->pending.store(false, std::memory_order_release);
    return 1;
}

// makes `s` wait for the keyset's last setup / update / set_iv, unless that is known to be complete
static int wait_ready(ptls_mi355x_keyset_t *ks, hipStream_t s)
{
    const int now = setup_now(ks, s);
    if (now != 0)
        return now < 0 ? -1 : 0;
    if (ks->ready_seen.load(std::memory_order_acquire))
        return 0;
    hipError_t q = hipEventQuery(ks->ready);
    if (q == hipSuccess) {
        ks->ready_seen.store(true, std::memory_order_release);
        return 0;
    }
    if (q != hipErrorNotReady)
        return fail("keyset setup failed: %s", hipGetErrorString(q));
    (void)hipGetLastError();  // (not an error: launches after this are checked with hipGetLastError)
    HIP_TRY(hipStreamWaitEvent(s, ks->ready, 0));
    return 0;
}

// records that the keyset's entries were used by work just launched on `s` (teardown and rekey wait for it); the
// caller holds ks->mu
static int note_use_locked(ptls_mi355x_keyset_t *ks, hipStream_t s)
{
    for (auto &u : ks->uses)
        if (u.first == s)
            return hipEventRecord(u.second, s) == hipSuccess ? 0 : fail("%s", "hipEventRecord failed");
    hipEvent_t e = event_get(ks->ds);
    if (e == nullptr)
        return fail("%s", "event creation failed");
    ks->uses.emplace_back(s, e);
    HIP_TRY(hipEventRecord(e, s));
    return 0;
}

static int note_use(ptls_mi355x_keyset_t *ks, hipStream_t s)
{
    std::lock_guard<std::mutex> lk(ks->mu);
    return note_use_locked(ks, s);
}

// orders the maintenance stream after every launch that used the keyset and after its last setup
static int maint_after_uses(ptls_mi355x_keyset_t *ks)
{
    if (setup_now(ks, ks->ds->maint) < 0)
        return -1;
    std::lock_guard<std::mutex> lk(ks->mu);
    for (auto &u : ks->uses)
        HIP_TRY(hipStreamWaitEvent(ks->ds->maint, u.second, 0));
    if (!ks->ready_seen.load(std::memory_order_acquire))
        HIP_TRY(hipStreamWaitEvent(ks->ds->maint, ks->ready, 0));
    return 0;
}

static int mark_ready(ptls_mi355x_keyset_t *ks, hipStream_t s)
{
    ks->ready_seen.store(false, std::memory_order_release);
    HIP_TRY(hipEventRecord(ks->ready, s));
    return 0;
}

static void keyset_destroy(ptls_mi355x_keyset_t *ks)
{
    DeviceState *ds = ks->ds;
    for (auto &u : ks->uses)
        event_put(ds, u.second);
    event_put(ds, ks->ready);
    if (ks->group_ev != nullptr)
        (void)hipEventDestroy(ks->group_ev);
    clear_memory(ks->ivs.data(), ks->ivs.size());
    clear_memory(&ks->raw, sizeof(ks->raw));
    delete ks;
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
    DeviceState *ds = current_device_state();
    if (ds == nullptr)
        return NULL;
    ptls_mi355x_keyset_t *ks = new (std::nothrow) st_ptls_mi355x_keyset_t();
    if (ks == nullptr) {
        fail("%s", "out of memory");
        return NULL;
    }
    ks->ds = ds;
    ks->device = ds->device;
    ks->nkeys = nkeys, ks->key_size = key_size, ks->nr = key_size == 16 ? 10 : 14;
    ks->ct = ds->ct_default;
    ks->ready_seen.store(false);
    ks->pending.store(false);
    ks->ivs.assign((const uint8_t *)ivs, (const uint8_t *)ivs + nkeys * 12);
    if ((ks->ready = event_get(ds)) == nullptr) {
        fail("%s", "ptls_mi355x_keyset_new: event creation failed");
        delete ks;
        return NULL;
    }
    if (nkeys == 1) {
        // a picotls context: a slab entry, and the setup launch (the key in its arguments) deferred to the first use,
        // on that use's stream (setup_now)
        if ((ks->d_keys = slot_get(ds, &ks->slab)) == nullptr) {
            keyset_destroy(ks);
            return NULL;
        }
        ks->slot = true;
        memcpy(ks->raw.key, keys, key_size);
        memcpy(ks->raw.iv, ivs, 12);
        ks->raw.key_size = (u32)key_size;
        ks->pending.store(true, std::memory_order_release);
        return ks;
    }
    // many keys: entries and the raw key material in stream-ordered memory on the setup stream. The caller's arrays are
    // pageable host memory, so the call waits (for the setup stream only) until the copies have consumed them.
    uint8_t *d_raw = nullptr;
    const size_t raw_bytes = nkeys * (key_size + 12);
    bool ok = hipMallocAsync((void **)&ks->d_keys, nkeys * sizeof(KeyEntry), ds->setup) == hipSuccess &&
              hipMallocAsync((void **)&d_raw, raw_bytes, ds->setup) == hipSuccess &&
              hipMemcpyAsync(d_raw, keys, nkeys * key_size, hipMemcpyHostToDevice, ds->setup) == hipSuccess &&
              hipMemcpyAsync(d_raw + nkeys * key_size, ivs, nkeys * 12, hipMemcpyHostToDevice, ds->setup) == hipSuccess;
    if (ok) {
        LAUNCH_CLEAR();
        keyset_setup_kernel<<<(unsigned)((nkeys + 127) / 128), 128, 0, ds->setup>>>(d_raw, d_raw + nkeys * key_size, ks->d_keys,
                                                                                   (u32)nkeys, (u32)key_size);
        ok = hipGetLastError() == hipSuccess;
    }
    if (d_raw != nullptr) {
        (void)hipMemsetAsync(d_raw, 0, raw_bytes, ds->setup);
        (void)hipFreeAsync(d_raw, ds->setup);
    }
    if (ok)
        ok = mark_ready(ks, ds->setup) == 0 && hipStreamSynchronize(ds->setup) == hipSuccess;
    if (!ok) {
        if (ks->d_keys != nullptr)
            (void)hipFreeAsync(ks->d_keys, ds->setup);
        fail("%s", "ptls_mi355x_keyset_new: device setup failed");
        keyset_destroy(ks);
        return NULL;
    }
    return ks;
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
    DeviceScope scope(ks->device);
    DeviceState *ds = ks->ds;
    // stream-ordered on the maintenance stream: after every launch already made with the old entries, before any made
    // after this call (they wait for `ready`)
    if (maint_after_uses(ks) != 0)
        return -1;
    uint8_t *d = NULL;
    const size_t kb = n * ks->key_size, ib = n * 12, sb = n * 4;
    HIP_TRY(hipMallocAsync((void **)&d, kb + ib + sb, ds->maint));
    int ret = -1;
    if (hipMemcpyAsync(d, keys, kb, hipMemcpyHostToDevice, ds->maint) == hipSuccess &&
        hipMemcpyAsync(d + kb, ivs, ib, hipMemcpyHostToDevice, ds->maint) == hipSuccess &&
        hipMemcpyAsync(d + kb + ib, key_idx, sb, hipMemcpyHostToDevice, ds->maint) == hipSuccess) {
        LAUNCH_CLEAR();
        keyset_setup_kernel<<<(unsigned)((n + 127) / 128), 128, 0, ds->maint>>>(d, d + kb, ks->d_keys, (u32)n, (u32)ks->key_size,
                                                                               (const u32 *)(d + kb + ib));
        if (hipGetLastError() == hipSuccess && mark_ready(ks, ds->maint) == 0)
            ret = 0;
    }
    (void)hipMemsetAsync(d, 0, kb + ib, ds->maint);
    (void)hipFreeAsync(d, ds->maint);
    // the caller's pageable arrays must have been consumed before returning
    if (hipStreamSynchronize(ds->maint) != hipSuccess)
        ret = -1;
    if (ret != 0)
        return fail("%s", "keyset_update: device setup failed");
    for (size_t i = 0; i < n; ++i)
        memcpy(ks->ivs.data() + (size_t)key_idx[i] * 12, (const uint8_t *)ivs + i * 12, 12);
    return 0;
}

void ptls_mi355x_keyset_free(ptls_mi355x_keyset_t *ks)
{
    if (ks == NULL)
        return;
    DeviceScope scope(ks->device);
    DeviceState *ds = ks->ds;
    ks->pending.store(false, std::memory_order_release);  // never used: its setup never ran (the raw key is cleared below)
    // key material is cleared (ptls_clear_memory, lib/fusion.c:1045) after the keyset's last launch, on the maintenance
    // stream; nothing here waits on the host
    bool ordered = !ds->fault_order && maint_after_uses(ks) == 0;
    if (ks->group_ev != nullptr && hipStreamWaitEvent(ds->maint, ks->group_ev, 0) != hipSuccess)
        ordered = false;
    if (!ordered) {
        // the teardown cannot be ordered after the keyset's launches on the device: wait for each of them (the recorded
        // uses on every stream, the setup, the key grouping) on the host before clearing; if even that fails, keep the
        // entries as they are and never reuse them, rather than clear them under a launch still reading them
        bool drained = true;
        {
            std::lock_guard<std::mutex> lk(ks->mu);
            for (auto &u : ks->uses)
                drained = hipEventSynchronize(u.second) == hipSuccess && drained;
        }
        drained = hipEventSynchronize(ks->ready) == hipSuccess && drained;
        if (ks->group_ev != nullptr)
            drained = hipEventSynchronize(ks->group_ev) == hipSuccess && drained;
        if (!drained) {
            keyset_destroy(ks);
            return;
        }
    }
    (void)hipMemsetAsync(ks->d_keys, 0, ks->nkeys * sizeof(KeyEntry), ds->maint);
    if (ks->d_group != nullptr)
        (void)hipFreeAsync(ks->d_group, ds->maint);
    if (ks->d_spread != nullptr)
        (void)hipFreeAsync(ks->d_spread, ds->maint);
    for (auto &f : ks->w8flags)
        (void)hipFreeAsync(f.second, ds->maint);
    ks->w8flags.clear();
    if (ks->slot) {
        // back to the pool once the clear has run (slot_get checks the event)
        hipEvent_t cleared = event_get(ds);
        if (cleared != nullptr && hipEventRecord(cleared, ds->maint) == hipSuccess) {
            std::lock_guard<std::mutex> lk(ds->mu);
            ds->pending.push_back({ks->d_keys, ks->slab, cleared});
        }
    } else {
        (void)hipFreeAsync(ks->d_keys, ds->maint);
    }
    keyset_destroy(ks);
}

#if ENGINE_PROFILE
int ptls_mi355x_debug_profile(unsigned long long *out, int reset)
{
    HIP_TRY(hipDeviceSynchronize());
    static unsigned long long rows[PROF_ROWS][PROF_SLOTS];
    HIP_TRY(hipMemcpyFromSymbol(rows, HIP_SYMBOL(g_prof), sizeof(g_prof)));
    for (int i = 0; i < PROF_SLOTS; ++i) {
        out[i] = 0;
        for (int r = 0; r < PROF_ROWS; ++r)
            out[i] += rows[r][i];
    }
    if (reset) {
        memset(rows, 0, sizeof(rows));
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), rows, sizeof(g_prof)));
    }
    return 0;
}
#endif

// ---- test and measurement hooks (include/picotls/mi355x_debug.h)

// reads (and with reset, zeroes in the same atomic exchange) the per-workgroup run counters, so that a launch finishing
// meanwhile is counted once, in this read or the next
__global__ void ext_runs_take_kernel(unsigned long long *out, int reset)
{
    for (u32 i = threadIdx.x; i < EXT_RUN_ROWS * 8; i += blockDim.x) {
        unsigned long long *c = &g_ext_runs[i / 8][i % 8];
        out[i] = reset ? atomicExch(c, 0ull) : __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int ptls_mi355x_debug_counters(uint64_t *out, int reset)
{
    if (out == NULL)
        return fail("%s", "debug_counters: invalid arguments");
    // (test-only) every launch made so far has finished, and counted its runs, before anything is read
    HIP_TRY(hipDeviceSynchronize());
    for (int i = 0; i < 8; ++i)
        out[i] = reset ? g_launches[i].exchange(0) : g_launches[i].load();
    std::vector<unsigned long long> rows((size_t)EXT_RUN_ROWS * 8);
    unsigned long long *d = nullptr;
    HIP_TRY(hipMalloc(&d, rows.size() * sizeof(rows[0])));
    LAUNCH_CLEAR();
    ext_runs_take_kernel<<<1, 256>>>(d, reset);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpy(rows.data(), d, rows.size() * sizeof(rows[0]), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess)
        return fail("debug_counters: %s", hipGetErrorString(e));
    for (int i = 0; i < 8; ++i) {
        out[8 + i] = 0;
        for (int r = 0; r < EXT_RUN_ROWS; ++r)
            out[8 + i] += rows[(size_t)r * 8 + i];
    }
    return 0;
}

int ptls_mi355x_debug_kernel_clock(void *buf, unsigned cap)
{
    unsigned long long *b = (unsigned long long *)buf;
    const unsigned zero = 0, c = buf != NULL ? cap : 0;
    HIP_TRY(hipDeviceSynchronize());  // (test-only: no launch may be sampling while the buffer changes)
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_kclock_n), &zero, sizeof(zero)));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_kclock_cap), &c, sizeof(c)));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_kclock_buf), &b, sizeof(b)));
    return 0;
}

int ptls_mi355x_debug_kernel_clock_count(void)
{
    unsigned n = 0;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_kclock_n), sizeof(n)));
    return (int)n;
}

int ptls_mi355x_debug_inject_error(void)
{
    // a handled-looking failure of the kind the per-record path meets (hipHostGetDevicePointer on memory HIP did not
    // allocate), deliberately NOT cleared: the thread's last error is left set, as a handled failure used to leave it
    static uint8_t pageable[64];
    void *p = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&p, pageable, 0);
    return (int)(e != hipSuccess ? hipPeekAtLastError() : hipSuccess);
}

int ptls_mi355x_debug_clock_sample(void *out, void *stream)
{
    if (out == NULL)
        return fail("%s", "debug_clock_sample: invalid arguments");
    LAUNCH_CLEAR();
    clock_probe_kernel<<<1, 64, 0, (hipStream_t)stream>>>((unsigned long long *)out);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ptls_mi355x_debug_wallclock_khz(void)
{
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
        return 0;
    return khz;
}

int ptls_mi355x_keyset_set_schedule(ptls_mi355x_keyset_t *ks, int schedule)
{
    if (ks == NULL || schedule < PTLS_MI355X_SCHEDULE_AUTO || schedule > PTLS_MI355X_SCHEDULE_CHUNKED)
        return fail("%s", "set_schedule: invalid arguments");
    ks->schedule = schedule;
    return 0;
}

int ptls_mi355x_keyset_set_constant_time(ptls_mi355x_keyset_t *ks, int on)
{
    if (ks == NULL)
        return fail("%s", "set_constant_time: invalid arguments");
    ks->ct = on != 0;
    return 0;
}

int ptls_mi355x_keyset_get_constant_time(const ptls_mi355x_keyset_t *ks) { return ks != NULL && ks->ct ? 1 : 0; }

size_t ptls_mi355x_keyset_size(const ptls_mi355x_keyset_t *ks) { return ks->nkeys; }
size_t ptls_mi355x_keyset_key_size(const ptls_mi355x_keyset_t *ks) { return ks->key_size; }
int ptls_mi355x_keyset_device(const ptls_mi355x_keyset_t *ks) { return ks->device; }

size_t ptls_mi355x_staging_bytes(void)
{
    size_t n = 0;
    for (int d = 0; d < MAX_DEVICES; ++d) {
        DeviceState *ds = g_devs[d].load(std::memory_order_acquire);
        if (ds == nullptr)
            continue;
        std::lock_guard<std::mutex> lk(ds->mu);
        n += ds->stage_idle + ds->stage_busy;
    }
    return n;
}

void ptls_mi355x_release_staging(void)
{
    for (int d = 0; d < MAX_DEVICES; ++d) {
        DeviceState *ds = g_devs[d].load(std::memory_order_acquire);
        if (ds == nullptr)
            continue;
        DeviceScope scope(d);
        release_idle_stagers(ds);
    }
}

int ptls_mi355x_keyset_get_iv(ptls_mi355x_keyset_t *ks, size_t key_idx, void *iv)
{
    if (ks == NULL || key_idx >= ks->nkeys || iv == NULL)
        return fail("%s", "get_iv: bad key index");
    memcpy(iv, ks->ivs.data() + key_idx * 12, 12);
    return 0;
}

int ptls_mi355x_keyset_set_iv(ptls_mi355x_keyset_t *ks, size_t key_idx, const void *iv)
{
    if (ks == NULL || key_idx >= ks->nkeys || iv == NULL)
        return fail("%s", "set_iv: bad key index");
    DeviceScope scope(ks->device);
    if (maint_after_uses(ks) != 0)
        return -1;
    u32 w[3];
    memcpy(w, iv, 12);
    LAUNCH_CLEAR();
    keyset_set_iv_kernel<<<1, 1, 0, ks->ds->maint>>>(ks->d_keys + key_idx, w[0], w[1], w[2]);
    HIP_TRY(hipGetLastError());
    if (mark_ready(ks, ks->ds->maint) != 0)
        return -1;
    memcpy(ks->ivs.data() + key_idx * 12, iv, 12);
    return 0;
}

}  // extern "C"

// Schedule choice (ptls_mi355x_keyset_set_schedule): AUTO = chunked. Its uniform runs take the whole-record path,
// which measured at or above the lockstep kernel on one-key uniform batches (929 vs 841 GiB/s on 16 KiB records,
// 784 vs 751 on 1200 B), and its chunked runs balance mixed lengths and short key runs.
static bool use_chunked(int schedule) { return schedule != PTLS_MI355X_SCHEDULE_LOCKSTEP; }

// Since the window-major segment ends (SEG_COOP) the constant-time template argument changes no instruction of the
// chunked and span kernels: every keyset, constant-time or not, launches the CT instantiation, so the
// code object holds one set of these kernels
template <int NR, bool OPEN, int FRAME, int EXT = 0>
static void launch_chunked_x(bool ct, unsigned grid, hipStream_t s, const BatchArgs &a)
{
    COUNT_LAUNCH(EXT == 5 ? 4 : EXT);  // (the MK form of the serial W8 kernel counts as it)
#if SEG_COOP
    (void)ct;
    gcm_chunked_kernel<NR, OPEN, FRAME, true, EXT><<<grid, ENGINE_WG, CLDS_ALLOC, s>>>(a);
#else
    if (ct)
        gcm_chunked_kernel<NR, OPEN, FRAME, true, EXT><<<grid, ENGINE_WG, CLDS_ALLOC, s>>>(a);
    else
        gcm_chunked_kernel<NR, OPEN, FRAME, false, EXT><<<grid, ENGINE_WG, CLDS_ALLOC, s>>>(a);
#endif
}

// the instantiation for the launch: unframed batches with a spread plan (EXT 1) or header-protection masks (EXT 2)
// have their own (gcm_chunked_kernel)
template <int NR, bool OPEN, int FRAME>
static void launch_chunked(bool ct, unsigned grid, hipStream_t s, const BatchArgs &a)
{
    if constexpr (FRAME == 0) {
        if (a.spread) {
            launch_chunked_x<NR, OPEN, 0, 1>(ct, grid, s, a);
            return;
        }
        if constexpr (!OPEN) {
            if (a.hp != nullptr) {
                launch_chunked_x<NR, false, 0, 2>(ct, grid, s, a);
                return;
            }
        }
    }
    // The W8 kernels (the Horner step on an 8-bit H^8 table, ghash.h gmul8) for every run of an unframed or TLS-framed
    // batch: EXT 4 (segment ends by a serial lane Horner) takes all runs but those of long whole records, which EXT 3
    // (the butterfly end: on 16 KiB records it measured 1 % above the serial one) takes after it, each skipping the
    // other's runs and EXT 3 returning at once in the workgroups where EXT 4 saw none (BatchArgs::w8_split, w8_flags).
    // A batch of fewer than WHOLE_MIN_RECS records per workgroup in contiguous ranges holds no whole-record run: EXT 4
    // alone. Not for a per-record launch (it publishes completion words, and its 1-16-step units suit the 4-bit path),
    // nor a batch of fewer than W8_MIN_RECS records (the table build is not repaid). TLS 1.2 framing only with W8_TLS12
    // (on: faster despite EXT 4's 96-byte-per-lane seal spill, common.h).
    if constexpr (W8_HORNER && (FRAME != 2 || W8_TLS12)) {
        if (!a.one_inline && a.done_flag == nullptr && a.nrecs >= W8_MIN_RECS) {
            const bool whole_possible = a.chunk != 0 || a.bounds != nullptr || (a.nrecs + grid - 1) / grid >= WHOLE_MIN_RECS;
            BatchArgs b = a;
            b.w8_split = whole_possible ? 2u : 1u;
            if (!whole_possible)
                b.w8_flags = nullptr;
            // (round 6) many-key batches take EXT 5: EXT 4 plus multi-key runs (gcm_kernels.h scan_mk); one-key batches
            // keep EXT 4, whose code the MK path would grow (small launches slowed by 5-14 % with it compiled in)
            if (MK_RUNS && a.multi_key)
                launch_chunked_x<NR, OPEN, FRAME, 5>(ct, grid, s, b);
            else
                launch_chunked_x<NR, OPEN, FRAME, 4>(ct, grid, s, b);
            if (whole_possible)
                launch_chunked_x<NR, OPEN, FRAME, 3>(ct, grid, s, b);
            return;
        }
    }
    launch_chunked_x<NR, OPEN, FRAME>(ct, grid, s, a);
}

// Records per chunk of the chunked kernel's dealt-out assignment (BatchArgs::chunk), 0 for contiguous ranges. Each
// workgroup gets up to CHUNKS_PER_WG chunks spread over the batch, so that a batch ordered by record size (or by
// connections whose records differ in size) still shares its bytes evenly: 4M records of U[64 B, 16 KiB] sorted by
// length ran at 467 GiB/s seal+open with contiguous ranges against 802 in random order (bench.py, mixedsorted vs
// mixed1key). Chunks stay at least CHUNK_MIN_RECS records (whole-record runs need 128 and gain from more), and a
// batch too small for two such chunks per workgroup keeps contiguous ranges.
#ifndef CHUNKS_PER_WG
#define CHUNKS_PER_WG 8
#endif
#define CHUNK_MIN_RECS 256
#ifndef BALANCE
#define BALANCE 1  // many-key batches: workgroup ranges balanced by weight (balance_*_kernel)
#endif
#define BALANCE_MIN_RECS ((size_t)131072)  // ... from this many records (2 x 256 per workgroup)
static u64 deal_chunk(u64 nrecs, u64 grid)
{
    for (u64 k = CHUNKS_PER_WG; k >= 2; k /= 2) {
        const u64 c = (nrecs + grid * k - 1) / (grid * k);
        if (c >= CHUNK_MIN_RECS)
            return c;
    }
    return 0;
}

// scratch of spread launches: per-record piece counters (SPREAD_MAX_RECS, zero between launches), then the pieces'
// partials: at most one piece per spare workgroup, or (records longer than 2^10 units x their share) 2^23 steps /
// SPREAD_UNIT_STEPS / 2^10 per record (PTLS_MI355X_MAX_RECORD_LEN)
#define SPREAD_MAX_RECS 255
#define SPREAD_CNT_BYTES ((size_t)256 * 4)

// Header-protection masks computed by the chunked seal launch itself (BatchArgs::hp; seal_batch_hp, encrypt_s)
struct HpLaunch {
    const ptls_mi355x_hp_t *hp;
    const KeyEntry *keys;
    u32 nkeys;
    int nr;
    uint8_t *masks;
};

// The GCM kernel launch of a batch over `nkeys` entries at `keys` (no key grouping, no keyset bookkeeping). ct: the
// constant-time GHASH variant of the chunked kernel (the lockstep schedule is not offered in that mode). hpl: the
// header-protection masks of the sealed records in the same launch (chunked seal of unframed records only).
static int launch_gcm(const KeyEntry *keys, u32 nkeys, int nr, int ncu, int schedule, bool ct, bool open,
                      const ptls_mi355x_record_t *recs, size_t nrecs, const void *in, const void *aad, void *out, uint8_t *ok,
                      hipStream_t s, int frame, u32 unit_log2, const ptls_mi355x_record_t *grouped = nullptr,
                      const u32 *perm = nullptr, const u32 *perm_on = nullptr, const ptls_mi355x_record_t *one = nullptr,
                      u32 *done_flag = nullptr, const u64 *bounds = nullptr, const HpLaunch *hpl = nullptr,
                      uint8_t *spread = nullptr, u32 done_token = 0, u32 *w8_flags = nullptr)
{
    BatchArgs a = {keys, recs, (u64)nrecs, (const uint8_t *)in, (const uint8_t *)aad, (uint8_t *)out, ok,
                   nkeys > 1 ? 1u : 0u, nkeys, unit_log2, grouped, perm, perm_on, 0u, {}, done_flag, 0, bounds};
    a.done_token = done_token;
    a.w8_flags = w8_flags;
    if (hpl != nullptr) {
        if (open || frame != 0 || !(ct || use_chunked(schedule)))
            return fail("%s", "launch_gcm: header-protection masks need the chunked seal of unframed records");
        a.hp = hpl->hp, a.hp_keys = hpl->keys, a.hp_nkeys = hpl->nkeys, a.hp_nr = (u32)hpl->nr, a.masks = hpl->masks;
    }
    if (one != nullptr && nrecs == 1)  // the chunked kernel takes a lone record's descriptor from its arguments
        a.one_inline = 1, a.one = *one;
    if (a.aad == NULL)
        a.aad = a.in;
    // one persistent workgroup per CU. A batch with fewer records than CUs takes one workgroup per record, or (spread,
    // an unframed batch: spread_pieces) one per CU, the workgroups beyond the records sharing its long records
    u64 grid = (u64)ncu;
    if (spread != nullptr && frame == 0 && nrecs >= 2 && nrecs < (u64)ncu && nrecs <= SPREAD_MAX_RECS &&
        hpl == nullptr && one == nullptr && (ct || use_chunked(schedule))) {
        a.spread = 1;
        a.spread_cnt = (u32 *)spread;
        a.spread_part = (u32x4 *)(spread + SPREAD_CNT_BYTES);
    }
    if (grid > nrecs && !a.spread)
        grid = nrecs;
    if (grid < 1)
        grid = 1;
    a.chunk = deal_chunk(nrecs, grid);
#define CHUNKED_LAUNCH(nr_, op, frame_) launch_chunked<nr_, op, frame_>(ct, (unsigned)grid, s, a)
#define CHUNKED_BY_KEY(frame_)                                                                                          \
    do {                                                                                                                \
        if (nr == 10) {                                                                                                 \
            if (open)                                                                                                   \
                CHUNKED_LAUNCH(10, true, frame_);                                                                       \
            else                                                                                                        \
                CHUNKED_LAUNCH(10, false, frame_);                                                                      \
        } else {                                                                                                        \
            if (open)                                                                                                   \
                CHUNKED_LAUNCH(14, true, frame_);                                                                       \
            else                                                                                                        \
                CHUNKED_LAUNCH(14, false, frame_);                                                                      \
        }                                                                                                               \
    } while (0)
    if (frame == 1)
        CHUNKED_BY_KEY(1);
    else if (frame == 2)
        CHUNKED_BY_KEY(2);
    else if (ct || use_chunked(schedule))
        CHUNKED_BY_KEY(0);
    else if ((COUNT_LAUNCH(5), nr == 10)) {
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
#undef CHUNKED_BY_KEY
#undef CHUNKED_LAUNCH
    HIP_TRY(hipGetLastError());
    return 0;
}

// One long record (descriptor `one`, key entry `key`) over many workgroups (span_kernels.h): `units` 16-step units in
// spans of 2^e, their partials at `part` (nspans x 16 B, device-addressable), then the combine launch, which writes the
// tag or ok[0] and sets done_flag[0] when given.
template <int NR, bool OPEN>
static void launch_span_kernel(bool ct, u32 nspans, hipStream_t s, const BatchArgs &a, u32 span, u32 units, void *part)
{
    COUNT_LAUNCH(6);
#if SEG_COOP  // (one instantiation for both settings, as launch_chunked_x)
    (void)ct;
    gcm_span_kernel<NR, OPEN, true><<<nspans, ENGINE_WG, SPAN_LDS, s>>>(a, span, units, (u32x4 *)part);
#else
    if (ct)
        gcm_span_kernel<NR, OPEN, true><<<nspans, ENGINE_WG, SPAN_LDS, s>>>(a, span, units, (u32x4 *)part);
    else
        gcm_span_kernel<NR, OPEN, false><<<nspans, ENGINE_WG, SPAN_LDS, s>>>(a, span, units, (u32x4 *)part);
#endif
}

static int launch_span(const KeyEntry *key, int nr, bool ct, bool open, const ptls_mi355x_record_t &one, const void *in,
                       const void *aad, void *out, uint8_t *ok, u32 units, u32 e, u32 nspans, void *part, u32 *done_flag,
                       u32 done_token, hipStream_t s)
{
    BatchArgs a = {key, nullptr, 1, (const uint8_t *)in, (const uint8_t *)aad, (uint8_t *)out, ok, 0u, 1u, CHUNK_LOG2,
                   nullptr, nullptr, nullptr, 1u, one, done_flag, 0, nullptr};
    a.done_token = done_token;
    const u32 span = 1u << e;
    if (nr == 10) {
        if (open)
            launch_span_kernel<10, true>(ct, nspans, s, a, span, units, part);
        else
            launch_span_kernel<10, false>(ct, nspans, s, a, span, units, part);
    } else {
        if (open)
            launch_span_kernel<14, true>(ct, nspans, s, a, span, units, part);
        else
            launch_span_kernel<14, false>(ct, nspans, s, a, span, units, part);
    }
    HIP_TRY(hipGetLastError());
    const size_t clds = GHASH_TABLE_BYTES + 16 * 257;
    if (open)
        span_combine_kernel<true><<<1, 256, clds, s>>>(a, nspans, e, (const u32x4 *)part);
    else
        span_combine_kernel<false><<<1, 256, clds, s>>>(a, nspans, e, (const u32x4 *)part);
    HIP_TRY(hipGetLastError());
    return 0;
}

// (pieces of a record: at most its units / 2^10 + 1, 2^23 / SPREAD_UNIT_STEPS / 2^10 + 1 for the longest record)
static size_t spread_bytes(int ncu, size_t nrecs)
{
    return SPREAD_CNT_BYTES + 16 * ((size_t)ncu + nrecs * (8192 / SPREAD_UNIT_STEPS + 1));
}

static bool spread_eligible(const ptls_mi355x_keyset_t *ks, size_t nrecs, int frame)
{
    return frame == 0 && nrecs >= 2 && nrecs < (size_t)ks->ds->ncu && nrecs <= SPREAD_MAX_RECS && (ks->ct || use_chunked(ks->schedule));
}

// a batch that may launch the W8 pair (launch_chunked): chunked, W8_MIN_RECS records (TLS 1.2 framing with W8_TLS12)
static bool w8_eligible(const ptls_mi355x_keyset_t *ks, size_t nrecs, int frame)
{
    return W8_HORNER && (frame != 2 || W8_TLS12) && nrecs >= W8_MIN_RECS && (ks->ct || use_chunked(ks->schedule));
}

// orders a launch on `s` that uses the keyset's spread scratch after the last launch that used it;
// the caller holds ks->mu from here through the launch and the use event recorded after it (launch_batch)
static int scratch_order_locked(ptls_mi355x_keyset_t *ks, hipStream_t s)
{
    // a launch on another stream than the last user waits for that launch (its use event, recorded after it by
    // note_use_locked); back-to-back launches on one stream add no event packets (a wait and a record per launch cost a
    // 23 us small-batch launch 7 us)
    if (ks->spread_used && ks->spread_stream != s) {
        for (auto &u : ks->uses)
            if (u.first == ks->spread_stream && hipStreamWaitEvent(s, u.second, 0) != hipSuccess)
                return -1;
    }
    ks->spread_stream = s;
    ks->spread_used = true;
    return 0;
}

// the keyset's W8 flag words for a launch on `s`: the stream's own buffer (every word is written by the pair's first
// kernel before its second reads it, and a stream runs its pairs in order), allocated in stream order on the stream's
// first pair. A stream beyond W8_FLAG_STREAMS takes over the least recently used buffer after that buffer's last use
// (the keyset's use event on its stream). nullptr on failure: the pair then runs without them (EXT 3 scans every run).
// The caller holds ks->mu through the launch and its use event (launch_batch).
#define W8_FLAG_STREAMS 8
static u32 *w8_flags_locked(ptls_mi355x_keyset_t *ks, hipStream_t s)
{
    auto &v = ks->w8flags;
    for (size_t i = 0; i < v.size(); ++i) {
        if (v[i].first == s) {
            std::rotate(v.begin() + i, v.begin() + i + 1, v.end());  // most recently used last
            return v.back().second;
        }
    }
    if (v.size() < W8_FLAG_STREAMS) {
        u32 *f = nullptr;
        if (hipMallocAsync((void **)&f, 4 * W8_FLAG_WORDS * (size_t)ks->ds->ncu, s) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        v.emplace_back(s, f);
        return f;
    }
    const hipStream_t prev = v.front().first;
    for (auto &u : ks->uses)
        if (u.first == prev && hipStreamWaitEvent(s, u.second, 0) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
    v.front().first = s;
    std::rotate(v.begin(), v.begin() + 1, v.end());
    return v.back().second;
}

// the keyset's spread scratch for a launch on `s` (allocated and zeroed in stream order on first use); nullptr on
// failure. The caller holds ks->mu from here through the launch and the use event recorded after it (launch_batch),
// so a launch on another stream always finds the previous user's event recorded.
static uint8_t *spread_scratch_locked(ptls_mi355x_keyset_t *ks, hipStream_t s, size_t nrecs)
{
    if (scratch_order_locked(ks, s) != 0)
        return nullptr;
    // sized for this batch's records (16 B x (CUs + 1025 pieces per record), 164 KiB for 10 records
    // instead of 4.2 MB for the largest batch), grown in stream order when a batch needs more
    const size_t bytes = spread_bytes(ks->ds->ncu, nrecs);
    if (ks->d_spread != nullptr && ks->spread_cap < bytes) {
        (void)hipFreeAsync(ks->d_spread, s);  // (ordered after its last user: scratch_order_locked)
        ks->d_spread = nullptr;
    }
    if (ks->d_spread == nullptr) {
        ks->spread_cap = 0;
        if (hipMallocAsync((void **)&ks->d_spread, bytes, s) != hipSuccess) {
            (void)hipGetLastError();
            ks->d_spread = nullptr;
            return nullptr;
        }
        if (hipMemsetAsync(ks->d_spread, 0, SPREAD_CNT_BYTES, s) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFreeAsync(ks->d_spread, s);
            ks->d_spread = nullptr;
            return nullptr;
        }
        ks->spread_cap = bytes;
    }
    return ks->d_spread;
}

// A batch call on a keyset: waits for the keyset's setup, groups an ungrouped many-key batch by key on the device, launches,
// and records the use (teardown and rekey are ordered after it).
static int launch_batch(ptls_mi355x_keyset_t *ks, bool open, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                        const void *aad, void *out, uint8_t *ok, void *stream, int frame = 0, const HpLaunch *hpl = nullptr)
{
    if (ks == NULL || (nrecs != 0 && (recs == NULL || in == NULL || out == NULL || (open && ok == NULL))))
        return fail("%s", "batch: invalid arguments");
    if (nrecs == 0)
        return 0;
    DeviceScope scope(ks->device);
    hipStream_t s = (hipStream_t)stream;
    if (wait_ready(ks, s) != 0)
        return -1;
    LAUNCH_CLEAR();  // (the grouping kernels and launch_gcm's launch are checked after this)
    // ungrouped many-key batches: group the records by key on the device first (see key_hist_kernel)
#ifndef KEY_GROUP_DISABLE
    const bool group = use_chunked(ks->schedule) && ks->nkeys > 1 && ks->nkeys <= KEY_GROUP_MAX_KEYS && nrecs > 1 &&
                       nrecs <= 0xffffffffu;
#else
    const bool group = false;
#endif
    int ret;
    // the keyset's scratch (spread pieces, key grouping) is shared by its launches on every stream: ks->mu is held from
    // taking it through the launch and the use event after it
    std::unique_lock<std::mutex> lk(ks->mu, std::defer_lock);
    // small batches with long records: the spread scratch
    uint8_t *spread = nullptr;
    u32 *w8flags = nullptr;
    if (hpl == nullptr && spread_eligible(ks, nrecs, frame)) {
        lk.lock();
        spread = spread_scratch_locked(ks, s, nrecs);
    } else if (hpl == nullptr && w8_eligible(ks, nrecs, frame)) {  // (a spread launch never takes the W8 pair)
        lk.lock();
        w8flags = w8_flags_locked(ks, s);
    }
    if (group) {
        if (!lk.owns_lock())
            lk.lock();
        // scratch: ctl[2] | counts[nkeys + 1] | perm[n] | (8-byte aligned) grouped descriptors[n] | balance tiles | bounds
        const bool balance = BALANCE && nrecs >= BALANCE_MIN_RECS;
        const size_t ntiles = (nrecs + BALANCE_TILE - 1) / BALANCE_TILE, ncu = (size_t)ks->ds->ncu;
        const size_t gwords = ((2 + ks->nkeys + 1 + nrecs + 1) & ~(size_t)1) + nrecs * (sizeof(ptls_mi355x_record_t) / 4);
        const size_t twords = balance ? (ntiles + 1) & ~(size_t)1 : 0, bwords = balance ? 2 * (ncu + 1) : 0;
        const size_t nb = ks->nkeys + 1, words = gwords + twords + bwords;
        if (ks->group_ev == NULL)
            HIP_TRY(hipEventCreateWithFlags(&ks->group_ev, hipEventDisableTiming));
        HIP_TRY(hipStreamWaitEvent(s, ks->group_ev, 0));  // a batch on another stream may still use the scratch
        if (words > ks->group_cap) {  // grown in stream order on this stream (no device-wide free)
            if (ks->d_group != NULL)
                HIP_TRY(hipFreeAsync(ks->d_group, s));
            ks->d_group = NULL;
            ks->group_cap = 0;
            HIP_TRY(hipMallocAsync((void **)&ks->d_group, words * 4, s));
            ks->group_cap = words;
        }
        u32 *ctl = ks->d_group, *cnt = ctl + 2, *perm = cnt + nb;
        HIP_TRY(hipMemsetAsync(ctl, 0, (2 + nb) * 4, s));
        const unsigned gh = (unsigned)min((nrecs + 255) / 256, (size_t)ks->ds->ncu * 8);
        key_changes_kernel<<<(unsigned)min((nrecs + 255) / 256, (size_t)ks->ds->ncu * KEY_CHANGES_WG_PER_CU), 256, 0, s>>>(recs, nrecs, ctl);
        key_hist_kernel<<<gh, 256, 0, s>>>(recs, nrecs, (u32)ks->nkeys, cnt, ctl);
        key_scan_kernel<<<1, 1024, 0, s>>>(cnt, (u32)nb, nrecs, ctl);
        ptls_mi355x_record_t *grouped = (ptls_mi355x_record_t *)(ctl + ((2 + nb + nrecs + 1) & ~(size_t)1));
        key_scatter_kernel<<<gh, 256, 0, s>>>(recs, nrecs, (u32)ks->nkeys, cnt, perm, grouped, ctl);
        u64 *bounds = nullptr;
        if (balance && use_chunked(ks->schedule)) {  // workgroup ranges of equal work (balance_bounds_kernel)
            u32 *tiles = ks->d_group + gwords;
            bounds = (u64 *)(ks->d_group + gwords + twords);
            const u32 grid = (u32)(ncu < nrecs ? ncu : nrecs);
            balance_tiles_kernel<<<(unsigned)min((ntiles + 3) / 4, ncu * 8), 256, 0, s>>>(recs, grouped, ctl + 1, nrecs, (u32)frame, tiles);
            balance_bounds_kernel<<<1, 1024, 0, s>>>(tiles, nrecs, grid, bounds);
        }
        ret = launch_gcm(ks->d_keys, (u32)ks->nkeys, ks->nr, ks->ds->ncu, ks->schedule, ks->ct, open, recs, nrecs, in, aad, out, ok, s,
                         frame, CHUNK_LOG2, grouped, perm, ctl + 1, nullptr, nullptr, bounds, hpl, spread, 0, w8flags);
        if (ret == 0)
            HIP_TRY(hipEventRecord(ks->group_ev, s));
    } else {
        ret = launch_gcm(ks->d_keys, (u32)ks->nkeys, ks->nr, ks->ds->ncu, ks->schedule, ks->ct, open, recs, nrecs, in, aad, out, ok,
                         s, frame, CHUNK_LOG2, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, hpl, spread, 0, w8flags);
    }
    // (a failed launch may have queued part of its work, e.g. EXT 4 of a W8 pair before its EXT 3 failed: the use is
    // recorded either way, so that a later takeover of this stream's flag buffer or a scratch regrow waits for it;
    // ADVICE round 4)
    const int noted = lk.owns_lock() ? note_use_locked(ks, s) : note_use(ks, s);
    return ret != 0 ? -1 : noted;
}

static unsigned aux_grid(size_t n, int ncu)
{
    u64 grid = (n + 255) / 256;
    return (unsigned)(grid > (u64)ncu * 4 ? (u64)ncu * 4 : grid);
}

static int launch_ecb(const KeyEntry *keys, u32 nkeys, int nr, int ncu, const uint32_t *key_idx, const void *in, void *out,
                      size_t nblocks, hipStream_t s)
{
    LAUNCH_CLEAR();
    if (nr == 10)
        ecb_kernel<10><<<aux_grid(nblocks, ncu), 256, LDS_AES_BYTES, s>>>(keys, nkeys, key_idx, (const uint8_t *)in, (uint8_t *)out,
                                                                          nblocks);
    else
        ecb_kernel<14><<<aux_grid(nblocks, ncu), 256, LDS_AES_BYTES, s>>>(keys, nkeys, key_idx, (const uint8_t *)in, (uint8_t *)out,
                                                                          nblocks);
    HIP_TRY(hipGetLastError());
    return 0;
}

static int launch_hp(const KeyEntry *keys, u32 nkeys, int nr, int ncu, const ptls_mi355x_hp_t *hp, size_t n, const void *base,
                     void *masks, hipStream_t s, u32 *done_flag = nullptr, u32 done_token = 0)
{
    LAUNCH_CLEAR();
    if (nr == 10)
        hp_kernel<10><<<aux_grid(n, ncu), 256, LDS_AES_BYTES, s>>>(keys, nkeys, hp, (const uint8_t *)base, (uint8_t *)masks, n, done_flag,
                                                                    done_token);
    else
        hp_kernel<14><<<aux_grid(n, ncu), 256, LDS_AES_BYTES, s>>>(keys, nkeys, hp, (const uint8_t *)base, (uint8_t *)masks, n, done_flag,
                                                                    done_token);
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" {

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
    DeviceScope scope(ks->device);
    hipStream_t s = (hipStream_t)stream;
    if (wait_ready(ks, s) != 0 || launch_ecb(ks->d_keys, (u32)ks->nkeys, ks->nr, ks->ds->ncu, key_idx, in, out, nblocks, s) != 0)
        return -1;
    return note_use(ks, s);
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
    DeviceScope scope(ks->device);
    LAUNCH_CLEAR();
    tls_unpad_kernel<<<aux_grid(nrecs, ks->ds->ncu), 256, 0, (hipStream_t)stream>>>(recs, nrecs, (const uint8_t *)in,
                                                                                     (const uint8_t *)out, ok, results);
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
    DeviceScope scope(ks->device);
    LAUNCH_CLEAR();
    tls12_check_kernel<<<aux_grid(nrecs, ks->ds->ncu), 256, 0, (hipStream_t)stream>>>(recs, nrecs, (const uint8_t *)in, ok,
                                                                                       results);
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
    DeviceScope scope(hp_ks->device);
    hipStream_t s = (hipStream_t)stream;
    if (wait_ready(hp_ks, s) != 0 || launch_hp(hp_ks->d_keys, (u32)hp_ks->nkeys, hp_ks->nr, hp_ks->ds->ncu, hp, n, base, masks, s) != 0)
        return -1;
    return note_use(hp_ks, s);
}

int ptls_mi355x_seal_batch_hp(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                              const void *aad, void *out, ptls_mi355x_keyset_t *hp_ks, const ptls_mi355x_hp_t *hp,
                              void *masks, void *stream)
{
    if (ks == NULL || hp_ks == NULL || (nrecs != 0 && (hp == NULL || masks == NULL)))
        return fail("%s", "seal_batch_hp: invalid arguments");
    if (hp_ks->device != ks->device)
        return fail("%s", "seal_batch_hp: the keysets are on different devices");
    if (nrecs == 0)
        return 0;
    if (!ks->ct && !use_chunked(ks->schedule)) {  // the lockstep schedule: the seal, then the masks (a second launch)
        if (launch_batch(ks, false, recs, nrecs, in, aad, out, NULL, stream) != 0)
            return -1;
        return ptls_mi355x_hp_mask_batch(hp_ks, hp, nrecs, out, masks, stream);
    }
    // one launch: the chunked seal computes each run's masks after sealing it (hp_masks_pass)
    DeviceScope scope(ks->device);
    if (wait_ready(hp_ks, (hipStream_t)stream) != 0)
        return -1;
    const HpLaunch hpl = {hp, hp_ks->d_keys, (u32)hp_ks->nkeys, hp_ks->nr, (uint8_t *)masks};
    if (launch_batch(ks, false, recs, nrecs, in, aad, out, NULL, stream, 0, &hpl) != 0)
        return -1;
    return note_use(hp_ks, (hipStream_t)stream);
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
    DeviceScope scope(ks->device);
    hipStream_t s = (hipStream_t)stream;
    if (wait_ready(ks, s) != 0)
        return -1;
    LAUNCH_CLEAR();
    quiclb_kernel<10><<<aux_grid(n, ks->ds->ncu), 256, LDS_AES_BYTES, s>>>(ks->d_keys, (u32)ks->nkeys, cids, (const uint8_t *)in,
                                                                            (uint8_t *)out, n);
    HIP_TRY(hipGetLastError());
    return note_use(ks, s);
}

}  // extern "C"

#ifndef PERREC_FLAG
#define PERREC_FLAG 1                       // a lone record's launch publishes a completion word the host polls (roundtrip)
#endif
#define PERREC_FLAG_SPIN_US 2000  // + 0.5 us per staged KiB: long records (the span path) poll to their end too
#ifndef SPAN_MIN_BYTES
#define SPAN_MIN_BYTES ((size_t)262144)  // a lone record from this length runs over many workgroups (launch_span)
#endif
#define PERREC_FLAG_MAX_BYTES ((size_t)1 << 20)  // staged bytes of a call that polls (larger ones wait for the stream)
#ifndef CT_UNIT_SHIFT
#define CT_UNIT_SHIFT 0  // per-record launches of a constant-time keyset: unit length x 2^CT_UNIT_SHIFT
#endif
#ifndef PERREC_HP_FUSED
#define PERREC_HP_FUSED 1  // encrypt_s: the header-protection mask computed by the seal launch (BatchArgs::hp)
#endif

// PTLS_MI355X_COMBINE_STATS=1: per-record launches, calls and the host time of run_calls, printed at exit (tools/gpu_mt.sh)
static struct CombineStats {
    std::atomic<uint64_t> launches{0}, calls{0}, ns{0}, wait_ns{0};
    bool on = getenv("PTLS_MI355X_COMBINE_STATS") != nullptr;
    ~CombineStats()
    {
        if (on && launches.load() != 0)
            fprintf(stderr, "combine stats: %llu launches, %llu calls (%.2f per launch), %.1f us per launch in run_calls, %.1f us of it waiting\n",
                    (unsigned long long)launches.load(), (unsigned long long)calls.load(), (double)calls.load() / (double)launches.load(),
                    (double)ns.load() / 1e3 / (double)launches.load(), (double)wait_ns.load() / 1e3 / (double)launches.load());
    }
} g_cstats;

// ---- the synchronous host-buffer helpers (the per-record picotls path)
//
// One call = a staging buffer and its stream from the device pool, a host copy of the inputs into it, launches whose
// kernels read and write the pinned buffer in place over PCIe (or, where it cannot be mapped, an H2D copy before and a
// D2H copy after), a wait for that stream only, a host copy of the results, and the staged bytes cleared.
// Measured against copying (tools/latency.py, interleaved): 16 B 29 -> 26 us, 1200 B 31 -> 29, 16 KiB 52 -> 38,
// 4 MiB 1.70 -> 1.58 ms.
struct StageCall {
    DeviceState *ds;
    Stager *st = nullptr;
    size_t total = 0;
    size_t clear_lo = 0, clear_hi = SIZE_MAX;  // the staged bytes that held plaintext (all unless narrowed)
    StageCall(DeviceState *d) : ds(d) {}
    ~StageCall()
    {
        if (st != nullptr) {
            // staged plaintext does not outlive the call (with it gone, the ciphertext beside it reveals nothing)
            const size_t hi = clear_hi < total ? clear_hi : total;
            if (hi > clear_lo)
                memset(st->h + clear_lo, 0, hi - clear_lo);
            stager_put(ds, st);
        }
    }
    int acquire(size_t bytes)
    {
        total = bytes;
        return (st = stager_get(ds, bytes)) != nullptr ? 0 : -1;
    }
    uint8_t *host() const { return st->h; }
    uint8_t *dev() const { return st->h_dev != nullptr ? st->h_dev : st->d; }
    hipStream_t stream() const { return st->stream; }
    // runs launch() on the staged buffer: H2D of [0, up) before and D2H of [up, total) after on the copy path; then waits
    // flag_off (mapped staging only, 0: none): nflags words, one per workgroup of the launch's last kernel, that it sets
    // once its results are written (BatchArgs::done_flag); the call returns when it sees them all, without the
    // stream's completion signal (the next user of this stager's stream is ordered after the kernel anyway). After
    // PERREC_FLAG_SPIN_US (+ 0.5 us per staged KiB) without them (a launch queued behind others) the call waits for the
    // stream as usual.
    bool mapped() const { return st->h_dev != nullptr; }
    template <typename Launch>
    int roundtrip(size_t up, Launch launch, size_t flag_off = 0, size_t nflags = 0, u32 token = 0)
    {
        const bool copy = st->h_dev == nullptr;
        if (copy)
            HIP_TRY(hipMemcpyAsync(st->d, st->h, up, hipMemcpyHostToDevice, st->stream));
        LAUNCH_CLEAR();  // (the launches below are checked with hipGetLastError)
        if (launch() != 0) {
            // a kernel of this call may already be queued (the span launch before its combine, the GCM launch before
            // the header-protection one): the buffer is cleared and reused only once nothing of it is in flight
            (void)hipStreamSynchronize(st->stream);
            return -1;
        }
        if (copy)
            HIP_TRY(hipMemcpyAsync(st->h + up, st->d + up, total - up, hipMemcpyDeviceToHost, st->stream));
        const auto t0 = std::chrono::steady_clock::now();
        if (flag_off != 0 && token != 0 && !copy) {
            const u32 *flag = (const u32 *)(st->h + flag_off);
            size_t seen = 0;  // flags [0, seen) are set
            for (unsigned k = 0;; ++k) {
                while (seen < nflags && __atomic_load_n(flag + seen, __ATOMIC_ACQUIRE) == token)
                    ++seen;
                if (seen == nflags) {
                    if (g_cstats.on)
                        g_cstats.wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
                    return 0;
                }
                __builtin_ia32_pause();
                if ((k & 255) == 255 &&
                    std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(PERREC_FLAG_SPIN_US + (int64_t)(total >> 11)))
                    break;
            }
        }
        HIP_TRY(hipStreamSynchronize(st->stream));
        if (g_cstats.on)
            g_cstats.wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        return 0;
    }
};

// completion tokens of per-record calls (StageCall::roundtrip): process-wide, nonzero, and consecutive calls on one
// staging buffer never share one
static std::atomic<u32> g_done_token{0};
static u32 next_done_token(void)
{
    u32 t;
    while ((t = g_done_token.fetch_add(1, std::memory_order_relaxed) + 1) == 0) {
    }
    return t;
}

// after a synchronous call on `ks` completed on a stager stream, its setup is complete too
static void seen_ready(ptls_mi355x_keyset_t *ks) { ks->ready_seen.store(true, std::memory_order_release); }

// ---- per-record calls, combined across threads
//
// picotls' per-record calls are synchronous, so one thread's records can never share a launch -- but the calls of
// several threads can. A call of a one-key keyset (a picotls context) goes to its device's combiner for its kind (seal
// or open, AES-128 or -256, constant-time or not, header-protection key size): when fewer than `combine` launches of
// that kind are in flight it takes every queued call, itself included, into one batch (flat combining); otherwise it
// queues and waits until a batch that took it completes, or until a launch slot frees and it can take the queue
// itself. A lone caller thus launches at once, as before, while N threads calling together share launches instead of
// queueing theirs on the device's few hardware queues (tools/mt_records.py). The entries of one-key keysets live in
// per-device slabs, so a combined batch addresses them as key indices from the lowest entry of the batch.
// PTLS_MI355X_COMBINE=k turns it on with k launches in flight per kind (default 0: every call on its own). Measured
// (tools/mt_records.c, 1200-byte seals): while a call waited for its stream's completion signal, 16 threads made 222K
// calls/s on their own and 264-269K combined (2.7 calls a launch). Once calls poll their completion words (roundtrip)
// a lone call is cheaper than a share of a batch: 16 threads 302K calls/s on their own against 249K combined (16 B:
// 352K / 270K; 16 KiB: 179K / 189K), so combining is off by default
// (profiles/r2_per_record/final_mt_and_skew.txt).

struct OneCall {
    ptls_mi355x_keyset_t *ks;
    size_t key_idx;
    bool open;
    void *output;
    const ptls_mi355x_iovec_t *vec;
    size_t incnt, len;
    uint64_t seq;
    const void *aad;
    size_t aadlen;
    int *verified;
    ptls_mi355x_keyset_t *hp_ks;  // header-protection mask of the sealed output's sample (fusion's supp) when set
    size_t hp_key_idx, sample_off;
    void *mask;
    int ret = -1;
    char err[sizeof(g_err)] = {};
    std::atomic<bool> done{false};
    const KeyEntry *entry() const { return ks->d_keys + key_idx; }
    const KeyEntry *hp_entry() const { return hp_ks->d_keys + hp_key_idx; }
};

#define COMBINE_MAX_CALLS 256               // calls per combined launch
#define COMBINE_MAX_BYTES ((size_t)65536)   // larger records and AADs run on their own
#ifndef COMBINE_WAIT_US
#define COMBINE_WAIT_US 5                   // how long a call that could lead waits for the rest of the last batch's callers
#endif


// Runs the calls `c[0..n)` (all of one kind) as one batch through one staging buffer and sets each call's ret (and
// err), then its done flag. Staging layout: [descriptors | hp entries | every call's input and AAD] is read by the
// device, [every call's output | ok bytes | masks] written (the copy path moves the first part up, the second down).
static void run_calls(DeviceState *ds, OneCall *const *c, size_t n)
{
    const auto t_start = std::chrono::steady_clock::now();
    const OneCall &c0 = *c[0];
    const bool open = c0.open, hp = c0.hp_ks != nullptr;
    const int nr = c0.ks->nr, hp_nr = hp ? c0.hp_ks->nr : 0;
    auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    // the key indices of the batch: entries from the lowest one of the batch (all of them one-key slab entries when
    // n > 1; a lone call uses its own keyset's entries as they are)
    const KeyEntry *kbase = c0.entry(), *hbase = hp ? c0.hp_entry() : nullptr;
    for (size_t i = 1; i < n; ++i) {
        kbase = c[i]->entry() < kbase ? c[i]->entry() : kbase;
        if (hp)
            hbase = c[i]->hp_entry() < hbase ? c[i]->hp_entry() : hbase;
    }
    const size_t off_rec = 0, off_hp = a16(n * sizeof(ptls_mi355x_record_t)), off_data = off_hp + a16(n * sizeof(ptls_mi355x_hp_t));
    size_t up = off_data;
    for (size_t i = 0; i < n; ++i)
        up += a16(c[i]->len + (open ? 16 : 0)) + a16(c[i]->aadlen);
    size_t off_ok = up;
    for (size_t i = 0; i < n; ++i)
        off_ok += a16(c[i]->len + (open ? 0 : 16));
    // a lone long record runs over many workgroups (launch_span): 16-step units in spans of 2^e, at most one span per CU
    u32 span_units = 0, span_e = 0, span_n = 0;
    if (SPAN_MIN_BYTES != 0 && n == 1 && c0.len >= SPAN_MIN_BYTES && c0.ks->schedule != PTLS_MI355X_SCHEDULE_LOCKSTEP) {
        const size_t steps = ((c0.aadlen + 15) / 16 + (c0.len + 15) / 16 + 1 + ENGINE_G - 1) / ENGINE_G;
        span_units = (u32)((steps + CHUNK_STEPS - 1) / CHUNK_STEPS);
        const u32 cap = ds->ncu < 256 ? (u32)ds->ncu : 256u;
        while (((span_units + (1u << span_e) - 1) >> span_e) > cap)
            ++span_e;
        span_n = (span_units + (1u << span_e) - 1) >> span_e;
        if ((1u << span_e) > SPAN_MAX_UNITS)
            span_units = span_e = span_n = 0;
    }
    // header-protection masks: computed by the chunked seal launch itself (PERREC_HP_FUSED), else by a second launch
    // (hp_kernel) after the seal, or after the span kernels
    const bool hp_fused = hp && PERREC_HP_FUSED && span_n == 0 && (c0.ks->ct || use_chunked(c0.ks->schedule));
    // completion words: one per workgroup of the last kernel (the GCM launch: one workgroup per record up to the CU
    // count; the header-protection launch: aux_grid)
    const size_t nflags = hp && !hp_fused ? (size_t)aux_grid(n, ds->ncu) : (n < (size_t)ds->ncu ? n : (size_t)ds->ncu);
    const size_t off_mask = off_ok + a16(n), off_flag = off_mask + 16 * n, off_span = off_flag + a16(4 * nflags),
                 total = off_span + 16 * (size_t)span_n;
    int ret = -1;
    {
        StageCall call(ds);
        // the plaintext side: a seal's inputs (up), an open's outputs (down); the copy path's device buffer is not cleared
        if (open)
            call.clear_lo = up;
        else
            call.clear_hi = up;
        if (call.acquire(total) == 0) {
            uint8_t *h = call.host(), *d = call.dev();
            const hipStream_t s = call.stream();
            u32 nkeys = 1, hp_nkeys = 1;
            size_t in_at = off_data, out_at = up;
            ptls_mi355x_record_t first = {};
            ret = 0;
            for (size_t i = 0; i < n && ret == 0; ++i) {
                const OneCall &x = *c[i];
                const size_t kd = (size_t)(x.entry() - kbase);
                const size_t inbytes = x.len + (open ? 16 : 0);
                for (size_t v = 0, off = 0; v < x.incnt; off += x.vec[v].len, ++v)
                    if (x.vec[v].len != 0)
                        memcpy(h + in_at + off, x.vec[v].base, x.vec[v].len);
                const size_t aad_at = in_at + a16(inbytes);
                if (x.aadlen != 0)
                    memcpy(h + aad_at, x.aad, x.aadlen);
                const ptls_mi355x_record_t r = {in_at, out_at, x.seq, (u32)aad_at, (u32)x.len, (u32)kd, (uint16_t)x.aadlen,
                                                (uint16_t)(x.aadlen >> 16)};
                memcpy(h + off_rec + i * sizeof(r), &r, sizeof(r));
                if (i == 0)
                    first = r;
                nkeys = (u32)kd + 1 > nkeys ? (u32)kd + 1 : nkeys;
                if (hp) {
                    const size_t hd = (size_t)(x.hp_entry() - hbase);
                    const ptls_mi355x_hp_t e = {out_at + x.sample_off, (u32)hd, 0};
                    memcpy(h + off_hp + i * sizeof(e), &e, sizeof(e));
                    hp_nkeys = (u32)hd + 1 > hp_nkeys ? (u32)hd + 1 : hp_nkeys;
                }
                in_at = aad_at + a16(x.aadlen);
                out_at += a16(x.len + (open ? 0 : 16));
                if (wait_ready(x.ks, s) != 0 || (hp && wait_ready(x.hp_ks, s) != 0))
                    ret = -1;
            }
            // one record on one workgroup: shorter units put more of its waves to work (a unit step costs a lone
            // wave ~2 us of latency, a unit combine ~0.15 us); steps / 2^k units balance the two (tools/latency.py).
            // Long records, and batches (one workgroup per record), pass CHUNK_LOG2: the kernel's scan then picks.
            const size_t steps = ((c0.aadlen + 15) / 16 + (c0.len + 15) / 16 + 1 + ENGINE_G - 1) / ENGINE_G;
            // (the constant-time variant: units CT_UNIT_SHIFT times longer, whose ends cost it 4 GHASH multiplies and
            // whose combine links a whole gmul_tab each)
            const u32 ushift = c0.ks->ct ? CT_UNIT_SHIFT : 0u;
            u32 unit_log2 = n > 1 ? CHUNK_LOG2 : steps <= 24 ? 0 : steps <= 96 ? 1 : steps <= 400 ? 2 : steps <= 1600 ? 3 : CHUNK_LOG2;
            if (n == 1)
                unit_log2 = unit_log2 + ushift < CHUNK_LOG2 ? unit_log2 + ushift : CHUNK_LOG2;
            // (calls staging at most 1 MiB: a larger record's launch runs for hundreds of microseconds or more, which
            // the caller need not spend spinning on a core)
            const bool flag = PERREC_FLAG && call.mapped() && c0.ks->schedule != PTLS_MI355X_SCHEDULE_LOCKSTEP &&
                              (total <= PERREC_FLAG_MAX_BYTES || span_n != 0);
            // this call's completion token (never 0, and never the value an earlier call left in these words)
            const u32 token = flag ? next_done_token() : 0u;
            if (flag)
                memset(h + off_flag, 0, 4 * nflags);
            if (ret == 0)
                ret = call.roundtrip(up, [&] {
                    if (span_n != 0) {
                        if (launch_span(kbase, nr, c0.ks->ct, open, first, d, d, d, d + off_ok, span_units, span_e, span_n, d + off_span,
                                        flag && !hp ? (u32 *)(d + off_flag) : nullptr, token, s) != 0)
                            return -1;
                    } else {
                        const HpLaunch hpl = {(const ptls_mi355x_hp_t *)(d + off_hp), hbase, hp_nkeys, hp_nr, d + off_mask};
                        if (launch_gcm(kbase, nkeys, nr, ds->ncu, c0.ks->schedule, c0.ks->ct, open, (const ptls_mi355x_record_t *)(d + off_rec),
                                       n, d, d, d, d + off_ok, s, 0, unit_log2, nullptr, nullptr, nullptr, n == 1 ? &first : nullptr,
                                       flag && (!hp || hp_fused) ? (u32 *)(d + off_flag) : nullptr, nullptr, hp_fused ? &hpl : nullptr,
                                       nullptr, token) != 0)
                            return -1;
                    }
                    return !hp || hp_fused ? 0
                               : launch_hp(hbase, hp_nkeys, hp_nr, ds->ncu, (const ptls_mi355x_hp_t *)(d + off_hp), n, d, d + off_mask, s,
                                           flag ? (u32 *)(d + off_flag) : nullptr, token);
                }, flag ? off_flag : 0, nflags, token);
            if (ret == 0) {
                out_at = up;
                for (size_t i = 0; i < n; ++i) {
                    OneCall &x = *c[i];
                    seen_ready(x.ks);
                    if (hp)
                        seen_ready(x.hp_ks);
                    const size_t outbytes = x.len + (open ? 0 : 16);
                    if (outbytes != 0)
                        memcpy(x.output, h + out_at, outbytes);
                    if (open)
                        *x.verified = h[off_ok + i];
                    if (hp)
                        memcpy(x.mask, h + off_mask + 16 * i, 16);
                    out_at += a16(outbytes);
                }
                if (ds->diag && flag && call.mapped()) {
                    // (diagnosis: did any result byte change after the completion words were seen?)
                    (void)hipStreamSynchronize(s);
                    size_t at = up;
                    for (size_t i = 0; i < n; ++i) {
                        const OneCall &x = *c[i];
                        const size_t outbytes = x.len + (open ? 0 : 16);
                        size_t diff = 0, first = SIZE_MAX;
                        for (size_t b = 0; b < outbytes; ++b)
                            if (h[at + b] != ((const uint8_t *)x.output)[b])
                                diff++, first = first == SIZE_MAX ? b : first;
                        const bool okchg = open && h[off_ok + i] != (uint8_t)*x.verified;
                        if (diff != 0 || okchg)
                            fprintf(stderr, "ptls_mi355x diag: %s of %zu bytes: %zu result bytes (first at %zu)%s changed after the "
                                            "completion words were seen\n", open ? "open" : "seal", x.len, diff,
                                    first == SIZE_MAX ? (size_t)0 : first, okchg ? " and the ok byte" : "");
                        at += a16(outbytes);
                    }
                }
            }
        }
    }
    if (g_cstats.on) {
        g_cstats.launches += 1, g_cstats.calls += n;
        g_cstats.ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_start).count();
    }
    for (size_t i = 0; i < n; ++i) {
        c[i]->ret = ret;
        if (ret != 0)
            memcpy(c[i]->err, g_err, sizeof(g_err));
        c[i]->done.store(true, std::memory_order_release);
    }
}

// the combiner of a call's kind (index into DeviceState::comb), or -1 when the call runs on its own
static int combine_kind(const OneCall &c)
{
    if (!c.ks->slot || c.ks->schedule == PTLS_MI355X_SCHEDULE_LOCKSTEP || c.len > COMBINE_MAX_BYTES || c.aadlen > COMBINE_MAX_BYTES ||
        (c.hp_ks != nullptr && !c.hp_ks->slot))
        return -1;
    return (c.open ? 1 : 0) | (c.ks->nr == 14 ? 2 : 0) | (c.ks->ct ? 4 : 0) | (c.hp_ks == nullptr ? 0 : c.hp_ks->nr == 14 ? 16 : 8);
}

static int submit(DeviceState *ds, OneCall *c)
{
    const int kind = ds->combine > 0 ? combine_kind(*c) : -1;
    if (kind < 0) {
        run_calls(ds, &c, 1);
    } else {
        Combiner &cb = ds->comb[kind];
        std::vector<OneCall *> batch;
        const auto t_enq = std::chrono::steady_clock::now();
        std::unique_lock<std::mutex> lk(cb.mu);
        cb.q.push_back(c);
        while (!c->done.load(std::memory_order_acquire)) {
            // a launch slot is free: take the queue -- unless fewer calls have queued than the last batch held and this
            // call has waited less than COMBINE_WAIT_US: threads whose calls just completed are about to submit their
            // next ones, and a batch taken at once would hold only the first of them (a lone caller never waits)
            if (cb.inflight < ds->combine && !cb.q.empty() &&
                (cb.q.size() >= cb.expect ||
                 std::chrono::steady_clock::now() - t_enq >= std::chrono::microseconds(COMBINE_WAIT_US))) {
                // as many queued calls as fit one staging buffer (each call's share is about its bytes up and down)
                size_t take = 0, bytes = 0;
                while (take < cb.q.size() && take < COMBINE_MAX_CALLS) {
                    const OneCall &x = *cb.q[take];
                    bytes += 2 * x.len + x.aadlen + 128;
                    if (take > 0 && bytes > ds->stage_limit / 2)
                        break;
                    ++take;
                }
                batch.assign(cb.q.begin(), cb.q.begin() + (long)take);
                cb.q.erase(cb.q.begin(), cb.q.begin() + (long)take);
                ++cb.inflight;
                cb.expect = take;
                lk.unlock();
                // a batch's calls address their entries as key indices from its lowest entry, which is defined only
                // within one slab (slabs are separate allocations): calls whose entries lie in several slabs run one
                // by one
                auto one_slab = [&](bool hp_entries) {
                    const KeyEntry *slab = hp_entries ? batch[0]->hp_ks->slab : batch[0]->ks->slab;
                    for (OneCall *x : batch)
                        if ((hp_entries ? x->hp_ks->slab : x->ks->slab) != slab)
                            return false;
                    return true;
                };
                if (batch.size() == 1 || (one_slab(false) && (batch[0]->hp_ks == nullptr || one_slab(true)))) {
                    run_calls(ds, batch.data(), batch.size());
                } else {
                    for (OneCall *x : batch)
                        run_calls(ds, &x, 1);
                }
                lk.lock();
                --cb.inflight;
                continue;
            }
            lk.unlock();
            for (int k = 0; k < 256 && !c->done.load(std::memory_order_acquire); ++k)
                __builtin_ia32_pause();
            if (!c->done.load(std::memory_order_acquire))
                sched_yield();
            lk.lock();
        }
    }
    if (c->ret != 0)
        return fail("%s", c->err);
    return 0;
}

// one record on host buffers (input as iovecs), optionally with the header-protection mask of a sample of the sealed
// output under hp_ks (fusion's supp, lib/fusion.c:425-430,636-651): a batch of one through a staging buffer, or a
// share of a batch combined with other threads' calls (submit)
static int single(ptls_mi355x_keyset_t *ks, size_t key_idx, bool open, void *output, const ptls_mi355x_iovec_t *vec, size_t incnt,
                  size_t len, uint64_t seq, const void *aad, size_t aadlen, int *verified, ptls_mi355x_keyset_t *hp_ks = NULL,
                  size_t hp_key_idx = 0, size_t sample_off = 0, void *mask = NULL)
{
    if (ks == NULL || key_idx >= ks->nkeys || (aadlen != 0 && aad == NULL) || (len != 0 && output == NULL))
        return fail("%s", "single: invalid arguments");
    if (len > PTLS_MI355X_MAX_RECORD_LEN || aadlen > PTLS_MI355X_MAX_AAD_LEN)
        return fail("%s", "single: record or AAD longer than PTLS_MI355X_MAX_RECORD_LEN / PTLS_MI355X_MAX_AAD_LEN");
    if (hp_ks != NULL && (hp_key_idx >= hp_ks->nkeys || hp_ks->device != ks->device || sample_off > len))
        return fail("%s", "single: invalid header-protection arguments");
    DeviceScope scope(ks->device);
    OneCall c;
    c.ks = ks, c.key_idx = key_idx, c.open = open, c.output = output, c.vec = vec, c.incnt = incnt, c.len = len, c.seq = seq;
    c.aad = aad, c.aadlen = aadlen, c.verified = verified, c.hp_ks = hp_ks, c.hp_key_idx = hp_key_idx;
    c.sample_off = sample_off, c.mask = mask;
    return submit(ks->ds, &c);
}

extern "C" {

int ptls_mi355x_encrypt(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                        const void *aad, size_t aadlen)
{
    const ptls_mi355x_iovec_t v = {input, inlen};
    return single(ks, key_idx, false, output, &v, 1, inlen, seq, aad, aadlen, NULL);
}

int ptls_mi355x_encrypt_v(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const ptls_mi355x_iovec_t *input, size_t incnt,
                          uint64_t seq, const void *aad, size_t aadlen)
{
    size_t len = 0;
    for (size_t i = 0; i < incnt; ++i) {
        if (input[i].len != 0 && input[i].base == NULL)
            return fail("%s", "encrypt_v: invalid iovec");
        len += input[i].len;
    }
    return single(ks, key_idx, false, output, input, incnt, len, seq, aad, aadlen, NULL);
}

int ptls_mi355x_encrypt_s(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                          const void *aad, size_t aadlen, ptls_mi355x_keyset_t *hp_ks, size_t hp_key_idx, size_t sample_off,
                          void *mask)
{
    if (hp_ks == NULL || mask == NULL)
        return fail("%s", "encrypt_s: invalid arguments");
    const ptls_mi355x_iovec_t v = {input, inlen};
    return single(ks, key_idx, false, output, &v, 1, inlen, seq, aad, aadlen, NULL, hp_ks, hp_key_idx, sample_off, mask);
}

size_t ptls_mi355x_decrypt(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                           const void *aad, size_t aadlen)
{
    if (inlen < 16)
        return SIZE_MAX;
    int verified = 0;
    const ptls_mi355x_iovec_t v = {input, inlen};
    if (single(ks, key_idx, true, output, &v, 1, inlen - 16, seq, aad, aadlen, &verified) != 0)
        return SIZE_MAX;
    return verified ? inlen - 16 : SIZE_MAX;
}

int ptls_mi355x_quiclb_transform(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t len, int encrypt)
{
    if (ks == NULL || key_idx >= ks->nkeys || output == NULL || input == NULL || len < PTLS_MI355X_QUICLB_MIN_LEN ||
        len > PTLS_MI355X_QUICLB_MAX_LEN || ks->key_size != 16)
        return fail("%s", "quiclb_transform: invalid arguments");
    DeviceScope scope(ks->device);
    StageCall call(ks->ds);
    // staging: [0, 32) CID in, [32, 56) descriptor | [64, 96) CID out
    if (call.acquire(96) != 0)
        return -1;
    const ptls_mi355x_cid_t c = {0, 64, 0, (uint8_t)len, (uint8_t)(encrypt != 0), 0};
    memcpy(call.host(), input, len);
    memcpy(call.host() + 32, &c, sizeof(c));
    uint8_t *d = call.dev();
    const hipStream_t s = call.stream();
    if (wait_ready(ks, s) != 0 || call.roundtrip(64, [&] {
            quiclb_kernel<10><<<1, 256, LDS_AES_BYTES, s>>>(ks->d_keys + key_idx, 1, (const ptls_mi355x_cid_t *)(d + 32), d, d, 1);
            HIP_TRY(hipGetLastError());
            return 0;
        }) != 0)
        return -1;
    seen_ready(ks);
    memcpy(output, call.host() + 64, len);
    return 0;
}

int ptls_mi355x_encrypt_blocks(ptls_mi355x_keyset_t *ks, size_t key_idx, void *out, const void *in, size_t nblocks)
{
    if (ks == NULL || key_idx >= ks->nkeys || (nblocks != 0 && (out == NULL || in == NULL)) || nblocks > ((size_t)1 << 26))
        return fail("%s", "encrypt_blocks: invalid arguments");
    if (nblocks == 0)
        return 0;
    DeviceScope scope(ks->device);
    StageCall call(ks->ds);
    // staging: [0, n) blocks in | [n', n' + n) blocks out, n' = n rounded up to 32 bytes
    const size_t n = nblocks * 16, up = (n + 31) & ~(size_t)31;
    if (call.acquire(2 * up) != 0)
        return -1;
    memcpy(call.host(), in, n);
    uint8_t *d = call.dev();
    const hipStream_t s = call.stream();
    if (wait_ready(ks, s) != 0 ||
        call.roundtrip(up, [&] { return launch_ecb(ks->d_keys + key_idx, 1, ks->nr, ks->ds->ncu, NULL, d, d + up, nblocks, s); }) != 0)
        return -1;
    seen_ready(ks);
    memcpy(out, call.host() + up, n);
    return 0;
}

int ptls_mi355x_encrypt_block(ptls_mi355x_keyset_t *ks, size_t key_idx, void *out, const void *in)
{
    if (ks == NULL || key_idx >= ks->nkeys || out == NULL || in == NULL)
        return fail("%s", "encrypt_block: invalid arguments");
    return ptls_mi355x_encrypt_blocks(ks, key_idx, out, in, 1);
}

}  // extern "C"
