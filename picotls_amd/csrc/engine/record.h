// picotls_amd/csrc/engine/record.h -- Byte-exact record I/O, the batch arguments, TLS framing rules.
// Part of the single translation unit picotls_amd/csrc/aesgcm_engine.hip (included in order; not standalone).
#ifndef PTLS_MI355X_ENGINE_RECORD_H
#define PTLS_MI355X_ENGINE_RECORD_H

// ------------------------------------------------------------------------------------------------ byte-exact I/O

// zero bytes n..15
__device__ __forceinline__ u32x4 mask_tail(u32x4 v, u32 n)
{
    u32x4 r;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        int nb = (int)n - 4 * c;
        u32 m = nb >= 4 ? 0xffffffffu : nb <= 0 ? 0u : (0xffffffffu >> (32 - 8 * nb));
        r[c] = v[c] & m;
    }
    return r;
}

// loads n (< 16) bytes, zero padded. As fusion's loadn128 (lib/fusion.c:355-368): when the 16 bytes at p stay inside
// p's 4 KiB page (which holds valid data, so it is mapped) one unaligned 16-byte load plus a mask replaces n byte loads;
// only a tail within 15 bytes of a page end is read byte by byte. Bytes past n are never used. n = 0 reads nothing (p
// may then be one past the end of a buffer).
__device__ __forceinline__ u32x4 load_partial(const uint8_t *p, u32 n)
{
    if (n != 0 && ((uintptr_t)p & 4095u) <= 4096u - 16u)
        return mask_tail(*(const u32x4_u *)p, n);
    u32x4 v = {0, 0, 0, 0};
#pragma unroll
    for (u32 i = 0; i < 15; ++i)
        if (i < n)
            v[i >> 2] |= (u32)p[i] << (8 * (i & 3));
    return v;
}

// load_partial without the mask, for a load issued ahead of its use: bytes n..15 are unspecified until mask_tail (so
// the wait for the load can sit after the work issued behind it)
__device__ __forceinline__ u32x4 load_partial_raw(const uint8_t *p, u32 n)
{
    if (n != 0 && ((uintptr_t)p & 4095u) <= 4096u - 16u)
        return *(const u32x4_u *)p;
    u32x4 v = {0, 0, 0, 0};
#pragma unroll
    for (u32 i = 0; i < 15; ++i)
        if (i < n)
            v[i >> 2] |= (u32)p[i] << (8 * (i & 3));
    return v;
}

// stores bytes 0..n-1 of v (n < 16): (round 6, STORE_PARTIAL_BITS) an 8-, 4-, 2- and 1-byte store by the bits of n,
// each from the low end of the bytes left, instead of n byte stores (a wave looped max n times over its lanes)
typedef unsigned long long __attribute__((aligned(1))) u64_u;
typedef unsigned short __attribute__((aligned(1))) u16_u;
#ifndef STORE_PARTIAL_BITS
#define STORE_PARTIAL_BITS 1
#endif
__device__ __forceinline__ void store_partial(uint8_t *p, u32x4 v, u32 n)
{
    if constexpr (STORE_PARTIAL_BITS) {
        u32 a = v[0], b = v[1];
        if (n & 8) {
            *(u64_u *)p = (unsigned long long)b << 32 | a;
            p += 8, a = v[2], b = v[3];
        }
        if (n & 4) {
            *(u32_u *)p = a;
            p += 4, a = b;
        }
        if (n & 2) {
            *(u16_u *)p = (unsigned short)a;
            p += 2, a >>= 16;
        }
        if (n & 1)
            *p = (uint8_t)a;
    } else {
        for (u32 i = 0; i < n; ++i)
            p[i] = (uint8_t)(v[i >> 2] >> (8 * (i & 3)));
    }
}

// ------------------------------------------------------------------------------------------------ main kernel

struct BatchArgs {
    const KeyEntry *keys;
    const ptls_mi355x_record_t *recs;
    u64 nrecs;
    const uint8_t *in;
    const uint8_t *aad;
    uint8_t *out;
    uint8_t *ok;
    u32 multi_key;  // 0: every record uses key 0 (no key-run scan)
    u32 nkeys;      // records whose key_idx >= nkeys are skipped (open: ok = 0)
    u32 unit_log2;  // chunked kernel: units of 2^unit_log2 steps; CHUNK_LOG2 = each run's scan picks (run_unit_log2)
    // chunked kernel, ungrouped many-key batches (key_*_kernel): when *perm_on != 0 the kernel walks `grouped` (the
    // descriptors in key order) and perm[i] is the batch index of grouped[i] (for the ok bytes)
    const ptls_mi355x_record_t *grouped;
    const u32 *perm;
    const u32 *perm_on;
    // chunked kernel, a batch of one (the per-record path): when one_inline != 0 the descriptor is `one` (it travels in
    // the kernel arguments; `recs` is not read)
    u32 one_inline;
    ptls_mi355x_record_t one;
    // chunked kernel on the per-record path: workgroup w sets done_flag[w] to done_token (system scope) once every output byte
    // it writes is written, for the host thread that polls them (null: none)
    u32 *done_flag;
    // chunked kernel: 0 = workgroup w walks the contiguous records [n*w/grid, n*(w+1)/grid); else it walks the chunks
    // w, w + grid, w + 2*grid, ... of `chunk` records each (records are dealt out across the batch, so a batch whose
    // record sizes follow its order still gives every workgroup a similar share of bytes)
    u64 chunk;
    // chunked kernel: workgroup w walks records [bounds[w], bounds[w + 1]) (balance_bounds_kernel; null: chunk rule)
    const u64 *bounds;
    // chunked seal with QUIC header protection (seal_batch_hp; null hp: none): mask[i] (16 bytes at masks + 16 i) =
    // AES-ECB(hp_keys[hp[i].key_idx], 16 bytes at out + hp[i].sample_off), an hp_nr-round key; zero for a key index
    // >= hp_nkeys
    const ptls_mi355x_hp_t *hp;
    const KeyEntry *hp_keys;
    u32 hp_nkeys;
    u32 hp_nr;
    uint8_t *masks;
    // chunked kernel, a small one-key batch (nrecs < grid; spread_pieces): workgroups [0, nrecs) take record w each,
    // except long ones (spread_long), which the workgroups [nrecs, grid) share; spread_part (grid x 16 B) holds their
    // pieces' GHASH partials, spread_cnt (nrecs counters, zero between launches) counts finished pieces per record
    u32 spread;
    u32x4 *spread_part;
    u32 *spread_cnt;
    // chunked kernel, the W8 kernels (EXT 3, 4; launch_chunked): w8_split 1 = the EXT 4 kernel alone, 2 = a pair, in
    // which EXT 4 takes every run but those of long whole records and EXT 3 (launched after it) those. w8_flags (grid x
    // W8_FLAG_WORDS words, optional): the pair's EXT 4 workgroup w writes to its block how many runs it left to EXT 3
    // and (round 5) where they start; the EXT 3 workgroup w (same grid, same records) returns at once when it left none,
    // and visits just the listed runs when they fit the list, instead of scanning every run of its records again
    u32 w8_split;
    u32 *w8_flags;
    // the value each workgroup stores into done_flag[w] (the calling host thread's token for this call, never 0)
    u32 done_token;
};

#define RUN_SCAN_CAP 256  // records examined per key-run scan (multi-key batches)

// TLS 1.3 record framing (FRAME = 1; lib/picotls.c:719-749, :770-817, :5952-5974). Seal: the GCM plaintext is the
// record's len payload bytes plus the inner content type (flags & 0xff); the wire record at out_off is the 5-byte
// header {23, 3, 3, BE16(len + 17)} (also the AAD), the ciphertext, the tag. Open: the wire record at in_off is header
// (the AAD, as received), len ciphertext bytes (inner type and padding included), tag; the plaintext goes to out_off.
//
// TLS 1.2 AES-GCM record framing (FRAME = 2; buffer_push_encrypted_records lib/picotls.c:779-799, handle_input_tls12
// :6019-6060, build_tls12_aad :753-762). The wire record is header {type, 3, 3, BE16(8 + len + 16)} || explicit nonce
// (8 bytes, big endian: the record IV, tls12.record_iv_size) || ciphertext || tag. GCM nonce = static IV ^ (0^32 ||
// explicit nonce), i.e. ptls_aead_encrypt(..., seq = record IV), and the 13-byte AAD is BE64(seq) || type || 3 || 3 ||
// BE16(len) with seq the record sequence number. Seal: in_off holds the explicit nonce followed by the len payload
// bytes; the type is flags & 0xff. Open: the wire record is at in_off; the AAD takes the header's type.
#define TLS_HEADER_SIZE 5
#define TLS12_RECORD_IV_SIZE 8
#define TLS12_AAD_SIZE 13
template <bool OPEN, int FRAME>
__device__ __forceinline__ u32 gcm_text_len(const ptls_mi355x_record_t &r)
{
    return FRAME == 1 && !OPEN ? r.len + 1 : r.len;
}
// unframed records carry bits 16..31 of the AAD length in flags (PTLS_MI355X_RECORD_AAD_LEN)
template <bool OPEN, int FRAME>
__device__ __forceinline__ u32 gcm_aad_len(const ptls_mi355x_record_t &r)
{
    return FRAME == 1 ? (u32)TLS_HEADER_SIZE : FRAME == 2 ? (u32)TLS12_AAD_SIZE : (u32)r.aad_len | (u32)r.flags << 16;
}
// bytes in front of the GCM text in the input / output record
template <bool OPEN, int FRAME>
__device__ __forceinline__ constexpr u32 frame_in_skip()
{
    return FRAME == 1 ? (OPEN ? TLS_HEADER_SIZE : 0) : FRAME == 2 ? (OPEN ? TLS_HEADER_SIZE : 0) + TLS12_RECORD_IV_SIZE : 0;
}
template <bool OPEN, int FRAME>
__device__ __forceinline__ constexpr u32 frame_out_skip()
{
    return FRAME && !OPEN ? TLS_HEADER_SIZE + (FRAME == 2 ? TLS12_RECORD_IV_SIZE : 0) : 0;
}
// G-lane steps of a record's GHASH stream [pad | AAD | text | length]
template <bool OPEN, int FRAME>
__device__ __forceinline__ u32 gcm_steps(const ptls_mi355x_record_t &r)
{
    return (((gcm_aad_len<OPEN, FRAME>(r) + 15u) >> 4) + ((gcm_text_len<OPEN, FRAME>(r) + 15u) >> 4) + 1 + ENGINE_G - 1) /
           ENGINE_G;
}

#endif  // PTLS_MI355X_ENGINE_RECORD_H
