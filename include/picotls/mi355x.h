/*
 * picotls/mi355x.h -- MI355X (gfx950) AES-GCM record engine for picotls: the C-ABI drop-in boundary.
 *
 * Two layers, both plain C ABI (no HIP or torch types; device buffers are passed as void *, streams as void *
 * holding a hipStream_t, NULL = the device's default stream):
 *
 * 1. The batch engine (libptls_mi355x.so). picotls has only per-record synchronous AEAD calls, so a GPU backend
 *    adds one entry point that seals or opens N independent records in one launch. Each record of a batch gives
 *    exactly what one picotls call gets, so batch results equal N independent calls:
 *        ptls_mi355x_seal_batch(...)  record i  ==  ptls_aead_encrypt(ctx[key_idx], out+out_off, in+in_off, len, seq,
 *                                                                    aad+aad_off, aad_len)
 *                                     include/picotls.h:2102-2107 -> do_encrypt (fusion: lib/fusion.c:1136-1146 ->
 *                                     ptls_fusion_aesgcm_encrypt :401)
 *        ptls_mi355x_open_batch(...)  record i  ==  ptls_aead_decrypt(ctx[key_idx], out+out_off, in+in_off, len+16, seq,
 *                                                                    aad+aad_off, aad_len) != SIZE_MAX
 *                                     include/picotls.h:2160-2164 -> do_decrypt (fusion: lib/fusion.c:1154-1171 ->
 *                                     ptls_fusion_aesgcm_decrypt :661)
 *    A keyset replaces N ptls_aead_new_direct(algo, is_enc, key, iv) calls (lib/picotls.c:6553-6568; fusion's
 *    aesgcm_setup lib/fusion.c:1189-1211 / new_aesgcm :985-1011): AES key schedule, H = E_K(0^128) and the H-power
 *    tables are derived on the GPU. The static IV / do_set_iv semantics (lib/fusion.c:1173-1187,
 *    ptls_aead_xor_iv lib/picotls.c:6576-6585) are ptls_mi355x_keyset_set_iv / _get_iv.
 *
 * 2. The picotls algorithm objects (libptls_mi355x_picotls.so, built where picotls.h is available):
 *        extern ptls_aead_algorithm_t ptls_mi355x_aes128gcm, ptls_mi355x_aes256gcm;
 *    the exact counterparts of ptls_fusion_aes128gcm / ptls_fusion_aes256gcm (lib/fusion.c:1236-1261), each call a
 *    batch of one. They are declared in picotls/mi355x_picotls.h so that this header does not need picotls.h.
 *
 * Error behaviour follows the reference: sealing has no error path in picotls (fusion asserts on OOM,
 * lib/fusion.c:1143); here invalid arguments / launch failures return a negative value. Opening reports a per-record
 * ok byte (1 = tag verified) and, like fusion (lib/fusion.c:783-828), writes the plaintext even when the tag fails.
 */
#ifndef picotls_mi355x_h
#define picotls_mi355x_h

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/**
 * One record of a batch (40 bytes, little endian, 8-byte aligned array). Offsets are byte offsets into the arenas
 * passed to the batch call. The AAD length is aad_len | flags << 16 for seal_batch / open_batch (flags = 0 for AADs
 * below 64 KiB; PTLS_MI355X_RECORD_AAD_LEN); the framed calls below give flags their own meaning.
 *   seal: reads  in[in_off .. in_off+len)            plaintext
 *         writes out[out_off .. out_off+len+16)      ciphertext || tag   (out may alias in)
 *   open: reads  in[in_off .. in_off+len+16)         ciphertext || tag
 *         writes out[out_off .. out_off+len)         plaintext            (out may alias in)
 *   aad:  aad[aad_off .. aad_off+aad_len)
 *   nonce = static_iv(key_idx) ^ (0^32 || seq big-endian)        (lib/picotls.c:6587-6601, lib/fusion.c:1127-1134)
 * len is at most PTLS_MI355X_MAX_RECORD_LEN, the AAD at most PTLS_MI355X_MAX_AAD_LEN and key_idx is below the keyset
 * size: a record with a larger len, AAD or key_idx is rejected (nothing is written for it; open reports ok = 0), so a
 * corrupt descriptor cannot address memory beyond the offsets it names.
 */
typedef struct st_ptls_mi355x_record_t {
    uint64_t in_off;
    uint64_t out_off;
    uint64_t seq;
    uint32_t aad_off;
    uint32_t len;
    uint32_t key_idx;
    uint16_t aad_len;
    uint16_t flags; /* seal_batch / open_batch: bits 16..31 of the AAD length; TLS framing: the content type */
} ptls_mi355x_record_t;

#define PTLS_MI355X_RECORD_SIZE 40
#define PTLS_MI355X_MAX_RECORD_LEN (1u << 30) /* 1 GiB; TLS caps records at 2^14 + 256 */
#define PTLS_MI355X_MAX_AAD_LEN (1u << 30)
#define PTLS_MI355X_RECORD_AAD_LEN(r) ((uint32_t)(r)->aad_len | (uint32_t)(r)->flags << 16)

typedef struct st_ptls_mi355x_keyset_t ptls_mi355x_keyset_t;

/**
 * Returns 1 when a gfx950 device is usable and the engine's code object loads, 0 otherwise.
 */
int ptls_mi355x_is_supported(void);

/**
 * Creates a keyset of nkeys AES-GCM traffic keys on the current HIP device.
 * keys: nkeys * key_size bytes (host memory), ivs: nkeys * 12 bytes (host memory), key_size: 16 or 32.
 * Returns NULL on invalid arguments or device failure.
 *
 * Keysets are independent, like picotls contexts (lib/picotls.c:6553-6568): creating, rekeying or freeing one never
 * waits for the device as a whole, only (where stated) for that keyset's own work. A one-key keyset (what each
 * ptls_aead_new_direct on the MI355X objects makes) takes an entry from a per-device pool; its setup launch (the key in
 * the kernel arguments, held in host memory until then and cleared after) runs on the stream of its first use, ahead
 * of that use, so creating one launches nothing. A many-key keyset waits until its key arrays have been copied to the
 * device.
 */
ptls_mi355x_keyset_t *ptls_mi355x_keyset_new(const void *keys, const void *ivs, size_t nkeys, size_t key_size);
/**
 * Destroys a keyset. Device key material is cleared (ptls_clear_memory, lib/fusion.c:1045) in stream order after every
 * launch already made with the keyset, on any stream; the call itself does not wait.
 */
void ptls_mi355x_keyset_free(ptls_mi355x_keyset_t *ks);
size_t ptls_mi355x_keyset_size(const ptls_mi355x_keyset_t *ks);
size_t ptls_mi355x_keyset_key_size(const ptls_mi355x_keyset_t *ks);
/* the HIP device the keyset's entries live on (the current device when it was created) */
int ptls_mi355x_keyset_device(const ptls_mi355x_keyset_t *ks);
/**
 * Replaces the key and static IV of the n entries key_idx[0..n) (host arrays: n * key_size key bytes, n * 12 IV bytes),
 * deriving their schedules and H powers on the device: the rekey of some connections of a many-connection keyset, e.g.
 * after a TLS 1.3 KeyUpdate (picotls rekeys a sender once its record sequence number reaches 2^24,
 * lib/picotls.c:6220-6232, update_send_key -> setup_traffic_protection). Stream-ordered: launches made with the keyset
 * before the call use the old entries, launches made after it the new ones; the call waits for the keyset's launches in
 * flight (not for other work on the device) and for the copies of its arguments.
 * Returns 0, or -1 on invalid arguments / out-of-range or repeated indices (nothing changed) or device failure.
 */
int ptls_mi355x_keyset_update(ptls_mi355x_keyset_t *ks, const uint32_t *key_idx, const void *keys, const void *ivs, size_t n);
/**
 * Static IV accessors (do_get_iv / do_set_iv, include/picotls.h:475-481). Return 0 on success.
 */
int ptls_mi355x_keyset_get_iv(ptls_mi355x_keyset_t *ks, size_t key_idx, void *iv);
int ptls_mi355x_keyset_set_iv(ptls_mi355x_keyset_t *ks, size_t key_idx, const void *iv);

/**
 * Batch schedule used by seal_batch / open_batch on this keyset (no reference counterpart: fusion processes one record
 * per call). Results are identical under every schedule; only the work distribution differs.
 *   AUTO      = CHUNKED (the default)
 *   LOCKSTEP  one whole record per 8-lane group, records assigned statically; kept for comparison
 *   CHUNKED   waves pull work units from a per-run queue. Runs of uniform record lengths use whole records as units;
 *             other runs cut records into 2 KiB GHASH units recombined with H^128, which balances mixed lengths and
 *             short per-connection key runs
 * Returns 0, or -1 for an unknown schedule.
 */
#define PTLS_MI355X_SCHEDULE_AUTO 0
#define PTLS_MI355X_SCHEDULE_LOCKSTEP 1
#define PTLS_MI355X_SCHEDULE_CHUNKED 2
int ptls_mi355x_keyset_set_schedule(ptls_mi355x_keyset_t *ks, int schedule);

/**
 * Constant-time LDS access (no reference counterpart: fusion's AES-NI / PCLMUL code is constant-time by construction).
 * With on != 0 the keyset's batches and per-record calls use the variant in which every LDS access has a
 * data-independent pattern by construction (SQ_LDS_BANK_CONFLICT equal for any key and payload). Since
 * the window-major power tables (late round 3) the AES T-table lookups, the GHASH Horner steps, each lane's last block
 * position and the unit combines are built that way in both settings, so the two run the same kernels and the setting
 * costs no throughput. Every keyset is constant-time when created (round 4; fusion, which this replaces, is constant-time
 * for every context); the environment variable PTLS_MI355X_CONSTANT_TIME=0 (read when a device is first used) creates
 * keysets with the setting off, and on = 0 turns it off for one keyset. Off, a keyset may take the lockstep schedule.
 * Returns 0, or -1.
 */
int ptls_mi355x_keyset_set_constant_time(ptls_mi355x_keyset_t *ks, int on);
/* 1 when the keyset uses the constant-time variant, else 0 */
int ptls_mi355x_keyset_get_constant_time(const ptls_mi355x_keyset_t *ks);

/**
 * Seals nrecs records in one launch. Asynchronous on `stream`. recs, in, aad, out (and ok, results of the calls below)
 * are addresses the device can access: device memory, host memory from hipHostMalloc (its address is the device
 * address), or host memory registered with hipHostRegister passed as the address hipHostGetDevicePointer returns for it
 * (that address may differ from the host pointer). Kernels reading and writing host memory do so over PCIe.
 * Records may come in any order: with a many-key keyset (up to 2^20 keys) a batch whose key runs would average under
 * 8 records is grouped by key_idx on the device first (scratch kept in the keyset; batches on different streams that
 * share the keyset are ordered through it).
 * Returns 0 on success, a negative value on invalid arguments or launch failure.
 */
int ptls_mi355x_seal_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                           const void *aad, void *out, void *stream);
/**
 * Opens nrecs records in one launch; ok[i] = 1 when record i authenticated, 0 otherwise. Pointers as for seal_batch.
 */
int ptls_mi355x_open_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                           const void *aad, void *out, uint8_t *ok, void *stream);

/**
 * AES-ECB of nblocks 16-byte blocks, block i under key key_idx[i] (key_idx may be NULL: key 0). Pointers as for seal_batch.
 * The single-block cipher of fusion (ptls_fusion_aesecb_encrypt, lib/fusion.c:924) batched; QUIC header-protection
 * masks are AES-ECB of the ciphertext sample (lib/fusion.c:1051-1101).
 */
int ptls_mi355x_ecb_batch(ptls_mi355x_keyset_t *ks, const uint32_t *key_idx, const void *in, void *out, size_t nblocks,
                          void *stream);

/**
 * TLS 1.3 record protection, batched (the record layer of lib/picotls.c: aead_encrypt :728-738 and
 * buffer_push_encrypted_records :770-817 on the send side, the decrypt + padding strip of :5952-5974 on the receive
 * side). The records' aad_off / aad_len are ignored: the AAD is the 5-byte record header.
 *
 * seal_tls_records: record i seals recs[i].len payload bytes at in + in_off followed by the inner content type
 * (recs[i].flags & 0xff; PTLS_CONTENT_TYPE_APPDATA = 23 for application data) and writes the wire record at
 * out + out_off: header {23, 3, 3, BE16(len + 17)} || ciphertext (len + 1 bytes) || tag, len + 22 bytes in total.
 * len must not exceed PTLS_MAX_PLAINTEXT_RECORD_SIZE (16384), as in buffer_push_encrypted_records.
 *
 * open_tls_records: record i is the wire record at in + in_off, whose recs[i].len = header length field - 16 (the
 * ciphertext including the inner type and padding). The plaintext (len bytes) goes to out + out_off. ok[i] = 1 only
 * if the tag verifies, the header is {23, 3, 3, BE16(len + 16)} and an inner content type is found; results (may be
 * NULL) gives the content length after stripping the type and the zero padding, the inner type and a status.
 */
#define PTLS_MI355X_TLS_OK 0
#define PTLS_MI355X_TLS_BAD_MAC 1            /* PTLS_ALERT_BAD_RECORD_MAC */
#define PTLS_MI355X_TLS_BAD_HEADER 2         /* outer type not application_data, wrong version or length */
#define PTLS_MI355X_TLS_UNEXPECTED_MESSAGE 3 /* PTLS_ALERT_UNEXPECTED_MESSAGE: no content type, or empty alert/handshake */
typedef struct st_ptls_mi355x_tls_result_t {
    uint32_t plain_len;   /* content bytes at out + out_off */
    uint8_t content_type; /* inner content type */
    uint8_t status;       /* PTLS_MI355X_TLS_* */
    uint16_t reserved;
} ptls_mi355x_tls_result_t;

int ptls_mi355x_seal_tls_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                 void *out, void *stream);
int ptls_mi355x_open_tls_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                 void *out, uint8_t *ok, ptls_mi355x_tls_result_t *results, void *stream);

/**
 * TLS 1.2 AES-GCM record protection, batched (the tls12 branch of buffer_push_encrypted_records lib/picotls.c:779-799
 * and handle_input_tls12 :6019-6060; the record IV sizes {4, 8} of ptls_non_temporal_aes{128,256}gcm,
 * lib/fusion.c:2159-2184). The keyset's static IV is the 4-byte fixed IV followed by 8 zero bytes; recs[i].seq is the
 * record sequence number that goes into the 13-byte AAD BE64(seq) || type || 3 || 3 || BE16(len) (build_tls12_aad
 * :753-762); the GCM nonce is fixed IV || the record's 8-byte explicit nonce (ptls_aead_encrypt with seq = record IV).
 *
 * seal_tls12_records: in + in_off holds the explicit nonce (8 bytes, big endian, as it goes on the wire) followed by
 * recs[i].len payload bytes; the content type is recs[i].flags & 0xff. Writes the wire record at out + out_off:
 * header {type, 3, 3, BE16(len + 24)} || explicit nonce || ciphertext || tag (len + 37 bytes).
 * open_tls12_records: in + in_off is the wire record, recs[i].len = header length field - 24; the plaintext goes to
 * out + out_off. ok[i] = 1 only if the tag verifies and the header is {type, 3, 3, BE16(len + 24)}; results (may be
 * NULL) gets plain_len = len, the record's content type and a status.
 */
int ptls_mi355x_seal_tls12_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                   void *out, void *stream);
int ptls_mi355x_open_tls12_records(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                                   void *out, uint8_t *ok, ptls_mi355x_tls_result_t *results, void *stream);

/**
 * QUIC header protection, batched. One entry per packet: the 16-byte sample at base + sample_off and the index of the
 * header-protection key in hp_ks. mask[i] (16 bytes at masks + 16 i) = AES-ECB(hp key, sample), i.e. the first
 * keystream block of the AES-CTR cipher initialised with the sample, which is what ptls_aead_encrypt_s writes into
 * supp->output (include/picotls.h:441-456, lib/picotls.c ptls_aead__do_encrypt_s; fusion fuses it into the seal,
 * lib/fusion.c:425-430,636-651). Entries with key_idx >= the keyset size get a zero mask. Pointers as for seal_batch.
 */
typedef struct st_ptls_mi355x_hp_t {
    uint64_t sample_off; /* byte offset of the 16-byte sample from base */
    uint32_t key_idx;    /* header-protection key */
    uint32_t reserved;   /* 0 */
} ptls_mi355x_hp_t;

/* masks for samples already in memory (a receiver removes header protection before it can open the packet) */
int ptls_mi355x_hp_mask_batch(ptls_mi355x_keyset_t *hp_ks, const ptls_mi355x_hp_t *hp, size_t n, const void *base,
                              void *masks, void *stream);

/* seal_batch plus the masks of samples taken from the sealed output (hp[i] for record i; base = out): the sample may
 * cover the tag, as in fusion's supp handling. One launch: the seal kernel computes each run's masks once the run's
 * records are sealed (with the LOCKSTEP schedule: the seal, then a second launch). hp_ks must be on ks's device. */
int ptls_mi355x_seal_batch_hp(ptls_mi355x_keyset_t *ks, const ptls_mi355x_record_t *recs, size_t nrecs, const void *in,
                              const void *aad, void *out, ptls_mi355x_keyset_t *hp_ks, const ptls_mi355x_hp_t *hp,
                              void *masks, void *stream);

/**
 * QUIC-LB connection-ID encryption, batched (draft-ietf-quic-load-balancers; lib/quiclb-impl.h:100-162, the cipher
 * behind ptls_fusion_quiclb lib/fusion.c:2186-2233 / ptls_openssl_quiclb). Entry i transforms len bytes at
 * in + in_off into out + out_off (may alias) under the AES-128 key key_idx of ks (a keyset created with key_size 16;
 * its IVs are unused): encrypt = 1 gives ptls_cipher_encrypt on a context made with ptls_cipher_new(&quiclb, 1, key),
 * encrypt = 0 the inverse (is_enc = 0). len is PTLS_QUICLB_MIN_BLOCK_SIZE (7) .. PTLS_QUICLB_MAX_BLOCK_SIZE (19)
 * (include/picotls.h:116-122); entries with another len or an out-of-range key_idx are skipped (nothing written), where
 * the reference asserts. Pointers as for seal_batch; returns -1 on invalid arguments or a keyset that is not AES-128.
 */
#define PTLS_MI355X_QUICLB_MIN_LEN 7
#define PTLS_MI355X_QUICLB_MAX_LEN 19
typedef struct st_ptls_mi355x_cid_t {
    uint64_t in_off;
    uint64_t out_off;
    uint32_t key_idx;
    uint8_t len;
    uint8_t encrypt;
    uint16_t reserved; /* 0 */
} ptls_mi355x_cid_t;

int ptls_mi355x_quiclb_batch(ptls_mi355x_keyset_t *ks, const ptls_mi355x_cid_t *cids, size_t n, const void *in, void *out,
                             void *stream);
/* one CID on HOST buffers (backs the ptls_mi355x_quiclb cipher object): returns 0, or -1 on invalid arguments */
int ptls_mi355x_quiclb_transform(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t len,
                                 int encrypt);

/**
 * Synchronous single-record helpers on HOST buffers: a batch of one through a pinned staging buffer taken from a
 * per-device pool for the duration of the call (its kernels read and write it in place over PCIe), so calls on different
 * keysets from different threads run concurrently and share nothing. These back the picotls vtable (do_encrypt /
 * do_decrypt / do_encrypt_v) and mirror ptls_aead_encrypt / ptls_aead_decrypt: encrypt writes len+16 bytes (output may
 * alias input); decrypt takes inlen = len+16 and returns the plaintext length or SIZE_MAX (tag mismatch, inlen < 16, or
 * an engine error, which ptls_mi355x_last_error then describes). len and aadlen are limited by
 * PTLS_MI355X_MAX_RECORD_LEN / PTLS_MI355X_MAX_AAD_LEN (fusion has no limit; TLS and QUIC records are far below it).
 * Environment, read when a device is first used: PTLS_MI355X_MAX_STAGE_BYTES caps the staging buffer of one call (a
 * larger record fails), PTLS_MI355X_STAGE_COPY=1 copies through device memory instead of mapping the pinned buffer.
 *
 * The staging pool is bounded (fusion's context owns one allocation and frees it, lib/fusion.c:1043-1049): per device
 * at most PTLS_MI355X_STAGE_POOL_BYTES (default 64 MiB) of idle pinned buffers are kept for later calls, a buffer above
 * 16 MiB (a call on a record above ~8 MiB) is freed when its call returns (hipHostFree, which waits for the device), and
 * the calls of a device share at most 16 streams.
 */
/* pinned host bytes the staging pools hold now, idle and in use, over all devices */
size_t ptls_mi355x_staging_bytes(void);
/* frees every idle staging buffer (e.g. before process exit); calls in progress keep theirs */
void ptls_mi355x_release_staging(void);
int ptls_mi355x_encrypt(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                        const void *aad, size_t aadlen);
size_t ptls_mi355x_decrypt(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen,
                           uint64_t seq, const void *aad, size_t aadlen);
/**
 * encrypt over the concatenation of incnt input vectors (do_encrypt_v, include/picotls.h:501-507; the TLS record layer's
 * {payload, content type}, lib/picotls.c:728-738), gathered straight into the staging buffer. Same layout as ptls_iovec_t.
 */
typedef struct st_ptls_mi355x_iovec_t {
    const void *base;
    size_t len;
} ptls_mi355x_iovec_t;
int ptls_mi355x_encrypt_v(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const ptls_mi355x_iovec_t *input, size_t incnt,
                          uint64_t seq, const void *aad, size_t aadlen);
/**
 * encrypt, then the QUIC header-protection mask of the 16 sealed bytes at output + sample_off (sample_off + 16 <=
 * inlen + 16) under key hp_key_idx of hp_ks, in the same round trip: ptls_aead_encrypt_s with supp (include/picotls.h:
 * 441-456, 2109-2113), whose mask fusion computes inside the seal (lib/fusion.c:425-430,636-651). mask: 16 bytes.
 */
int ptls_mi355x_encrypt_s(ptls_mi355x_keyset_t *ks, size_t key_idx, void *output, const void *input, size_t inlen, uint64_t seq,
                          const void *aad, size_t aadlen, ptls_mi355x_keyset_t *hp_ks, size_t hp_key_idx, size_t sample_off,
                          void *mask);

/**
 * One AES-ECB block on HOST buffers under key key_idx (ptls_fusion_aesecb_encrypt, lib/fusion.c:924). Backs the
 * 16-byte AES-CTR cipher objects (ptls_fusion_aes128ctr equivalents, lib/fusion.c:1051-1101) used for QUIC header
 * protection by the per-record vtable.
 */
int ptls_mi355x_encrypt_block(ptls_mi355x_keyset_t *ks, size_t key_idx, void *out, const void *in);
/**
 * nblocks AES-ECB blocks on HOST buffers under key key_idx in one launch (ptls_fusion_aesecb_encrypt, lib/fusion.c:924,
 * over many blocks). Backs the raw decrypt's counter blocks when the caller's counter does not start at 1
 * (ptls_mi355x_aesgcm_decrypt, the semantics of ptls_fusion_aesgcm_decrypt at lib/fusion.c:679-682).
 */
int ptls_mi355x_encrypt_blocks(ptls_mi355x_keyset_t *ks, size_t key_idx, void *out, const void *in, size_t nblocks);

/**
 * Returns a static string describing the last error on this thread (or "" if none).
 */
const char *ptls_mi355x_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
