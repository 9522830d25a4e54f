/*
 * picotls/mi355x_picotls.h -- picotls algorithm objects backed by the MI355X engine (libptls_mi355x_picotls.so).
 *
 * Drop-in counterparts of include/picotls/fusion.h:105,110 (ptls_fusion_aes{128,256}ctr, ptls_fusion_aes{128,256}gcm,
 * defined at lib/fusion.c:1224-1261). Every callback of ptls_aead_context_t (include/picotls.h:464-514) is
 * implemented on the GPU engine as a batch of one; the deprecated do_encrypt_init/update/final are NULL (tolerated
 * by picotls, t/picotls.c:280-283). Use the batch entry points of picotls/mi355x.h for throughput.
 */
#ifndef picotls_mi355x_picotls_h
#define picotls_mi355x_picotls_h

#include "picotls.h" /* from the picotls installation (-I <picotls>/include) */
#include "mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

extern ptls_cipher_algorithm_t ptls_mi355x_aes128ctr, ptls_mi355x_aes256ctr;
/* QUIC-LB connection-ID cipher, the counterpart of ptls_fusion_quiclb (include/picotls/fusion.h:121, lib/fusion.c:2226-2233) */
extern ptls_cipher_algorithm_t ptls_mi355x_quiclb;
extern ptls_aead_algorithm_t ptls_mi355x_aes128gcm, ptls_mi355x_aes256gcm;
/* TLS-1.2-capable variants (record IV sizes {4, 8}, non_temporal, align_bits 6): the counterparts of
 * ptls_non_temporal_aes{128,256}gcm (include/picotls/fusion.h:117, lib/fusion.c:2159-2184) */
extern ptls_aead_algorithm_t ptls_mi355x_non_temporal_aes128gcm, ptls_mi355x_non_temporal_aes256gcm;

/**
 * Returns the engine keyset behind an AEAD context created from one of the algorithms above (key index 0), so that a
 * caller can move from per-record calls to ptls_mi355x_seal_batch / ptls_mi355x_open_batch on the same traffic key.
 */
ptls_mi355x_keyset_t *ptls_mi355x_aead_get_keyset(ptls_aead_context_t *ctx);

/*
 * Counterparts of fusion's raw context API (include/picotls/fusion.h:40-94; lib/fusion.c:401-1049), for callers that
 * drive ptls_fusion_aesgcm_* / ptls_fusion_aesecb_* directly instead of the AEAD objects. No x86 types cross this
 * boundary: fusion's `__m128i ctr` is passed as its 16 bytes in memory (what _mm_storeu_si128(p, ctr) writes), so a
 * caller switches with one store. The GCM nonce is the counter's upper 12 bytes, byte-reversed (the layout
 * calc_counter builds, lib/fusion.c:1126-1133); as in fusion's encrypt, the low 32 bits are ignored there (fusion sets
 * them to 1 for E(K, J0), lib/fusion.c:489), and decrypt counts from them as fusion's does (below). One engine keyset per context; a call is a per-record launch, so use the
 * batch API of picotls/mi355x.h for throughput. The contexts are not thread-safe (fusion's are not either).
 */
typedef struct ptls_mi355x_aesgcm_context ptls_mi355x_aesgcm_context_t;

/* ptls_fusion_aesgcm_new: key of 16 or 32 bytes; capacity = the largest AAD + payload of a call (NULL on failure) */
ptls_mi355x_aesgcm_context_t *ptls_mi355x_aesgcm_new(const void *key, size_t key_size, size_t capacity);
/* ptls_fusion_aesgcm_set_capacity: grows the capacity; returns the context (possibly moved), or NULL on failure, in
 * which case ctx is unchanged */
ptls_mi355x_aesgcm_context_t *ptls_mi355x_aesgcm_set_capacity(ptls_mi355x_aesgcm_context_t *ctx, size_t capacity);
/* ptls_fusion_aesgcm_free */
void ptls_mi355x_aesgcm_free(ptls_mi355x_aesgcm_context_t *ctx);
/**
 * ptls_fusion_aesgcm_encrypt: writes inlen bytes of ciphertext and the 16-byte tag to output, and with supp the header
 * protection mask of supp->input (read after the seal, so it may point into output). inlen + aadlen must not exceed the
 * capacity. A call the engine cannot complete fails closed: output (inlen + 16 bytes) and supp->output are zeroed.
 */
void ptls_mi355x_aesgcm_encrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                                const void *ctr, const void *aad, size_t aadlen, ptls_aead_supplementary_encryption_t *supp);
/* ptls_fusion_aesgcm_decrypt: 1 if the tag verifies (plaintext in output), else 0 (the plaintext is written either way,
 * as fusion's). fusion's decrypt counts from the counter's low 32 bits (lib/fusion.c:679-682: a 64-bit add on the
 * register's low half, E(K, J0) at low + 1, data block b at low + 2 + b) while its encrypt ignores them; calc_counter
 * leaves them zero. This decrypt does the same for any value (round 6): with non-zero low bits the output is that
 * keystream XOR the input and the tag holds iff it equals GHASH ^ E(K, counter + 1), bit for bit fusion's result */
int ptls_mi355x_aesgcm_decrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                               const void *ctr, const void *aad, size_t aadlen, const void *tag);

/* ptls_fusion_aesecb_context_t: AES-ECB encryption of single blocks (fusion supports encryption only; so does this) */
typedef struct ptls_mi355x_aesecb_context {
    ptls_mi355x_keyset_t *ks;
} ptls_mi355x_aesecb_context_t;
/* ptls_fusion_aesecb_init without fusion's x86-only avx256 flag; is_enc must be 1 (fusion asserts it). 0 or an error */
int ptls_mi355x_aesecb_init(ptls_mi355x_aesecb_context_t *ctx, int is_enc, const void *key, size_t key_size);
void ptls_mi355x_aesecb_dispose(ptls_mi355x_aesecb_context_t *ctx);
/* ptls_fusion_aesecb_encrypt: one 16-byte block (aborts if the engine cannot produce it: any output would leak src) */
void ptls_mi355x_aesecb_encrypt(ptls_mi355x_aesecb_context_t *ctx, void *dst, const void *src);

#ifdef __cplusplus
}
#endif

#endif
