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

#ifdef __cplusplus
}
#endif

#endif
