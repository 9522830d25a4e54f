"""TLS 1.3 traffic-key derivation for the engine's keysets: the part of picotls' key schedule that ``ptls_aead_new``
runs before ``ptls_aead_new_direct`` (control plane, not the record hot path; Python's hmac/hashlib do the SHA-2).

    ptls_hkdf_expand         lib/picotls.c:6411-6441   HKDF-Expand (RFC 5869) with HMAC over the suite hash
    ptls_hkdf_expand_label   lib/picotls.c:6443-6468   HkdfLabel = u16 length || u8-block("tls13 " || label) ||
                                                       u8-block(hash_value)
    get_traffic_keys         lib/picotls.c:1627-1646   key = Expand-Label(secret, "key"), iv = Expand-Label(secret, "iv")
    ptls_aead_new            lib/picotls.c:6529-6551   new_aead -> ptls_aead_new_direct
"""
from __future__ import annotations

import hmac

PTLS_HKDF_EXPAND_LABEL_PREFIX = "tls13 "  # include/picotls.h:228
DIGEST_SIZE = {"sha256": 32, "sha384": 48, "sha512": 64}


def hkdf_expand(hash_name: str, prk: bytes, info: bytes, outlen: int) -> bytes:
    """ptls_hkdf_expand: T(i) = HMAC(prk, T(i-1) || info || i), i = 1, 2, ...; the first outlen bytes."""
    out, t, i = b"", b"", 0
    while len(out) < outlen:
        i += 1
        t = hmac.new(prk, t + info + bytes([i]), hash_name).digest()
        out += t
    return out[:outlen]


def hkdf_expand_label(hash_name: str, secret: bytes, label: str, outlen: int, hash_value: bytes = b"",
                      label_prefix: str | None = None) -> bytes:
    """ptls_hkdf_expand_label (label_prefix None = "tls13 ", as picotls)."""
    if label_prefix is None:
        label_prefix = PTLS_HKDF_EXPAND_LABEL_PREFIX
    full = (label_prefix + label).encode()
    info = outlen.to_bytes(2, "big") + bytes([len(full)]) + full + bytes([len(hash_value)]) + hash_value
    return hkdf_expand(hash_name, secret[:DIGEST_SIZE[hash_name]], info, outlen)


def traffic_keys(key_size: int, hash_name: str, secret: bytes, iv_size: int = 12,
                 label_prefix: str | None = None) -> tuple[bytes, bytes]:
    """get_traffic_keys: the AEAD key and static IV of a traffic secret (secret is digest_size bytes of it)."""
    key = hkdf_expand_label(hash_name, secret, "key", key_size, label_prefix=label_prefix)
    iv = hkdf_expand_label(hash_name, secret, "iv", iv_size, label_prefix=label_prefix)
    return key, iv
