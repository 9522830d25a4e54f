"""Shared test helpers: materialise golden vectors and convert fusion-internal GHASH values."""
import hashlib

from vectors import splitmix_bytes

POLY = 1 | (0xC2 << 120)  # lib/fusion.c:114, poly_ = {1, 0xc200000000000000}


def h_from_fusion_internal(h_int: bytes) -> bytes:
    """Inverse of fusion's H preprocessing (lib/fusion.c:997-999: byteswap then transformH :127-154, the '<<1 twist')."""
    v = int.from_bytes(h_int, "little")
    c = v & 1
    u = v ^ (POLY if c else 0)
    v = (u >> 1) | (c << 127)
    return v.to_bytes(16, "big")


def materialise(v: dict):
    """Returns (key, iv, seq, aad, pt) for one entry of tests/golden/fusion_vectors.json."""
    ks, al, ln = v["key_size"], v["aad_len"], v["len"]
    blob = splitmix_bytes(v["seed"], ks + 12 + 8 + al + ln)
    key, iv = blob[:ks], blob[ks:ks + 12]
    aad = blob[ks + 20:ks + 20 + al]
    pt = blob[ks + 20 + al:]
    return key, iv, v["seq"], aad, pt


def check_sealed(v: dict, sealed: bytes) -> bool:
    ln = v["len"]
    if sealed[ln:].hex() != v["tag"]:
        return False
    if "ct" in v:
        return sealed[:ln].hex() == v["ct"]
    return hashlib.sha256(sealed[:ln]).hexdigest() == v["ct_sha256"]
