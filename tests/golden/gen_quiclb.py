#!/usr/bin/env python3
"""Writes tests/golden/quiclb_vectors.json: QUIC-LB CID vectors produced by picotls' own lib/fusion.c.

ptls_fusion_quiclb (lib/fusion.c:2186-2233 over lib/quiclb-impl.h) is compiled unmodified from /root/reference by
oracle/Makefile (oracle/_ref/libfusion_ref.so) and driven through ptls_cipher_new / ptls_cipher_encrypt exactly as
t/quiclb.c:36-45 does. For every CID length 7..19 and a few seeded keys the fixture stores the splitmix64 seed of the
(key, plaintext) pair and the expected ciphertext; decryption must invert it.

    make -C oracle && python tests/golden/gen_quiclb.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, HERE)

from oracle import FusionRef  # noqa: E402
from vectors import splitmix_bytes  # noqa: E402


def main():
    ref = FusionRef()
    out = {"generator": "splitmix64(seed) bytes: key (16) | plaintext (len); see tests/golden/vectors.py",
           "source": "ptls_fusion_quiclb via ptls_cipher_new/ptls_cipher_encrypt (oracle/_ref/libfusion_ref.so)",
           "vectors": []}
    seed = 0x91CB0000
    for k in range(6):
        for ln in range(7, 20):
            seed += 1
            blob = splitmix_bytes(seed, 16 + ln)
            key, pt = blob[:16], blob[16:]
            ct = ref.quiclb(key, pt, True)
            assert ref.quiclb(key, ct, False) == pt
            out["vectors"].append({"seed": seed, "len": ln, "ct": ct.hex()})
    with open(os.path.join(HERE, "quiclb_vectors.json"), "w") as f:
        json.dump(out, f, indent=0)
        f.write("\n")
    print(len(out["vectors"]), "vectors")


if __name__ == "__main__":
    main()
