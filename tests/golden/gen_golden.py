#!/usr/bin/env python3
"""Writes tests/golden/fusion_vectors.json: AES-GCM vectors produced by picotls' own lib/fusion.c.

lib/fusion.c is compiled unmodified from /root/reference by oracle/Makefile (oracle/_ref/libfusion_ref.so) and driven
through the reference's plugin surface (ptls_aead_new_direct + ptls_aead_encrypt, as t/fusion.c:385-466 does).
Inputs are derived from a seeded splitmix64 stream (tests/golden/vectors.py) so the fixture stores only the
generator parameters, the expected ciphertext (whole for records <= 2 KiB, SHA-256 above that) and the tag.

    make -C oracle && python tests/golden/gen_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, HERE)

from oracle import FusionRef  # noqa: E402
from vectors import splitmix_bytes  # noqa: E402

LENS = [0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 255, 256, 1023, 1024, 1025, 1199, 1200, 1201,
        1500, 2047, 2048, 4095, 4096, 8191, 8192, 16383, 16384]
AADS = [0, 1, 5, 12, 13, 15, 16, 17, 32, 33, 64]


def main():
    ref = FusionRef()
    out = {"generator": "splitmix64(seed) bytes: key | iv | aad | pt drawn in that order; see tests/golden/vectors.py",
           "source": "lib/fusion.c via ptls_aead_new_direct/ptls_aead_encrypt (oracle/_ref/libfusion_ref.so)",
           "vectors": []}
    seed = 0x5EED0000
    for key_size in (16, 32):
        for i, ln in enumerate(LENS):
            for j, al in enumerate(AADS):
                if (i + j) % 3 != 0 and ln > 256:  # thin out the long records, keep every short one
                    continue
                seed += 1
                blob = splitmix_bytes(seed, key_size + 12 + 8 + al + ln)
                key, iv = blob[:key_size], blob[key_size:key_size + 12]
                seq = int.from_bytes(blob[key_size + 12:key_size + 20], "little") >> (seed % 64)
                aad = blob[key_size + 20:key_size + 20 + al]
                pt = blob[key_size + 20 + al:]
                sealed = ref.seal(key, iv, seq, aad, pt)
                assert ref.open(key, iv, seq, aad, sealed) == pt
                v = {"seed": seed, "key_size": key_size, "aad_len": al, "len": ln, "seq": seq, "tag": sealed[ln:].hex()}
                if ln <= 2048:
                    v["ct"] = sealed[:ln].hex()
                else:
                    v["ct_sha256"] = hashlib.sha256(sealed[:ln]).hexdigest()
                out["vectors"].append(v)
    with open(os.path.join(HERE, "fusion_vectors.json"), "w") as f:
        json.dump(out, f, indent=0)
        f.write("\n")
    print(len(out["vectors"]), "vectors")


if __name__ == "__main__":
    main()
