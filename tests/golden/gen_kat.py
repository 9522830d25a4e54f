#!/usr/bin/env python3
"""Writes tests/golden/kat.json: the known-answer vectors that picotls' own tests hold for the AES-GCM path.

Every value below is DATA transcribed from the reference's test files (inputs and expected outputs only), with
the file:line it comes from. No reference source is reproduced. Run from the repo root:

    python tests/golden/gen_kat.py

Vector kinds
  ecb       AES-ECB one block                    t/fusion.c:72-86, t/picotls.c:372-413 (FIPS-197 C.1 / C.3 keys),
                                                 t/picotls.c:429-437 (first AES-CTR keystream block = ECB of the IV)
  ghash     GHASH over zero-padded whole blocks  t/fusion.c:88-234. fusion keeps H in its internal byte-reversed,
            "<<1 twisted" form (lib/fusion.c:127-154, :997-999) and the test stores H and the result in that form,
            so the fixture records them as-is ("fusion_internal") and tests/test_oracle.py converts.
  gcm_zero_ctr  raw ptls_fusion_aesgcm_encrypt with counter 0, i.e. IV = 0^96   t/fusion.c:236-256, :277-288, :290-344
  gcm_seq   full AEAD through ptls_aead_new_direct / ptls_aead_encrypt with (key, iv, seq)  t/fusion.c:258-274, :346-380
  nist      McGrew-Viega GCM test cases 1-4 (AES-128, 96-bit IV) held in deps/cifra/src/testmodes.c:395-433; the
            8-/60-byte-IV and AES-192 cases there are skipped (picotls' AEADs take a 96-bit IV and have no AES-192).
            AES-256-GCM is pinned by vectors from lib/fusion.c itself (gen_golden.py -> fusion_vectors.json).
  hp_mask   the QUIC header-protection mask fused into seal (supp), t/fusion.c:290-344 second pass:
            mask = AES-ECB(hp_key = 01*16, sample = sealed[2:18])
  quiclb    the QUIC-LB CID cipher vector of t/quiclb.c:27-30 (7-byte CID; the plaintext array is 19 bytes, zero
            padded, and every prefix of length 7..19 must round-trip)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

ZERO16 = "00" * 16
K_00112233 = "00112233445566778899aabbccddeeff"
AAD_0_19 = bytes(range(20)).hex()
PT_HELLO7 = (b"hello world\n" * 7 + b"\0").hex()  # sizeof(plaintext) includes the NUL, t/fusion.c:263-265
EXP_HELLO7 = (
    "d3a81d964c9b02d79ab041074c8ce2e02e83545245cbd468c84345ca91fba37a67ede8d75ee233d13ebf50c24b86835511bb174ff578b865eb9a2b8f"
    "7708a9601773c507f304c93f674d12a10293c23cd3f85933d501c3bbaae63fbb2366942628"
    "43a5fd2f"
)


def cstr(s: bytes, size: int) -> str:
    """A C char array of `size` initialised from a string literal (zero padded)."""
    return (s + b"\0" * (size - len(s)))[:size].hex()


kat = {
    "ecb": [
        {"src": "t/fusion.c:77-80", "key": ZERO16, "pt": b"hello world!!!!!".hex(), "ct": "172afecb50b5f1237814b2f7cb51d0f7"},
        {"src": "t/fusion.c:82-85", "key": "00" * 32, "pt": b"hello world!!!!!".hex(), "ct": "2a033f0627b3554aa4fe5786550736ff"},
        {"src": "t/picotls.c:374-376,397-401", "key": bytes(range(16)).hex(), "pt": K_00112233,
         "ct": "69c4e0d86a7b0430d8cdb78070b4c55a"},
        {"src": "t/picotls.c:374-376,404-412", "key": bytes(range(32)).hex(), "pt": K_00112233,
         "ct": "8ea2b7ca516745bfeafc49904b496089"},
        {"src": "t/picotls.c:429-437", "key": "2b7e151628aed2a6abf7158809cf4f3c", "pt": "6bc1bee22e409f96e93d7e117393172a",
         "ct": "3ad77bb40d7a3660a89ecaf32466ef97"},
    ],
    "ghash": {
        "src": "t/fusion.c:88-234",
        "h_fusion_internal": cstr(b"hello world bye", 16),
        "cases": [
            {"nblocks": 1, "data": cstr(b"deaddeadbeefbeef", 16), "out_fusion_internal": "12d9d9148b3f20bd202aa59e17a8b07b"},
            {"nblocks": 2, "data": cstr(b"Lorem ipsum dolor sit amet, con", 32),
             "out_fusion_internal": "dadfe89bc78cbd5ca7c1839aa29f8055"},
            {"nblocks": 3, "data": cstr(b"The quick brown fox jumps over the lazy dog.", 48),
             "out_fusion_internal": "addf91523840f7c385af41b17ded4b56"},
            {"nblocks": 5, "data": cstr(b"Lorem ipsum dolor sit amet, consectetur adipiscing elit, sed do eiusmod tempor ", 80),
             "out_fusion_internal": "b8ab1ba8f292f389449d39f6b637ca5d"},
            {"nblocks": 6,
             "data": cstr(b"Lorem ipsum dolor sit amet, consectetur adipiscing elit, sed do eiusmod tempor incididunt ut la", 96),
             "out_fusion_internal": "52ce2522862c91a4e74ef99a3277bd3e"},
        ],
    },
    "gcm_zero_ctr": [
        {"src": "t/fusion.c:238-248", "key": ZERO16, "aad": b"hello".hex(), "pt": ZERO16,
         "sealed": "0388dace60b6a392f328c2b971b2fe78973fbca65477bf4785b0d561f7e3fd6c"},
        {"src": "t/fusion.c:277-288", "key": ZERO16, "aad": b"a".hex(), "pt": b"X".hex(),
         "sealed": "5b27215ed81a702e3941c80577d52fcb57"},
    ],
    "gcm_zero_ctr_tags": {
        "src": "t/fusion.c:290-344 (key 0^128, IV 0^96, aad = aadlen zero bytes, pt = ptlen zero bytes)",
        "cases": [
            [13, 17, "1b4e515384e8aa5bb781ee12549a2ccf", "4576f18ef3ae9dfd37cf72c4592da874"],
            [13, 32, "84030586f55adf8ac3c145913c6fd0f8", "a062016e90dcc316d061fde5424cf34f"],
            [13, 64, "66165d39739c50c90727e7d49127146b", "a062016e90dcc316d061fde5424cf34f"],
            [13, 65, "eb3b75e1d4431e1bb67da46f6a1a0edd", "a062016e90dcc316d061fde5424cf34f"],
            [13, 79, "8f4a96c7390c26bb15b68865e6a861b9", "a062016e90dcc316d061fde5424cf34f"],
            [13, 80, "5cc2554857b19e7a9e18d015feac61fd", "a062016e90dcc316d061fde5424cf34f"],
            [13, 81, "5a65f0d4db36c981bf7babd11691fe78", "a062016e90dcc316d061fde5424cf34f"],
            [13, 95, "6a8a51152efe928999a610d8a7b1df9d", "a062016e90dcc316d061fde5424cf34f"],
            [13, 96, "6b9c468e24ed96010687f3880a044d42", "a062016e90dcc316d061fde5424cf34f"],
            [13, 97, "1b4eb785b884a7d4fdebaff81c1c12e8", "a062016e90dcc316d061fde5424cf34f"],
            [22, 1328, "0507baaece8d573774c94e8103821316", "a062016e90dcc316d061fde5424cf34f"],
            [21, 1329, "dd70d59030eadb6313e778046540a253", "a062016e90dcc316d061fde5424cf34f"],
            [20, 1330, "f1b456b955afde7603188af0124a32ef", "a062016e90dcc316d061fde5424cf34f"],
            [13, 1337, "a22deec51250a7eb1f4384dea5f2e890", "a062016e90dcc316d061fde5424cf34f"],
            [12, 1338, "42102b0a499b2efa89702ece4b0c5789", "a062016e90dcc316d061fde5424cf34f"],
            [11, 1339, "9827f0b34252160d0365ffaa9364bedc", "a062016e90dcc316d061fde5424cf34f"],
            [0, 80, "98885a3a22bd4742fe7b72172193b163", "a062016e90dcc316d061fde5424cf34f"],
            [0, 96, "afd649fc51e14f3966e4518ad53b9ddc", "a062016e90dcc316d061fde5424cf34f"],
            [20, 85, "afe8b727057c804a0525c2914ef856b0", "a062016e90dcc316d061fde5424cf34f"],
        ],
        "hp_key": "01" * 16,
        "hp_sample_off": 2,
    },
    "gcm_seq": [
        {"src": "t/fusion.c:258-274", "key": K_00112233, "iv": bytes(range(20, 32)).hex(), "seq": 0, "aad": AAD_0_19,
         "pt": PT_HELLO7, "sealed": EXP_HELLO7},
        {"src": "t/fusion.c:346-380 (iv {20,20,20,20,24..31} xor seq32 {0,1,2,3} via ptls_aead_xor_iv)", "key": K_00112233,
         "iv": bytes([20, 20, 20, 20] + list(range(24, 32))).hex(), "xor_iv": "00010203", "seq": 0, "aad": AAD_0_19,
         "pt": PT_HELLO7, "sealed": EXP_HELLO7, "bad_xor_iv": "89abcdef"},
    ],
    "nist": [
        {"src": "deps/cifra/src/testmodes.c:395-400", "key": ZERO16, "iv": "00" * 12, "aad": "", "pt": "", "ct": "",
         "tag": "58e2fccefa7e3061367f1d57a4e7455a"},
        {"src": "deps/cifra/src/testmodes.c:401-406", "key": ZERO16, "iv": "00" * 12, "aad": "", "pt": ZERO16,
         "ct": "0388dace60b6a392f328c2b971b2fe78", "tag": "ab6e47d42cec13bdf53a67b21257bddf"},
        {"src": "deps/cifra/src/testmodes.c:407-419", "key": "feffe9928665731c6d6a8f9467308308",
         "iv": "cafebabefacedbaddecaf888", "aad": "",
         "pt": "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b391aafd255",
         "ct": "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e21d514b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e091473f5985",
         "tag": "4d5c2af327cd64a62cf35abd2ba6fab4"},
        {"src": "deps/cifra/src/testmodes.c:420-433", "key": "feffe9928665731c6d6a8f9467308308",
         "iv": "cafebabefacedbaddecaf888", "aad": "feedfacedeadbeeffeedfacedeadbeefabaddad2",
         "pt": "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b39",
         "ct": "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e21d514b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e091",
         "tag": "5bc94fbc3221a5db94fae95ae7121a47"},
    ],
    "quiclb": {
        "src": "t/quiclb.c:27-30 (draft-ietf-quic-load-balancers-21 vector; round trip for every length 7..19 at :34-46)",
        "key": "fdf726a9893ec05c0632d3956680baf0",
        "pt19": "31441a9c69c275" + "00" * 12,
        "ct7": "67947d29be054a",
    },
}

def main():
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
