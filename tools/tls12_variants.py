"""Tries simple explanations of the round-5 failing run's fusion TLS 1.2 tags (b22b0ab0... / 37cb0a33...,
profiles/r5/tls12_tag_recurrence.txt) with oracle/gcm_ref.c: other AAD sequence numbers, content types and AAD lengths,
neighbouring explicit nonces, J0 counters 0..9 and 2^32-1. None reproduces them (profiles/r6/tls12_pin.txt).
Test infrastructure; run from the repo root after `make -C oracle`."""
import ctypes, itertools
L = ctypes.CDLL("oracle/_ref/libtls12_ref.so"); G = ctypes.CDLL("oracle/_ref/libgcm_oracle.so")
rs = 0x1234567
def rnd(n):
    global rs
    out = bytearray(n)
    for i in range(n):
        rs ^= (rs << 13) & (2**64-1); rs ^= rs >> 7; rs ^= (rs << 17) & (2**64-1)
        out[i] = (rs >> 24) & 0xff
    return bytes(out)
targets = {16: "b22b0ab019791a83754fa9862da772d4", 32: "37cb0a337c0e30194d155ad9ef3d4517"}
good = {16: "542e39644d4660c7142ee58f157b1b87", 32: "09882a9a93516602338dd22b461646fe"}
for ks in (16, 32):
    ms = rnd(48); rnds = rnd(64); data = rnd(40000)
    key = ctypes.create_string_buffer(32); fixed = ctypes.create_string_buffer(4)
    assert L.ref_tls12_server_keys(ctypes.c_size_t(ks), ms, rnds, key, fixed) == 0
    iv = fixed.raw + bytes(8)
    def tag(seqexp, aad, text):
        out = ctypes.create_string_buffer(len(text) + 16)
        G.oracle_gcm_seal(key, ctypes.c_size_t(ks), iv, ctypes.c_uint64(seqexp), aad, ctypes.c_size_t(len(aad)), text, ctypes.c_size_t(len(text)), out)
        return out.raw[-16:].hex()
    R = 0x1122334455667788
    def aad12(seq, typ=23, n=16384):
        return seq.to_bytes(8, 'big') + bytes([typ, 3, 3, n >> 8, n & 255])
    t = tag(R, aad12(1), data[:16384]); print(ks, "baseline", t, t == good[ks])
    hits = []
    for seq in range(0, 8):
        for nonce in (R - 1, R, R + 1, 0, 1):
            for typ in (23, 22, 21, 0):
                for aad in (aad12(seq, typ), aad12(seq, typ)[8:], aad12(seq, typ)[:12], aad12(seq, typ) + b"\0"*3):
                    if tag(nonce, aad, data[:16384]) == targets[ks]:
                        hits.append((seq, hex(nonce), typ, aad.hex()))
    print(ks, "hits", hits)

print("--- J0 / GHASH-over-plaintext variants")
rs = 0x1234567
for ks in (16, 32):
    ms = rnd(48); rnds = rnd(64); data = rnd(40000)
    key = ctypes.create_string_buffer(32); fixed = ctypes.create_string_buffer(4)
    L.ref_tls12_server_keys(ctypes.c_size_t(ks), ms, rnds, key, fixed)
    R = 0x1122334455667788
    nonce = fixed.raw + R.to_bytes(8, 'big')
    def E(b):
        o = ctypes.create_string_buffer(16); G.oracle_aes_encrypt(key, ctypes.c_size_t(ks), o, b); return o.raw
    def xor(a, b): return bytes(x ^ y for x, y in zip(a, b))
    tgt = bytes.fromhex(targets[ks]); gd = bytes.fromhex(good[ks])
    ej0 = E(nonce + (1).to_bytes(4, 'big'))
    S = xor(gd, ej0)  # the correct GHASH value
    for c in list(range(0, 10)) + [2**32 - 1]:
        if xor(tgt, E(nonce + c.to_bytes(4, 'big'))) == S: print(ks, "hit: J0 counter", c)
    print(ks, "tag xor good", xor(tgt, gd).hex())
