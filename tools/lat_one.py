import sys, numpy as np
sys.path.insert(0, "/root/repo")
import torch, picotls_amd as pa
torch.cuda.init()
rng = np.random.default_rng(1)
enc = pa.aead_new_direct(pa.aes128gcm, True, rng.bytes(16), rng.bytes(12))
pt, aad = rng.bytes(int(sys.argv[1])), rng.bytes(13)
for _ in range(300):
    enc.encrypt(pt, 7, aad)
