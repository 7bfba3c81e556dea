"""SHA-256 of the k9 x6 weight gradients (conv1's and deconv3's shapes, B=4 and B=32 at 256²)
on seeded operands: compare two library builds for bit-identity
(ICLR17_LIB=... python tools/k9_sha.py). GPU."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for B, S, M in ((4, 256, 192), (32, 256, 192), (3, 144, 128)):
    g = torch.from_numpy(synth.normal_like(11 + B, (B, S // 4, S // 4, M), 0.3)).to(dev)
    x = torch.from_numpy(synth.normal_like(12 + B, (B, 3, S, S), 1.0)).to(dev)
    dw = kernels.wgrad_k9_x6(kernels.split_planes(g), x)
    torch.cuda.synchronize()
    out[f"B{B}_S{S}_M{M}"] = hashlib.sha256(dw.cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps(out))
