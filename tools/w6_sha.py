"""x6 conv3 with pre-split weights vs split in the loop: ŷ, y and the bit partials bit for bit
(B=64 and B=3 at 256² / 144², N=192 and 128, round and noise mode). GPU."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

dev = torch.device("cuda:0")
ok = True
for N, B, S in ((192, 64, 256), (128, 3, 144)):
    net = ImageCompressor(N)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
    net = net.to(dev).eval()
    w3 = net.Encoder.packed()[2]
    w3s = net.Encoder.packed_w3_split()
    rate, rtab = net.bitEstimator.packed(), net.bitEstimator.rate_table()
    hs = kernels.split_planes(torch.from_numpy(synth.normal_like(3, (B, S // 8, S // 8, N), 0.7)).to(dev))
    noise = torch.from_numpy(synth.uniform(4, (B, N, S // 16, S // 16), -0.5, 0.5)).to(dev)
    for nz in (None, noise):
        a = kernels.conv3_quant_rate_x6(hs, w3, rate, nz, want_y=True, rtab=rtab if nz is None else None)
        b = kernels.conv3_quant_rate_x6(hs, w3, rate, nz, want_y=True, rtab=rtab if nz is None else None,
                                        w_split=w3s)
        same = all(torch.equal(x, y) for x, y in zip(a, b))
        ok &= same
        print(f"N={N} B={B} S={S} {'noise' if nz is not None else 'round'}: bit-identical {same}")
print("ALL bit-identical" if ok else "DIFFERENT")
sys.exit(0 if ok else 1)
