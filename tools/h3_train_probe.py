"""Diagnostic: NaN / agreement probe of the h3 training forward stages at a small size against the
x6 forward (B, H, W from argv; default 1×32×32, N=192)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import autograd, kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

B, H, W = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (1, 32, 32)
N = 192
dev = torch.device("cuda", 0)
net = ImageCompressor(out_channel_N=N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev)
x = torch.from_numpy(synth.to_unit_float(synth.image_u8(5, B, H, W))).to(dev)
noise = torch.from_numpy(synth.uniform(6, (B, N, H // 16, W // 16), -0.5, 0.5)).to(dev)
enc = net.Encoder
with torch.no_grad():
    kernels.set_precision("x6")
    _, sx = autograd.analysis_features_train(enc, x)
    kernels.set_precision("h3")
    _, sh = autograd.analysis_features_train(enc, x)
    for k in ("u1", "u2"):
        a, b = sh[k], sx[k]
        print(k, "nan", torch.isnan(a).sum().item(), "max rel", ((a - b).abs().max() / b.abs().max()).item())
    for k in ("a1s", "a2s"):
        a, b = kernels.merge_planes(sh[k]), kernels.merge_planes(sx[k])
        print(k, "nan", torch.isnan(a).sum().item(), "max rel", ((a - b).abs().max() / b.abs().max()).item())
    a2 = kernels.merge_h3(sh["a2h"])
    print("a2h nan", torch.isnan(a2).sum().item())
    yt, bits, _, yh = kernels.conv3_quant_rate_h3(sh["a2h"], enc.packed_h3()[1], net.bitEstimator.packed(), noise)
    print("y_tilde nan", torch.isnan(yt).sum().item(), "bits nan", torch.isnan(bits).sum().item())
    yr, _, _, _ = kernels.conv3_quant_rate_h3(sh["a2h"], enc.packed_h3()[1], net.bitEstimator.packed())
    print("round-mode y_hat nan", torch.isnan(yr).sum().item())
