"""Debug: deconv_igdn_h3 with IGDN made the identity (β_eff = 1, γ = 0) on one-hot inputs,
against F.conv_transpose2d."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from iclr_17_compression_amd import kernels, _lib  # noqa
dev = torch.device("cuda", 0)
N, h, w = 192, 5, 7
torch.manual_seed(0)
W = (torch.randn(N, N, 5, 5) * 0.05)
bias = torch.zeros(N)
Wd = W.to(dev)
wh = kernels.pack_h3k(_lib.ICLR17_H3K_DECONV5, Wd, N)
be = torch.ones(N, device=dev)
g6 = torch.zeros(3, N * N, device=dev, dtype=torch.int16)
for (c, yy, xx) in [(5, 2, 3), (5, 0, 0), (0, 2, 3), (1, 2, 3), (2, 2, 3), (3, 2, 3), (4, 2, 3), (8, 2, 3), (16, 2, 3), (100, 2, 3)]:
    x = torch.zeros(1, N, h, w)
    x[0, c, yy, xx] = 1.0
    ref = torch.nn.functional.conv_transpose2d(x, W, bias, stride=2, padding=2, output_padding=1)
    xh = kernels.h3_planes(x.permute(0, 2, 3, 1).contiguous().to(dev))
    _, f, _ = kernels.deconv_igdn_h3(xh, wh, bias.to(dev), be, g6, want_h3=False, want_f32=True)
    f = f.cpu().permute(0, 3, 1, 2)
    e = (f - ref).abs().amax(dim=1)[0]
    bad = (e > 1e-5).nonzero().tolist()
    print(f"onehot c={c} y={yy} x={xx}: max err {e.max().item():.3e}; bad px {bad}")
