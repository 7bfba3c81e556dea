"""Per-layer timings of the bf16 throughput chain at B images of 256² (N=192): median over
rounds of HIP-event brackets around each layer on random bf16 activations. Diagnostic (GPU).

    [ICLR17_LIB=/tmp/ab_x/libiclr17.so] python tools/bf16_time.py [--tag name] [--batch 64]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tag", default="")
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--rounds", type=int, default=30)
args = ap.parse_args()
dev = torch.device("cuda:0")
N, B = 192, args.batch
net = ImageCompressor(N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
w1, w2, w3 = net.Encoder.packed_bf16()
d1, d2, d3 = net.Decoder.packed_bf16()
e1, e2 = net.Encoder.gdn1.effective_params_bf16(), net.Encoder.gdn2.effective_params_bf16()
q1, q2 = net.Decoder.igdn1.effective_params_bf16(), net.Decoder.igdn2.effective_params_bf16()
rate = net.bitEstimator.packed()
rtab = net.bitEstimator.rate_table()
torch.manual_seed(0)
x = torch.rand(B, 3, 256, 256, device=dev)
a1 = kernels.to_bf16(torch.randn(B, 64, 64, N, device=dev) * 0.5)
a2 = kernels.to_bf16(torch.randn(B, 32, 32, N, device=dev) * 0.5)
yq = kernels.to_bf16(torch.round(torch.randn(B, 16, 16, N, device=dev) * 2))
s1 = kernels.to_bf16(torch.randn(B, 32, 32, N, device=dev) * 0.5)
s2 = kernels.to_bf16(torch.randn(B, 64, 64, N, device=dev) * 0.3)
E = net.Encoder
D = net.Decoder
layers = {
    "conv1_gdn1": lambda: kernels.conv1_gdn_bf16(x, w1, E.conv1.bias, *e1, N),
    "conv2_gdn2": lambda: kernels.conv2_gdn_bf16(a1, w2, E.conv2.bias, *e2),
    "conv3_quant_rate": lambda: kernels.conv3_quant_rate_bf16(a2, w3, rate, rtab),
    "deconv1_igdn1": lambda: kernels.deconv_igdn_bf16(yq, d1, D.deconv1.bias, *q1),
    "deconv2_igdn2": lambda: kernels.deconv_igdn_bf16(s1, d2, D.deconv2.bias, *q2),
    "deconv3_clamp": lambda: kernels.deconv3_bf16(s2, d3, D.deconv3.bias),
}
times = {k: [] for k in layers}
for r in range(args.rounds + 3):
    for k, f in layers.items():
        e0, e1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1_.record()
        torch.cuda.synchronize()
        if r >= 3:
            times[k].append(e0.elapsed_time(e1_))
med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
print(json.dumps({"tag": args.tag, "ms": {k: round(v, 4) for k, v in med.items()},
                  "total_ms": round(sum(med.values()), 4)}))
