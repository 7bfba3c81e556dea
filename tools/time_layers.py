"""Time individual fused layers (HIP events, median of repeats) — diagnostic tool."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tag", default="")
ap.add_argument("--batch", type=int, default=64)
args = ap.parse_args()
dev = torch.device("cuda:0")
N, B = 192, args.batch
net = ImageCompressor(N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
w1, w2, w3, g1, g2 = net.Encoder.packed()
d1, d2, d3, q1, q2 = net.Decoder.packed()
x0 = torch.rand(B, 3, 256, 256, device=dev)
a1 = torch.randn(B, 64, 64, N, device=dev)
s1 = torch.randn(B, 32, 32, N, device=dev)
fns = {
    "conv1_gdn": lambda: kernels.conv1_gdn(x0, w1, net.Encoder.conv1.bias, g1[0], g1[1], N),
    "conv2_gdn": lambda: kernels.conv2_gdn(a1, w2, net.Encoder.conv2.bias, g2[0], g2[1]),
    "deconv2_igdn": lambda: kernels.deconv_igdn(s1, d2, net.Decoder.deconv2.bias, q2[0], q2[1]),
}
flops = {"conv1_gdn": 2.0 * B * 64 * 64 * (N * 243 + N * N),
         "conv2_gdn": 2.0 * B * (32 * 32 * N * N * 25 + 32 * 32 * N * N),
         "deconv2_igdn": 2.0 * B * (32 * 32 * N * N * 25 + 64 * 64 * N * N)}
out = []
with torch.no_grad():
    for name, fn in fns.items():
        for _ in range(3):
            fn()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); fn(); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        ms = ts[len(ts) // 2]
        out.append(f"{name}={ms:.3f}ms({flops[name] / ms / 1e9:.1f}TF)")
print(args.tag, " ".join(out), flush=True)
