"""Time the x6 and fp32 weight-gradient kernels at the train shapes (B=32: conv2/deconv2 32²→64²,
conv3/deconv1 16²→32²) — diagnostic tool (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels  # noqa: E402

dev = torch.device("cuda:0")
B, M = int(os.environ.get("B", "32")), 192
torch.manual_seed(0)


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[n // 2]


for Ho in (32, 16):
    G = torch.randn(B, Ho, Ho, M, device=dev)
    X = torch.randn(B, 2 * Ho, 2 * Ho, M, device=dev)
    Gs, Xs = kernels.split_planes(G), kernels.split_planes(X)
    fl = 2.0 * B * Ho * Ho * M * M * 25
    t6 = timeit(lambda: kernels.wgrad_k5_x6(Gs, Xs))
    t32 = timeit(lambda: kernels.wgrad_k5(G, X))
    print(f"Ho={Ho}: x6 {t6:.3f} ms ({fl / t6 / 1e9:.1f} TF)  fp32 {t32:.3f} ms ({fl / t32 / 1e9:.1f} TF)",
          flush=True)
