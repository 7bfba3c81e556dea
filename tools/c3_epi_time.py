"""x6 conv3 + quantiser timings by epilogue mode at B images of 256² (N=192): round mode with the
rate table, round mode evaluating element_bits per element (no table), and noise mode (training;
48-column tiles below 256 tiles·images). Median of HIP-event brackets. Diagnostic (GPU).

    python tools/c3_epi_time.py [--batch 32] [--rounds 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, nargs="+", default=[32, 64])
ap.add_argument("--rounds", type=int, default=30)
args = ap.parse_args()
dev = torch.device("cuda:0")
N = 192
net = ImageCompressor(N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
w3, w3s = net.Encoder.packed()[2], net.Encoder.packed_w3_split()
rate, rtab = net.bitEstimator.packed(), net.bitEstimator.rate_table()
torch.manual_seed(0)


def timed(fn, rounds):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


for B in args.batch:
    hs = kernels.split_planes(torch.randn(B, 32, 32, N, device=dev) * 0.5)
    noise = torch.rand(B, N, 16, 16, device=dev) - 0.5
    cases = {
        "round+table": lambda: kernels.conv3_quant_rate_x6(hs, w3, rate, rtab=rtab, w_split=w3s),
        "round, no table": lambda: kernels.conv3_quant_rate_x6(hs, w3, rate, w_split=w3s),
        "noise (w6)": lambda: kernels.conv3_quant_rate_x6(hs, w3, rate, noise, w_split=w3s),
        "noise (step split)": lambda: kernels.conv3_quant_rate_x6(hs, w3, rate, noise),
    }
    for name, fn in cases.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        print(f"B={B} {name}: {timed(fn, args.rounds):.4f} ms", flush=True)
