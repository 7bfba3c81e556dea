"""deconv1 on the bench's own ŷ (conv3_quant_rate_x6 output of bench.py's workload): the x6k
integer-input form vs its six-product form vs the 16x16x32 engine, timed interleaved."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

N, B, S = 192, 64, 256
dev = torch.device("cuda", 0)
net = ImageCompressor(out_channel_N=N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
x = torch.from_numpy(synth.to_unit_float(synth.image_u8(1000, B, S, S))).to(dev)
with torch.no_grad():
    q = net.encode_latents(x)
ys = q["y_split"]
print("y_hat absmax", q["y_hat"].abs().max().item(), "planes nonzero", [int((ys[p] != 0).sum()) for p in range(3)])
dec = net.Decoder
x1 = dec.packed_x6k()[0]
d1 = dec.packed()[0]
q1 = dec.igdn1.effective_params_x6()
runs = {"old": lambda: kernels.deconv_igdn_x6(ys, d1, dec.deconv1.bias, *q1),
        "x6k": lambda: kernels.deconv_igdn_x6k(ys, x1, dec.deconv1.bias, q1[0], q1[2]),
        "x6k_int": lambda: kernels.deconv_igdn_x6k(ys, x1, dec.deconv1.bias, q1[0], q1[2], int_in=True)}
with torch.no_grad():
    a, b = runs["x6k"](), runs["x6k_int"]()
    print("int == full:", torch.equal(a[0], b[0]))
    for k in runs:
        for _ in range(3):
            runs[k]()
    torch.cuda.synchronize()
    t = {k: [] for k in runs}
    for _ in range(20):
        for k in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            runs[k]()
            e1.record()
            t[k].append((e0, e1))
    torch.cuda.synchronize()
for k in runs:
    ms = sorted(a.elapsed_time(b) for a, b in t[k])
    print(f"{k}: median {ms[len(ms) // 2]:.4f} ms, min {ms[0]:.4f}")
