"""Per-wave phase timing of one bf16 k5 layer (diagnostic build -DICLR17_K5_STAMPS=1):
ICLR17_LIB=build/ab_k5st/libiclr17.so python tools/k5_stamps.py [deconv2|conv2|conv3|deconv1]. GPU.
Stamps: k5_body entry, main-loop start (after the prologue's DMA issue), main-loop end (after
the trailing vm_barrier), exit. Prints medians in shader cycles and the workgroup timeline."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

layer = sys.argv[1] if len(sys.argv) > 1 else "deconv2"
dev = torch.device("cuda:0")
N, B = 192, 64
net = ImageCompressor(N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
E, D = net.Encoder, net.Decoder
w1, w2, w3 = E.packed_bf16()
d1, d2, d3 = D.packed_bf16()
rate, rtab = net.bitEstimator.packed(), net.bitEstimator.rate_table()
a1 = kernels.to_bf16(torch.randn(B, 64, 64, N, device=dev) * 0.5)
a2 = kernels.to_bf16(torch.randn(B, 32, 32, N, device=dev) * 0.5)
yq = kernels.to_bf16(torch.round(torch.randn(B, 16, 16, N, device=dev) * 2))
s1 = kernels.to_bf16(torch.randn(B, 32, 32, N, device=dev) * 0.5)
fn = {
    "conv2": lambda: kernels.conv2_gdn_bf16(a1, w2, E.conv2.bias, *E.gdn2.effective_params_bf16()),
    "conv3": lambda: kernels.conv3_quant_rate_bf16(a2, w3, rate, rtab),
    "deconv1": lambda: kernels.deconv_igdn_bf16(yq, d1, D.deconv1.bias, *D.igdn1.effective_params_bf16()),
    "deconv2": lambda: kernels.deconv_igdn_bf16(s1, d2, D.deconv2.bias, *D.igdn2.effective_params_bf16()),
}[layer]
for _ in range(20):
    fn()
torch.cuda.synchronize()
buf = np.zeros(8192 * 16 * 8, dtype=np.uint64)
lib = ctypes.CDLL(os.environ["ICLR17_LIB"])
lib.iclr17_debug_k5_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert lib.iclr17_debug_k5_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(8192, 16, 8).astype(np.int64)
valid = st[:, :, 3] > 0
wgs = np.where(valid.any(axis=1))[0]
st = st[wgs]
waves = int(valid[wgs[0]].sum())
st = st[:, :waves]
t0 = st[:, :, 0].min()
pro = st[:, :, 1] - st[:, :, 0]
main = st[:, :, 2] - st[:, :, 1]
epi = st[:, :, 3] - st[:, :, 2]
life = st[:, :, 3].max(axis=1) - st[:, :, 0].min(axis=1)
print(f"{layer}: {len(wgs)} workgroups x {waves} waves; kernel span {st[:, :, 3].max() - t0} cycles")
for n, v in (("prologue", pro), ("main loop", main), ("epilogue", epi)):
    print(f"  {n:10s} median {np.median(v):8.0f}  p10 {np.percentile(v, 10):8.0f}  p90 {np.percentile(v, 90):8.0f}")
print(f"  wg life   median {np.median(life):8.0f}")
if layer != "conv3":   # GDN epilogue split: x² + γ ready | contraction | y tile | stores
    parts = [st[:, :, 4] - st[:, :, 2], st[:, :, 5] - st[:, :, 4], st[:, :, 6] - st[:, :, 5], st[:, :, 3] - st[:, :, 6]]
    print("  epilogue parts (x2+gamma, contraction, y tile, stores):", [int(np.median(v)) for v in parts])
else:   # K-split exchange | quantiser + rate + stores | bit reduction
    parts = [st[:, :, 5] - st[:, :, 2], st[:, :, 6] - st[:, :, 5], st[:, :, 3] - st[:, :, 6]]
    for g in range(2):
        w = slice(4 * g, 4 * g + 4)
        print(f"  group {g} epilogue parts (exchange, quant+rate+stores, bits):", [int(np.median(v[:, w])) for v in parts])
starts = np.sort(st[:, :, 0].min(axis=1) - t0)
print("  wg start times (cycles) at quantiles 0/.25/.5/.75/1:", [int(np.quantile(starts, q)) for q in (0, .25, .5, .75, 1)])
if layer.startswith("deconv"):
    per = len(wgs) // 4
    for ph in range(4):
        sl = slice(ph * per, (ph + 1) * per)
        print(f"  phase {ph}: main {np.median(main[sl]):8.0f} epi {np.median(epi[sl]):8.0f} pro {np.median(pro[sl]):8.0f}")
