"""Times the h3 layers (B=64, N=192, the bench workload's shapes) — conv1+GDN1, conv2+GDN2,
conv3+quantiser, deconv1+IGDN1, deconv2+IGDN2, some beside their x6 forms — interleaved, with HIP
events; a short program for PMC passes (ONLY=name,name… selects)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

N, B = 192, 64
REPS = int(os.environ.get("REPS", "20"))
dev = torch.device("cuda", 0)
net = ImageCompressor(out_channel_N=N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
dec = net.Decoder
d1, d2 = dec.packed()[:2]
x1, x2 = dec.packed_h3k()[:2]
q1, q2 = dec.igdn1.effective_params_x6(), dec.igdn2.effective_params_x6()
h1, h2 = dec.igdn1.effective_params_h3(), dec.igdn2.effective_params_h3()
act = torch.from_numpy(synth.normal_like(6, (B, 32, 32, N), 0.7)).to(dev)
yq = torch.round(torch.from_numpy(synth.uniform(5, (B, 16, 16, N), -6, 6))).to(dev)
hs, ys = kernels.split_planes(act), kernels.split_planes(yq)
# each layer's input layout (kernels.CONV_CM / DECONV_CM chunk-major)
hh8, hh, yh = (kernels.h3_planes(act, cm=kernels.CONV_CM), kernels.h3_planes(act, cm=kernels.DECONV_CM),
               kernels.h3_planes(yq, cm=kernels.DECONV_CM))
enc = net.Encoder
w1h, (w2h, w3h) = enc.packed_conv1_h3(), enc.packed_h3()
ge1, ge2 = enc.gdn1.effective_params_h3(), enc.gdn2.effective_params_h3()
g1x = enc.gdn1.effective_params_x6()
img = torch.from_numpy(synth.uniform(7, (B, 3, 256, 256), 0.0, 1.0)).to(dev)
a1h = kernels.h3_planes(torch.from_numpy(synth.normal_like(8, (B, 64, 64, N), 0.7)).to(dev),
                        cm=kernels.CONV_CM)
rate, rtab = net.bitEstimator.packed(), net.bitEstimator.rate_table()
h64 = kernels.h3_planes(torch.from_numpy(synth.normal_like(11, (B, 64, 64, N), 0.7)).to(dev),
                        cm=kernels.DECONV3_CM)
hh8_32 = hh8[:, :32].contiguous()
a1h_32 = a1h[:, :32].contiguous()
yt32 = kernels.h3_planes(torch.from_numpy(synth.normal_like(10, (32, 16, 16, N), 2.0)).to(dev),
                         cm=kernels.DECONV_CM)
noise32 = torch.from_numpy(synth.uniform(9, (32, N, 16, 16), -0.5, 0.5)).to(dev)
runs = {
    "conv1_x6": lambda: kernels.conv1x6_gdn(img, enc.packed_conv1_x6(), enc.conv1.bias, g1x[0], g1x[2], N),
    "conv1_h3": lambda: kernels.conv1_gdn_h3(img, w1h, enc.conv1.bias, *ge1, N),
    "conv2_h3": lambda: kernels.conv2_gdn_h3(a1h, w2h, enc.conv2.bias, *ge2),
    # the training step's conv2 (B = 32: 8-row tiles) with its pre-activation and x6 outputs
    "conv2_h3_train32": lambda: kernels.conv2_gdn_h3(a1h_32, w2h, enc.conv2.bias, *ge2, want_x6=True,
                                                     want_pre=True),
    "conv3_h3": lambda: kernels.conv3_quant_rate_h3(hh8, w3h, rate, rtab=rtab),
    # the training step's conv3: noise mode at B = 32
    "conv3_h3_noise32": lambda: kernels.conv3_quant_rate_h3(hh8_32, w3h, rate, noise32),
    "deconv2_old": lambda: kernels.deconv_igdn_x6(hs, d2, dec.deconv2.bias, *q2, chunk_major=True),
    "deconv2_h3": lambda: kernels.deconv_igdn_h3(hh, x2, dec.deconv2.bias, *h2, want_h3=False,
                                                 want_x6=True, chunk_major=True),
    "deconv2_h3_h3out": lambda: kernels.deconv_igdn_h3(hh, x2, dec.deconv2.bias, *h2, chunk_major=True),
    "deconv3_h3": lambda: kernels.deconv3_h3(h64, dec.packed_h3k()[2], dec.deconv3.bias, x_ref=img),
    "deconv1_old": lambda: kernels.deconv_igdn_x6(ys, d1, dec.deconv1.bias, *q1),
    "deconv1_h3": lambda: kernels.deconv_igdn_h3(yh, x1, dec.deconv1.bias, *h1),
    # the training step's deconv1 (B = 32: 8-row tiles) on ỹ with its pre-activation and x6 outputs
    "deconv1_h3_train32": lambda: kernels.deconv_igdn_h3(yt32, x1, dec.deconv1.bias, *h1, want_x6=True,
                                                         want_pre=True),
    "deconv1_h3_int": lambda: kernels.deconv_igdn_h3(yh, x1, dec.deconv1.bias, *h1, int_in=True),
}
sel = os.environ.get("ONLY", "").split(",") if os.environ.get("ONLY") else list(runs)
with torch.no_grad():
    for k in sel:
        for _ in range(3):
            runs[k]()
    torch.cuda.synchronize()
    t = {k: [] for k in sel}
    for _ in range(REPS):
        for k in sel:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            runs[k]()
            e1.record()
            t[k].append((e0, e1))
    torch.cuda.synchronize()
for k in sel:
    ms = sorted(a.elapsed_time(b) for a, b in t[k])
    print(f"{k}: median {ms[len(ms) // 2]:.4f} ms, min {ms[0]:.4f}")


