"""x6 (bf16x6) vs exact-f32 engine: numerics against an fp64 torch reference + layer timings.
Diagnostic tool (GPU)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

dev = torch.device("cuda:0")
N, B = 192, int(os.environ.get("B", "64"))
net = ImageCompressor(N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
w1, w2, w3, g1, g2 = net.Encoder.packed()
d1, d2, d3, q1, q2 = net.Decoder.packed()
torch.manual_seed(0)
a1 = torch.randn(B, 64, 64, N, device=dev) * 0.5
s1 = torch.randn(B, 32, 32, N, device=dev) * 0.5
a1s, s1s = kernels.split_planes(a1), kernels.split_planes(s1)
s2 = torch.randn(B, 64, 64, N, device=dev) * 0.3
s2s = kernels.split_planes(s2)
x0 = torch.rand(B, 3, 256, 256, device=dev)
e2 = net.Encoder.gdn2.effective_params_x6()
q2x = net.Decoder.igdn2.effective_params_x6()
assert torch.equal(kernels.merge_planes(a1s), a1), "split not exact"


def gdn64(x, gdn, inverse):
    beta = torch.clamp(gdn.beta.double(), min=float(gdn.beta_bound)) ** 2 - float(gdn.pedestal)
    gamma = torch.clamp(gdn.gamma.double(), min=float(gdn.gamma_bound)) ** 2 - float(gdn.pedestal)
    n = F.conv2d(x * x, gamma[:, :, None, None], beta)
    return x * torch.sqrt(n) if inverse else x / torch.sqrt(n)


def ref_conv2(x):   # x NHWC fp32 → NHWC fp64
    e = net.Encoder
    h = F.conv2d(x.permute(0, 3, 1, 2).double(), e.conv2.weight.double(), e.conv2.bias.double(), 2, 2)
    return gdn64(h, e.gdn2, False).permute(0, 2, 3, 1)


def ref_deconv2(x):
    d = net.Decoder
    h = F.conv_transpose2d(x.permute(0, 3, 1, 2).double(), d.deconv2.weight.double(),
                           d.deconv2.bias.double(), 2, 2, 1)
    return gdn64(h, d.igdn2, True).permute(0, 2, 3, 1)


def err(a, r):
    d = (a.double() - r).abs()
    return f"max|d|={d.max().item():.3e} rms={d.pow(2).mean().sqrt().item():.3e} (|ref| rms {r.pow(2).mean().sqrt().item():.3e})"


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[n // 2]


TIME_ONLY = os.environ.get("X6_TIME_ONLY") == "1"
TAG = os.environ.get("TAG", "")


def numerics():
    nb = 4   # numerics on a slice (fp64 reference cost)
    r2 = ref_conv2(a1[:nb])
    f32 = kernels.conv2_gdn(a1[:nb].contiguous(), w2, net.Encoder.conv2.bias, g2[0], g2[1])
    x6s, x6f, _ = kernels.conv2_gdn_x6(kernels.split_planes(a1[:nb].contiguous()), w2,
                                       net.Encoder.conv2.bias, *e2, want_f32=True)
    print("conv2_gdn  fp32:", err(f32, r2))
    print("conv2_gdn  x6  :", err(x6f, r2), " split==f32:", torch.equal(kernels.merge_planes(x6s), x6f))
    rd = ref_deconv2(s1[:nb])
    f32 = kernels.deconv_igdn(s1[:nb].contiguous(), d2, net.Decoder.deconv2.bias, q2[0], q2[1])
    _, x6f, _ = kernels.deconv_igdn_x6(kernels.split_planes(s1[:nb].contiguous()), d2,
                                       net.Decoder.deconv2.bias, *q2x, want_split=False,
                                       want_f32=True)
    print("deconv2_igdn fp32:", err(f32, rd))
    print("deconv2_igdn x6  :", err(x6f, rd))
    d = net.Decoder
    r3 = F.conv_transpose2d(s2[:nb].permute(0, 3, 1, 2).double(), d.deconv3.weight.double(),
                            d.deconv3.bias.double(), 4, 4, 3)
    _, f32, _ = kernels.deconv3(s2[:nb].contiguous(), d3, d.deconv3.bias, want_recon=True)
    _, x6r, _ = kernels.deconv3_x6(kernels.split_planes(s2[:nb].contiguous()), d.packed_x6(), d.deconv3.bias,
                                   want_recon=True)
    print("deconv3 fp32:", err(f32, r3))
    print("deconv3 x6  :", err(x6r, r3))


def timings():
    fl2 = 2.0 * B * (32 * 32 * N * N * 25 + 32 * 32 * N * N)
    fld = 2.0 * B * (32 * 32 * N * N * 25 + 64 * 64 * N * N)
    fl3 = 2.0 * B * 64 * 64 * N * 3 * 81
    fl1 = 2.0 * B * 64 * 64 * (N * 243 + N * N)
    e1 = net.Encoder.gdn1.effective_params_x6()
    w1x6 = net.Encoder.packed_conv1_x6()
    t = {
        "conv1 x6": (timeit(lambda: kernels.conv1_gdn_x6(x0, w1, net.Encoder.conv1.bias, g1[0], g1[1], N,
                                                         g6=e1[2])), fl1),
        "conv1 x6x6": (timeit(lambda: kernels.conv1x6_gdn(x0, w1x6, net.Encoder.conv1.bias, e1[0], e1[2], N)), fl1),
        "conv2 fp32": (timeit(lambda: kernels.conv2_gdn(a1, w2, net.Encoder.conv2.bias, g2[0], g2[1])), fl2),
        "conv2 x6": (timeit(lambda: kernels.conv2_gdn_x6(a1s, w2, net.Encoder.conv2.bias, *e2)), fl2),
        "deconv2 fp32": (timeit(lambda: kernels.deconv_igdn(s1, d2, net.Decoder.deconv2.bias, q2[0], q2[1])), fld),
        "deconv2 x6": (timeit(lambda: kernels.deconv_igdn_x6(s1s, d2, net.Decoder.deconv2.bias, *q2x,
                                                             want_split=False, want_f32=True)), fld),
        "deconv3 fp32": (timeit(lambda: kernels.deconv3(s2, d3, net.Decoder.deconv3.bias)), fl3),
        "deconv3 x6": (timeit(lambda: kernels.deconv3_x6(s2s, net.Decoder.packed_x6(), net.Decoder.deconv3.bias)), fl3),
    }
    print(TAG, " ".join(f"{k}={v[0]:.3f}ms({v[1] / v[0] / 1e9:.1f}TF)" for k, v in t.items()), flush=True)


with torch.no_grad():
    if not TIME_ONLY:
        numerics()
    timings()
