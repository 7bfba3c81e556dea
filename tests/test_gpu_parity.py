"""GPU parity: every HIP kernel of the hot path against the CPU oracle (oracle/codec_ref.py,
itself pinned to the reference's outputs by tests/test_oracle_golden.py) and against the
reference-generated golden fixtures, called through the C ABI (libiclr17.so).

Bars (north_star): quantised latents bit-identical in round mode; bpp and PSNR within 1e-5
relative. Intermediate fp32 activations: max |Δ| ≤ 2e-5 · max |ref| (different but exact-f32
summation order on the MFMA).
"""
import json
import os

import numpy as np
import pytest
import torch

from iclr_17_compression_amd import _lib, kernels, synth
from iclr_17_compression_amd.model import ImageCompressor
from iclr_17_compression_amd.models import GDN, Analysis_net_17, BitEstimator, Synthesis_net_17
from oracle import codec_ref as oracle

pytestmark = pytest.mark.gpu

REL = 2e-5          # fp32 activations
METRIC_REL = 1e-5   # bpp / PSNR (north_star)


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def net_for(N, seed, device):
    net = ImageCompressor(out_channel_N=N)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, seed).items()})
    return net.to(device).eval()


def sd_for(N, seed):
    return oracle.state_dict_to_torch(synth.trained_like_state_dict(N, seed))


def image(seed, B, H, W):
    return torch.from_numpy(synth.to_unit_float(synth.image_u8(seed, B, H, W)))


def nhwc(t):
    return t.permute(0, 2, 3, 1)


def planes_nhwc(t):
    """A chunk-major h3 / split tensor [P,B,N/c,h,w,c] → NHWC planes [P,B,h,w,N] (bit patterns)."""
    P, B, nc, h, w, c = t.shape
    return t.permute(0, 1, 3, 4, 2, 5).reshape(P, B, h, w, nc * c)


@pytest.fixture(params=["h3", "x6", "fp32"])
def precision(request):
    """Run a test in each inference contraction mode (kernels.set_precision)."""
    old = kernels.precision()
    kernels.set_precision(request.param)
    yield request.param
    kernels.set_precision(old)


def test_split_planes_exact(device):
    """The x6 split is exact: hi + mid + lo == x bit for bit, each part a bf16."""
    x = torch.from_numpy(synth.normal_like(3, (4096,), 2.0)) * torch.from_numpy(
        np.exp(synth.uniform(4, (4096,), -30, 30)).astype(np.float32))
    x[:8] = torch.tensor([0.0, -0.0, 1.0, -1.0, 3.0e38, -1e-30, 0.1, 1 / 3])
    s = kernels.split_planes(x.to(device))
    assert s.shape == (3, 4096) and s.dtype == torch.int16
    assert torch.equal(kernels.merge_planes(s).cpu(), x)
    # each part is a bf16 (its fp32 image has zero low 16 bits) and |mid| ≤ 2^-8 |hi|
    parts = ((s.to(torch.int32) & 0xFFFF) << 16).view(torch.float32).cpu()
    hi, mid = parts[0].double(), parts[1].double()
    assert bool(((mid.abs() <= hi.abs() * 2.0 ** -7) | (hi == 0)).all())


@pytest.mark.parametrize("N", [192, 128])
def test_x6_layers(device, N):
    """x6-mode layers (split-form in/out) against the oracle, each from the oracle's input."""
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    F = torch.nn.functional
    x = image(11, 2, 64, 96)
    w1, w2, w3, g1, g2 = net.Encoder.packed()
    e1, e2 = net.Encoder.gdn1.effective_params_x6(), net.Encoder.gdn2.effective_params_x6()
    rate = net.bitEstimator.packed()
    with torch.no_grad():
        r_u1 = F.conv2d(x, sd["Encoder.conv1.weight"], sd["Encoder.conv1.bias"], stride=4, padding=4)
        r_a1 = oracle.gdn(r_u1, sd["Encoder.gdn1.beta"], sd["Encoder.gdn1.gamma"], False)
        for g6 in (None, e1[2]):   # exact-f32 GDN contraction, then the x6 one
            a1s, a1, u1 = kernels.conv1_gdn_x6(x.to(device), w1, net.Encoder.conv1.bias, g1[0], g1[1], N,
                                               want_f32=True, want_pre=True, g6=g6)
            assert rel_err(a1, nhwc(r_a1)) < REL and rel_err(u1, nhwc(r_u1)) < REL
            assert torch.equal(kernels.merge_planes(a1s), a1)
        a2s, a2, u2 = kernels.conv2_gdn_x6(kernels.split_planes(nhwc(r_a1).contiguous().to(device)), w2,
                                           net.Encoder.conv2.bias, *e2, want_f32=True, want_pre=True)
        r_u2 = F.conv2d(r_a1, sd["Encoder.conv2.weight"], sd["Encoder.conv2.bias"], stride=2, padding=2)
        r_a2 = oracle.gdn(r_u2, sd["Encoder.gdn2.beta"], sd["Encoder.gdn2.gamma"], False)
        assert rel_err(u2, nhwc(r_u2)) < REL and rel_err(a2, nhwc(r_a2)) < REL
        assert torch.equal(kernels.merge_planes(a2s), a2)
        y_hat, _, y, y_hat_s = kernels.conv3_quant_rate_x6(kernels.split_planes(nhwc(r_a2).contiguous().to(device)),
                                                           w3, rate, want_y=True)
        r_y = F.conv2d(r_a2, sd["Encoder.conv3.weight"], None, stride=2, padding=2)
        assert rel_err(y, nhwc(r_y)) < REL
        assert torch.equal(kernels.merge_planes(y_hat_s), y_hat)
        check_latents(y_hat.permute(0, 3, 1, 2), y.permute(0, 3, 1, 2), torch.round(r_y), r_y)
        # synthesis
        yq = torch.round(torch.from_numpy(synth.uniform(5, (2, N, 4, 6), -4, 4)))
        d1, d2 = net.Decoder.packed()[:2]
        q1, q2 = net.Decoder.igdn1.effective_params_x6(), net.Decoder.igdn2.effective_params_x6()
        s1s, s1, v1 = kernels.deconv_igdn_x6(kernels.split_planes(nhwc(yq).contiguous().to(device)), d1,
                                             net.Decoder.deconv1.bias, *q1,
                                             want_f32=True, want_pre=True)
        r_v1 = F.conv_transpose2d(yq, sd["Decoder.deconv1.weight"], sd["Decoder.deconv1.bias"], stride=2, padding=2,
                                  output_padding=1)
        r_s1 = oracle.gdn(r_v1, sd["Decoder.igdn1.beta"], sd["Decoder.igdn1.gamma"], True)
        assert rel_err(v1, nhwc(r_v1)) < REL and rel_err(s1, nhwc(r_s1)) < REL
        assert torch.equal(kernels.merge_planes(s1s), s1)
        _, s2, _ = kernels.deconv_igdn_x6(kernels.split_planes(nhwc(r_s1).contiguous().to(device)), d2,
                                          net.Decoder.deconv2.bias, *q2, want_split=False, want_f32=True)
        r_s2 = oracle.gdn(F.conv_transpose2d(r_s1, sd["Decoder.deconv2.weight"], sd["Decoder.deconv2.bias"],
                                             stride=2, padding=2, output_padding=1),
                          sd["Decoder.igdn2.beta"], sd["Decoder.igdn2.gamma"], True)
        assert rel_err(s2, nhwc(r_s2)) < REL


@pytest.mark.parametrize("N", [192, 128])
@pytest.mark.parametrize("shape", [(2, 64, 96), (1, 80, 112), (1, 256, 256)])
def test_conv1x6(device, N, shape):
    """conv1 + GDN1 with both contractions in x6 (reordered K, split patch in LDS, weight planes
    from L2) against the oracle; partial 8×8 tiles at 80×112."""
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    F = torch.nn.functional
    x = image(12, *shape)
    e1 = net.Encoder.gdn1.effective_params_x6()
    with torch.no_grad():
        r_u1 = F.conv2d(x, sd["Encoder.conv1.weight"], sd["Encoder.conv1.bias"], stride=4, padding=4)
        r_a1 = oracle.gdn(r_u1, sd["Encoder.gdn1.beta"], sd["Encoder.gdn1.gamma"], False)
        a1s, a1, u1 = kernels.conv1x6_gdn(x.to(device), net.Encoder.packed_conv1_x6(),
                                          net.Encoder.conv1.bias, e1[0], e1[2], N,
                                          want_f32=True, want_pre=True)
    assert rel_err(u1, nhwc(r_u1)) < REL and rel_err(a1, nhwc(r_a1)) < REL
    assert torch.equal(kernels.merge_planes(a1s), a1)


@pytest.mark.parametrize("N", [192, 128])
@pytest.mark.parametrize("shape", [(2, 64, 96), (1, 80, 112), (1, 256, 256)])
def test_deconv3_x6(device, N, shape):
    """The halo-tiled x6 deconv3 (16×16 base blocks, partial blocks at 80/112) against the
    oracle from the oracle's input: clipped / unclipped output and the per-8×8-tile SSE
    partials (both SSE modes) in the fp32 kernel's layout."""
    B, H, W = shape
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    F = torch.nn.functional
    d3, d3x6 = net.Decoder.packed()[2], net.Decoder.packed_x6()
    s2 = torch.from_numpy(synth.normal_like(21, (B, N, H // 4, W // 4), 0.6))
    x = image(12, B, H, W)
    with torch.no_grad():
        r_out = F.conv_transpose2d(s2, sd["Decoder.deconv3.weight"], sd["Decoder.deconv3.bias"],
                                   stride=4, padding=4, output_padding=3)
        hs = kernels.split_planes(nhwc(s2).contiguous().to(device))
        xd = x.to(device)
        for unclipped in (False, True):
            clipped, recon, part = kernels.deconv3_x6(hs, d3x6, net.Decoder.deconv3.bias, x_ref=xd,
                                                      want_recon=True, sse_unclipped=unclipped)
            assert rel_err(recon, r_out) < REL
            assert rel_err(clipped, r_out.clamp(0, 1)) < REL
            assert part.shape == (B, kernels.output_partials_per_image(H, W))
            per, _ = kernels.reduce_partials(part)
            ref = ((r_out if unclipped else r_out.clamp(0, 1)) - x.double()).pow(2).sum((1, 2, 3))
            assert rel_err(per, ref) < METRIC_REL
            # tile for tile against the fp32 kernel's partials
            _, _, part32 = kernels.deconv3(nhwc(s2).contiguous().to(device), d3,
                                           net.Decoder.deconv3.bias, x_ref=xd, want_recon=True,
                                           sse_unclipped=unclipped)
            assert rel_err(part, part32) < 1e-4
        c2, r2, p2 = kernels.deconv3_x6(hs, d3x6, net.Decoder.deconv3.bias)
        assert r2 is None and p2 is None and torch.equal(c2, clipped)


# ------------------------------------------------------------------------------------ layers
@pytest.mark.parametrize("N", [192, 128])
def test_analysis_layers(device, N):
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    x = image(11, 2, 64, 96)
    w1, w2, w3, g1, g2 = net.Encoder.packed()
    with torch.no_grad():
        a1, u1 = kernels.conv1_gdn(x.to(device), w1, net.Encoder.conv1.bias, g1[0], g1[1], N, want_pre=True)
        r_u1 = torch.nn.functional.conv2d(x, sd["Encoder.conv1.weight"], sd["Encoder.conv1.bias"], stride=4, padding=4)
        r_a1 = oracle.gdn(r_u1, sd["Encoder.gdn1.beta"], sd["Encoder.gdn1.gamma"], False)
        assert rel_err(u1, nhwc(r_u1)) < REL
        assert rel_err(a1, nhwc(r_a1)) < REL
        # next layer from the ORACLE's input so errors do not compound across the check
        a2, u2 = kernels.conv2_gdn(nhwc(r_a1).contiguous().to(device), w2, net.Encoder.conv2.bias,
                                   g2[0], g2[1], want_pre=True)
        r_u2 = torch.nn.functional.conv2d(r_a1, sd["Encoder.conv2.weight"], sd["Encoder.conv2.bias"], stride=2, padding=2)
        r_a2 = oracle.gdn(r_u2, sd["Encoder.gdn2.beta"], sd["Encoder.gdn2.gamma"], False)
        assert rel_err(u2, nhwc(r_u2)) < REL
        assert rel_err(a2, nhwc(r_a2)) < REL
        y = kernels.conv3(nhwc(r_a2).contiguous().to(device), w3)
        r_y = torch.nn.functional.conv2d(r_a2, sd["Encoder.conv3.weight"], None, stride=2, padding=2)
        assert rel_err(y, nhwc(r_y)) < REL


@pytest.mark.parametrize("N", [192, 128])
def test_synthesis_layers(device, N):
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    y = torch.round(torch.from_numpy(synth.uniform(5, (2, N, 4, 6), -4, 4)))
    d1, d2, d3, g1, g2 = net.Decoder.packed()
    F = torch.nn.functional
    with torch.no_grad():
        s1, v1 = kernels.deconv_igdn(nhwc(y).contiguous().to(device), d1, net.Decoder.deconv1.bias,
                                     g1[0], g1[1], want_pre=True)
        r_v1 = F.conv_transpose2d(y, sd["Decoder.deconv1.weight"], sd["Decoder.deconv1.bias"], stride=2, padding=2, output_padding=1)
        r_s1 = oracle.gdn(r_v1, sd["Decoder.igdn1.beta"], sd["Decoder.igdn1.gamma"], True)
        assert rel_err(v1, nhwc(r_v1)) < REL
        assert rel_err(s1, nhwc(r_s1)) < REL
        s2 = kernels.deconv_igdn(nhwc(r_s1).contiguous().to(device), d2, net.Decoder.deconv2.bias, g2[0], g2[1])
        r_s2 = oracle.gdn(F.conv_transpose2d(r_s1, sd["Decoder.deconv2.weight"], sd["Decoder.deconv2.bias"],
                                             stride=2, padding=2, output_padding=1),
                          sd["Decoder.igdn2.beta"], sd["Decoder.igdn2.gamma"], True)
        assert rel_err(s2, nhwc(r_s2)) < REL
        clipped, recon, _ = kernels.deconv3(nhwc(r_s2).contiguous().to(device), d3, net.Decoder.deconv3.bias,
                                            want_recon=True)
        r_out = F.conv_transpose2d(r_s2, sd["Decoder.deconv3.weight"], sd["Decoder.deconv3.bias"], stride=4, padding=4, output_padding=3)
        assert rel_err(recon, r_out) < REL
        assert rel_err(clipped, r_out.clamp(0, 1)) < REL


@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
@pytest.mark.parametrize("inverse", [False, True])
def test_gdn_module(device, layout, inverse):
    C = 192
    sd = sd_for(C, 2)
    key = "Decoder.igdn1" if inverse else "Encoder.gdn1"
    m = GDN(C, inverse=inverse)
    m.load_state_dict({"beta": sd[key + ".beta"], "gamma": sd[key + ".gamma"]})
    m = m.to(device).eval()
    x = torch.from_numpy(synth.normal_like(9, (2, C, 7, 13), 1.5))
    xd = x.to(device)
    if layout == "nhwc":
        xd = xd.contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(xd)
    ref = oracle.gdn(x, sd[key + ".beta"], sd[key + ".gamma"], inverse)
    assert rel_err(y, ref) < REL
    # 5-D input path of GDN.py:65-69
    with torch.no_grad():
        y5 = m(xd.contiguous().reshape(2, C, 7, 13, 1))
    assert rel_err(y5.reshape(2, C, 7, 13), ref) < REL


def test_bit_estimator_module(device, golden_dir):
    g = np.load(os.path.join(golden_dir, "g2_bit_estimator_n192.npz"), allow_pickle=False)
    sd = sd_for(192, 1)
    be = BitEstimator(192)
    be.load_state_dict({k[len("bitEstimator."):]: v for k, v in sd.items() if k.startswith("bitEstimator.")})
    be = be.to(device).eval()
    for tag in ("int", "noisy"):
        z = torch.from_numpy(g[f"z_{tag}"])
        with torch.no_grad():
            cdf = be(z.to(device))
            f1 = be.f1(z.to(device))
        assert rel_err(cdf, torch.from_numpy(g[f"cdf_{tag}"])) < 1e-5
        assert rel_err(f1, oracle.bitparm(z, sd["bitEstimator.f1.h"], sd["bitEstimator.f1.b"], sd["bitEstimator.f1.a"])) < 1e-6
        partial = kernels.rate_bits(z.to(device), be.packed())
        per, _ = kernels.reduce_partials(partial)
        assert per.sum().item() == pytest.approx(float(g[f"total_bits_{tag}"]), rel=METRIC_REL)


# ---------------------------------------------------------------------------------- end to end
def flips(a, b):
    return int((a.detach().cpu() != b.detach().cpu()).sum().item())


def reference_tie_band():
    """The reference's own largest |Δy| between its fp32 CPU summation orders on the G9 set
    (tests/golden/gen_g9s.py → g9s_reference_orders_n192.json, set_spread_fp32.max_abs_dy):
    a fixed bar from the reference's behaviour, not from the GPU's own error."""
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "golden", "g9s_reference_orders_n192.json")) as f:
        return json.load(f)["set_spread_fp32"]["max_abs_dy"]


def check_latents(y_hat, y, r_yhat, r_y, max_rate=1e-4):
    """ŷ must equal round(y_ref) bit for bit except at near-ties. The GPU's y must lie within the
    reference's own cross-order band of y_ref everywhere (max |y − y_ref| ≤ reference_tie_band()),
    and a flip is legitimate only where y_ref lies within that band of a rounding boundary k + ½.
    Returns the flip count."""
    band = reference_tie_band()
    y_hat, y = y_hat.detach().cpu(), y.detach().cpu()
    noise = (y - r_y).abs().max().item()
    assert noise <= band, (noise, band)
    diff = y_hat != r_yhat
    n = int(diff.sum())
    if n:
        dist = (r_y[diff] - (torch.floor(r_y[diff]) + 0.5)).abs()
        assert dist.max().item() <= band, (n, dist.max().item(), band)
        assert n <= max_rate * r_yhat.numel(), n
    return n


def test_c1_golden_end_to_end(device, precision, golden_dir):
    g = np.load(os.path.join(golden_dir, "g3_c1_n192_256px.npz"), allow_pickle=False)
    meta = json.load(open(os.path.join(golden_dir, "g3_c1_n192_256px.json")))
    net = net_for(192, 1, device)
    x = image(0, 1, 256, 256).to(device)
    with torch.no_grad():
        clipped, y_hat, bpp = net(x)
        ev = net.evaluate(x)
    assert y_hat.shape == (1, 192, 16, 16)
    ref = torch.from_numpy(g["y_hat"].astype(np.float32))
    assert flips(y_hat, ref) == 0
    assert bpp.item() == pytest.approx(meta["bpp"], rel=METRIC_REL)
    assert ev["bpp"][0].item() == pytest.approx(meta["bpp"], rel=METRIC_REL)
    assert ev["mse"][0].item() == pytest.approx(meta["mse_clipped"], rel=METRIC_REL)
    assert ev["psnr"][0].item() == pytest.approx(meta["psnr"], rel=METRIC_REL)
    mse = torch.mean((clipped - x) ** 2).item()
    assert mse == pytest.approx(meta["mse_clipped"], rel=METRIC_REL)
    # the stand-alone Encoder / Decoder modules (NewTests/testReconSeperateEandD.py:67-68)
    with torch.no_grad():
        y = net.Encoder(x)
        assert rel_err(y, torch.from_numpy(g["y"])) < REL
        recon = net.Decoder(torch.round(y))
    assert rel_err(recon[:, :, :64, :64], torch.from_numpy(g["recon_crop"])) < REL


@pytest.mark.parametrize("N,B,H,W", [(192, 3, 48, 80), (128, 2, 16, 16), (192, 1, 16, 48), (128, 2, 96, 64)])
def test_module_shapes_vs_oracle(device, precision, N, B, H, W):
    net, sd = net_for(N, 4, device), sd_for(N, 4)
    x = image(7, B, H, W)
    with torch.no_grad():
        clipped, y_hat, bpp = net(x.to(device))
        y = net.run(x.to(device), want_y=True)["y"].permute(0, 3, 1, 2)
    r_clipped, r_yhat, r_bpp, _, r_y = oracle.codec_forward(x, sd)
    check_latents(y_hat, y, r_yhat, r_y)
    assert bpp.item() == pytest.approx(r_bpp.item(), rel=METRIC_REL)
    assert rel_err(clipped, r_clipped) < REL


def test_training_mode_noise(device, precision):
    N = 192
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    x = image(3, 2, 64, 64)
    noise = torch.from_numpy(synth.uniform(4, (2, N, 4, 4), -0.5, 0.5))
    net.train()
    with torch.no_grad():
        clipped, y_tilde, bpp = net(x.to(device), noise=noise.to(device))
    r_clipped, r_ytilde, r_bpp, _, _ = oracle.codec_forward(x, sd, training=True, noise=noise)
    assert rel_err(y_tilde, r_ytilde) < REL
    assert bpp.item() == pytest.approx(r_bpp.item(), rel=METRIC_REL)
    assert rel_err(clipped, r_clipped) < REL


def test_kodak_synth_subset(device, precision, golden_dir):
    meta = json.load(open(os.path.join(golden_dir, "g5_kodak24_synth_n192.json")))
    net, sd = net_for(meta["N"], meta["weight_seed"], device), sd_for(meta["N"], meta["weight_seed"])
    for row in [meta["images"][i] for i in (0, 3, 9, 23)]:
        x = torch.from_numpy(synth.to_unit_float(
            synth.smooth_image_u8(meta["image_seed_base"] + row["index"], row["height"], row["width"])))[None]
        ev = net.evaluate(x.to(device), want_y=True, want_msssim=True)
        assert ev["bpp"][0].item() == pytest.approx(row["bpp"], rel=METRIC_REL)
        assert ev["psnr"][0].item() == pytest.approx(row["psnr"], rel=METRIC_REL)
        # MS-SSIM kernel parity on the same pair (GPU recon, x) against the oracle restatement
        r_ms = oracle.ms_ssim(ev["clipped"].cpu(), x, 1.0)
        assert ev["ms_ssim"][0].item() == pytest.approx(r_ms.item(), rel=1e-5)
        # end to end against the reference's value: these ~6.6 dB reconstructions give
        # MS-SSIM ≈ 0.02, a product whose relative error is Σ w_l·δcs_l / cs_l with small cs_l,
        # so recon-level fp32 differences are amplified; the bar is 1e-3 relative here
        assert ev["ms_ssim"][0].item() == pytest.approx(row["ms_ssim"], rel=1e-3)
        _, r_yhat, _, _, r_y = oracle.codec_forward(x, sd)
        n = check_latents(ev["y_hat"], ev["y"], r_yhat, r_y)
        print(f"kodak-synth[{row['index']}] {precision}: {n} near-tie latent flips of {r_yhat.numel()}")


def test_determinism_and_batch_independence(device, precision):
    net = net_for(192, 1, device)
    x = image(21, 4, 64, 64).to(device)
    ev1 = net.evaluate(x)
    ev2 = net.evaluate(x)
    for k in ("clipped", "y_hat", "bpp", "mse"):
        assert torch.equal(ev1[k], ev2[k]), k
    # per-image results do not depend on the batch an image sits in (sharding by image is exact)
    for i in range(4):
        evi = net.evaluate(x[i:i + 1])
        assert torch.equal(evi["y_hat"][0], ev1["y_hat"][i])
        assert torch.equal(evi["bpp"][0], ev1["bpp"][i])
        assert torch.equal(evi["clipped"][0], ev1["clipped"][i])


def test_evaluate_many_matches_sequential(device, precision):
    """evaluate_many (batches of different shapes on concurrent streams, as the Kodak bench runs
    landscape and portrait images) gives bitwise the sequential evaluate() results."""
    net = net_for(192, 1, device)
    land = image(31, 2, 192, 256).to(device)   # MS-SSIM's 5 levels need ≥ 176 px per side
    port = image(32, 1, 256, 192).to(device)
    seq = [net.evaluate(b, want_msssim=True) for b in (land, port)]
    for _ in range(2):
        many = net.evaluate_many([land, port], want_msssim=True)
        torch.cuda.synchronize()
        for a, b in zip(many, seq):
            for k in ("clipped", "y_hat", "bpp", "mse", "psnr", "ms_ssim"):
                assert torch.equal(a[k], b[k]), k


def test_ms_ssim_vs_reference_fixture(device, golden_dir):
    """GPU MS-SSIM against the reference's values on the G6 pairs (incl. odd pyramid levels and
    B = 2). The fp32 filter sums run in another order than oneDNN's, so the bar is 1e-5 rel."""
    meta = json.load(open(os.path.join(golden_dir, "g6_ms_ssim.json")))
    for c in meta["cases"]:
        x8, y8 = synth.noisy_pair_u8(c["B"], c["H"], c["W"], c["image_seed"], c["noise_seed"], c["noise_div"])
        x, y = (torch.from_numpy(synth.to_unit_float(a)).to(device) for a in (x8, y8))
        got = kernels.ms_ssim(y, x, 1.0).cpu()
        assert got.tolist() == pytest.approx(c["ms_ssim"], rel=1e-5), (c, got)
        assert torch.equal(kernels.ms_ssim(y, x, 1.0).cpu(), got)   # deterministic


def test_ms_ssim_vs_oracle(device):
    """Random pairs, three sizes, against the oracle restatement."""
    for (B, H, W) in [(3, 176, 192), (1, 256, 256), (2, 333, 181)]:
        x = torch.from_numpy(synth.uniform(31, (B, 3, H, W)))
        y = (x + torch.from_numpy(synth.normal_like(32, (B, 3, H, W), 0.05))).clamp(0, 1)
        ref = oracle.ms_ssim(y, x, 1.0)
        got = kernels.ms_ssim(y.to(device), x.to(device), 1.0).cpu()
        assert got.tolist() == pytest.approx(ref.tolist(), rel=1e-5), (B, H, W, got, ref)
    with pytest.raises(_lib.Iclr17Error, match="too small"):
        kernels.ms_ssim(torch.rand(1, 3, 64, 64, device=device), torch.rand(1, 3, 64, 64, device=device))


def test_errors_are_loud(device):
    net = net_for(192, 1, device)
    with pytest.raises(_lib.Iclr17Error, match="multiples of 16"):
        net(torch.rand(1, 3, 40, 64, device=device))
    with pytest.raises(_lib.Iclr17Error, match="float32"):
        net(torch.rand(1, 3, 64, 64, device=device, dtype=torch.float64))


def test_c5_2048_full_size_properties(device):
    """C5's full image size (2048×2048, N=192), through properties that do not need a CPU
    reference of that size: the h3 (the default) and x6 modes each agree with the exact-f32 mode
    (latents bit for bit except at near-ties of the fp32 y, bpp / PSNR within 1e-5 relative); an
    image's results do not depend on its batch; compress → decompress returns the latents and
    reconstruction bit for bit. At 2048² the activations are 512² per channel, where the h3 range
    flag (|x| ≥ 2^22) matters most: it must stay clear."""
    net = net_for(192, 1, device)
    x = image(41, 2, 2048, 2048).to(device)
    old = kernels.precision()
    res = {}
    try:
        kernels.set_precision("fp32")
        ev32 = net.evaluate(x[:1], want_y=True)
        for mode in ("h3", "x6"):
            kernels.set_precision(mode)
            ev = net.evaluate(x[:1], want_y=True)
            evb = net.evaluate(x)                      # the same image inside a batch of two
            enc = net.compress(x[:1])
            dec = net.decompress(enc["strings"], enc["shape"])
            res[mode] = (ev, evb, dec)
        kernels.check_h3_range(device)
    finally:
        kernels.set_precision(old)
    for mode, (ev, evb, dec) in res.items():
        n = check_latents(ev["y_hat"], ev["y"], ev32["y_hat"].cpu(), ev32["y"].cpu())
        print(f"{mode} vs fp32 near-tie flips at 2048²: {n}; rel bpp "
              f"{abs(ev['bpp'].item() / ev32['bpp'].item() - 1):.2e}, rel PSNR "
              f"{abs(ev['psnr'].item() / ev32['psnr'].item() - 1):.2e}")
        assert ev["bpp"].item() == pytest.approx(ev32["bpp"].item(), rel=METRIC_REL)
        assert ev["psnr"].item() == pytest.approx(ev32["psnr"].item(), rel=METRIC_REL)
        for k in ("y_hat", "bpp", "clipped"):
            assert torch.equal(evb[k][0], ev[k][0]), (mode, k)
        assert torch.equal(dec["y_hat"].cpu(), ev["y_hat"].cpu()), mode
        assert torch.equal(dec["x_hat"].cpu(), ev["clipped"].cpu()), mode


def test_batched_packs_match_single(device):
    """kernels.batched_packs (iclr17_pack_batch: every layout of a parameter update in two
    launches, more than one launch's worth of jobs) gives bitwise the single-pack results."""
    net = net_for(192, 1, device)
    enc, dec, be = net.Encoder, net.Decoder, net.bitEstimator
    g = enc.gdn1

    def all_packs():
        out = []
        for _ in range(4):   # 22 first-phase jobs: more than one launch of the batch kernel
            out += [kernels.pack_weight(_lib.ICLR17_W_CONV1, enc.conv1.weight, 192),
                    kernels.pack_weight(_lib.ICLR17_W_CONV5, enc.conv2.weight, 192),
                    kernels.pack_weight(_lib.ICLR17_W_DECONV5, dec.deconv1.weight, 192),
                    kernels.pack_weight(_lib.ICLR17_W_DECONV9, dec.deconv3.weight, 192),
                    kernels.pack_conv1_x6(enc.conv1.weight, 192)]
        bb, gb, ped = g.bounds_f32()
        be_, gp, gpt = kernels.pack_gdn(g.beta, g.gamma, bb, gb, ped, transposed=True)
        out += [be_, gp, gpt, kernels.split_packed(gp, 1, 192, 192), kernels.split_packed(gpt, 1, 192, 192),
                kernels.pack_rate(be.params_in_order())]
        return out

    single = all_packs()
    with kernels.batched_packs():
        batched = all_packs()
    torch.cuda.synchronize()
    assert len(single) == len(batched)
    for a, b in zip(single, batched):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N", [128, 192])
def test_batched_h3_packs_match_single(device, N):
    """kernels.batched_h3_packs (iclr17_pack_h3_batch: the max pass and the packing pass of
    every job in one launch each; more jobs than one call holds, one all-zero tensor) gives
    bitwise the single-pack results, trailer included."""
    net = net_for(N, 1, device)
    enc, dec = net.Encoder, net.Decoder
    gp = enc.gdn1.effective_params()[1]
    w3 = enc.packed()[2]
    d3 = dec.packed()[2]
    zero = torch.zeros_like(dec.deconv2.weight)

    def all_packs():
        out = []
        for _ in range(3):   # 21 jobs: two batch calls
            out += [kernels.pack_h3k(_lib.ICLR17_H3K_CONV1, enc.conv1.weight, N),
                    kernels.pack_h3k(_lib.ICLR17_H3K_CONV5, enc.conv2.weight, N),
                    kernels.pack_h3k(_lib.ICLR17_H3K_DECONV5, dec.deconv1.weight, N),
                    kernels.split_packed_h3(w3, 25, N, N),
                    kernels.split_packed_h3(d3, 9, N, 48),
                    kernels.split_packed_h3(gp, 1, N, N)]
        out.append(kernels.pack_h3k(_lib.ICLR17_H3K_DECONV5, zero, N))
        return out

    single = all_packs()
    with kernels.batched_h3_packs():
        batched = all_packs()
    torch.cuda.synchronize()
    assert len(single) == len(batched)
    for a, b in zip(single, batched):   # the trailer's last 8 bytes are padding, never written
        assert torch.equal(a[:-4], b[:-4])
    assert float(batched[-1][-8:].view(torch.float32)[0]) == 0.0   # max|w| of the zero tensor


@pytest.mark.parametrize("mode", ["h3", "x6", "fp32", "bf16"])
def test_encoder_matches_codec_forward(device, mode):
    """The separate encode / decode path (NewTests/testReconSeperateEandD.py:67-68): in every
    precision ``torch.round(net.Encoder(x))`` is bitwise the codec forward's ŷ, the latents are
    contiguous NCHW like the reference's (model.py:56, 80) so ``.view(B, -1)`` works
    (model_fc.py:60), and Decoder(round(Encoder(x))) is the forward's reconstruction."""
    old = kernels.precision()
    kernels.set_precision(mode)
    try:
        net = net_for(192, 1, device)
        x = image(5, 2, 64, 96).to(device)
        with torch.no_grad():
            y = net.Encoder(x)
            clipped, y_hat, _ = net(x)
            recon = net.Decoder(torch.round(y))
    finally:
        kernels.set_precision(old)
    assert y.is_contiguous() and y_hat.is_contiguous() and y.shape == (2, 192, 4, 6)
    assert y.view(2, -1).shape == (2, 192 * 24) and y_hat.view(2, -1).shape == (2, 192 * 24)
    assert torch.equal(torch.round(y), y_hat)
    assert torch.equal(recon.clamp(0.0, 1.0), clipped)


@pytest.mark.parametrize("mode", ["h3", "x6", "fp32", "bf16"])
def test_encoder_with_grad_matches_codec_forward(device, mode):
    """NewTests/testReconSeperateEandD.py:67 calls ``torch.round(net.Encoder(x))`` with autograd
    ON, which takes AnalysisFn: its y must be the codec's own (same analysis kernels), contiguous
    NCHW, and still carry a gradient into the encoder."""
    old = kernels.precision()
    kernels.set_precision(mode)
    try:
        net = net_for(192, 1, device)
        x = image(5, 2, 64, 96).to(device)
        y = net.Encoder(x)
        assert y.requires_grad
        with torch.no_grad():
            _, y_hat, _ = net(x)
            y_ng = net.Encoder(x)
        y.sum().backward()
    finally:
        kernels.set_precision(old)
    assert y.is_contiguous() and y.shape == (2, 192, 4, 6)
    assert torch.equal(y.detach(), y_ng)
    assert torch.equal(torch.round(y.detach()), y_hat)
    assert net.Encoder.conv1.weight.grad is not None
    assert torch.isfinite(net.Encoder.conv1.weight.grad).all()


@pytest.mark.parametrize("N", [192, 128])
def test_chunk_major_split_deconv2_to_deconv3(device, N):
    """deconv2+IGDN2 writing the chunk-major split form [3,B,N/32,h,w,32] (what deconv3's halo
    kernel reads without sharing cache lines between chunks) holds exactly the NHWC split's
    values, and deconv3_x6 gives bit-identical outputs from either form."""
    net = net_for(N, 3, device)
    dec = net.Decoder
    d1, d2, d3, q1, q2 = dec.packed()
    e2 = dec.igdn2.effective_params_x6()
    torch.manual_seed(0)
    h1 = (torch.randn(2, 8, 12, N) * 0.5).to(device)
    hs = kernels.split_planes(h1)
    with torch.no_grad():
        s_nhwc, f_nhwc, _ = kernels.deconv_igdn_x6(hs, d2, dec.deconv2.bias, *e2, want_f32=True)
        s_cm, f_cm, _ = kernels.deconv_igdn_x6(hs, d2, dec.deconv2.bias, *e2, want_f32=True,
                                               chunk_major=True)
        assert s_cm.shape == (3, 2, N // 32, 16, 24, 32)
        assert torch.equal(f_nhwc, f_cm)
        assert torch.equal(kernels.merge_planes(s_cm), kernels.merge_planes(s_nhwc))
        x = image(9, 2, 64, 96).to(device)
        a = kernels.deconv3_x6(s_nhwc, dec.packed_x6(), dec.deconv3.bias, x_ref=x, want_recon=True)
        b = kernels.deconv3_x6(s_cm, dec.packed_x6(), dec.deconv3.bias, x_ref=x, want_recon=True)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_h3_planes(device):
    """The h3 form (common.h): hi + lo·2^-11 reproduces x·2^-6 to 2^-22 relative (22 significant
    bits) wherever lo is a normal fp16, hi is the RNE fp16 of x·2^-6, small values keep an
    absolute error below 2^-36·2^6, and a value of magnitude ≥ 2^22 sets the range flag."""
    x = torch.from_numpy(synth.normal_like(3, (8192,), 2.0)) * torch.from_numpy(
        np.exp(synth.uniform(4, (8192,), -20, 12)).astype(np.float32))
    x[:8] = torch.tensor([0.0, -0.0, 1.0, -1.0, 4.0e6, -1e-30, 0.1, 1 / 3])
    flag = kernels.h3_range_flag(device)
    flag.zero_()
    s = kernels.h3_planes(x.to(device))
    assert s.shape == (2, 8192) and s.dtype == torch.int16
    assert int(flag.item()) == 0
    back = kernels.merge_h3(s).cpu().double()
    xd = x.double()
    err = (back - xd).abs()
    assert bool((err <= torch.maximum(xd.abs() * 2.0 ** -22, torch.full_like(xd, 2.0 ** -30))).all())
    hi = s[0].view(torch.float16).float().cpu()
    assert torch.equal(hi, (x * 2.0 ** -6).to(torch.float16).float())
    big = torch.tensor([1.0, 2.0 ** 22 * 1.01, -3.0, 5.0], device=device)
    kernels.h3_planes(big)
    assert int(flag.item()) == 1
    with pytest.raises(kernels.Iclr17Error):
        kernels.check_h3_range(device)
    assert int(flag.item()) == 1   # sticky until the next chain begins
    kernels.h3_chain_begin(device)
    assert int(flag.item()) == 0


@pytest.mark.parametrize("N", [192, 128])
def test_h3_encoder_layers(device, N):
    """conv1 / conv2 / conv3 of the h3 chain against the oracle, each from the oracle's input:
    conv1's h3 output is the h3 form of its fp32 output; conv2+GDN2 in the h3 form (three fp16
    part products per MAC, per-tap two-level accumulation) at the fp32 bar and as close to the x6
    conv2 as two fp32 summation orders, with its h3 / x6 outputs encoding its fp32 output exactly;
    conv3 + quantiser + rate: y at the fp32 bar, latents within the reference's own near-tie band,
    ŷ's h3 form exact, bits equal to the x6 kernel's up to summation order."""
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    F = torch.nn.functional
    x = image(11, 2, 64, 96)
    w1, w2, w3, g1, g2 = net.Encoder.packed()
    w2h, w3h = net.Encoder.packed_h3()
    e1, e2 = net.Encoder.gdn1.effective_params_x6(), net.Encoder.gdn2.effective_params_x6()
    h1, h2 = net.Encoder.gdn1.effective_params_h3(), net.Encoder.gdn2.effective_params_h3()
    rate, rtab = net.bitEstimator.packed(), net.bitEstimator.rate_table()
    flag = kernels.h3_range_flag(device)
    flag.zero_()
    with torch.no_grad():
        a1h, a1 = kernels.conv1_gdn_h3(x.to(device), net.Encoder.packed_conv1_h3(), net.Encoder.conv1.bias,
                                       *h1, N, want_f32=True)
        _, a1x6, _ = kernels.conv1x6_gdn(x.to(device), net.Encoder.packed_conv1_x6(), net.Encoder.conv1.bias,
                                         e1[0], e1[2], N, want_f32=True)
        assert rel_err(a1, a1x6) < 2e-6 and torch.equal(a1h, kernels.h3_planes(a1, cm=kernels.CONV_CM))
        r_u1 = F.conv2d(x, sd["Encoder.conv1.weight"], sd["Encoder.conv1.bias"], stride=4, padding=4)
        r_a1 = oracle.gdn(r_u1, sd["Encoder.gdn1.beta"], sd["Encoder.gdn1.gamma"], False)
        assert rel_err(a1, nhwc(r_a1)) < REL
        a1r = nhwc(r_a1).contiguous().to(device)
        a2h, a2, a2s = kernels.conv2_gdn_h3(kernels.h3_planes(a1r, cm=kernels.CONV_CM), w2h, net.Encoder.conv2.bias, *h2,
                                            want_f32=True, want_x6=True)
        r_u2 = F.conv2d(r_a1, sd["Encoder.conv2.weight"], sd["Encoder.conv2.bias"], stride=2, padding=2)
        r_a2 = oracle.gdn(r_u2, sd["Encoder.gdn2.beta"], sd["Encoder.gdn2.gamma"], False)
        assert rel_err(a2, nhwc(r_a2)) < REL
        assert torch.equal(kernels.merge_planes(a2s), a2) and torch.equal(a2h, kernels.h3_planes(a2, cm=kernels.CONV_CM))
        _, a2x6, _ = kernels.conv2_gdn_x6(kernels.split_planes(a1r), w2, net.Encoder.conv2.bias, *e2,
                                          want_f32=True)
        assert rel_err(a2, a2x6) < 2e-6
        a2r = nhwc(r_a2).contiguous().to(device)
        y_hat, part, y, yh = kernels.conv3_quant_rate_h3(kernels.h3_planes(a2r, cm=kernels.CONV_CM), w3h, rate, want_y=True,
                                                         rtab=rtab)
        r_y = F.conv2d(r_a2, sd["Encoder.conv3.weight"], None, stride=2, padding=2)
        assert rel_err(y, nhwc(r_y)) < REL
        assert torch.equal(yh, kernels.h3_planes(y_hat, cm=kernels.DECONV_CM))
        check_latents(y_hat.permute(0, 3, 1, 2), y.permute(0, 3, 1, 2), torch.round(r_y), r_y)
        yx, px, _, _ = kernels.conv3_quant_rate_x6(kernels.split_planes(a2r), w3, rate, rtab=rtab)
        if torch.equal(yx, y_hat):
            # fp32 per-lane bit sums grouped by the h3 engine's tiles vs the x6 kernel's
            assert abs(part.sum().item() - px.sum().item()) <= 1e-6 * px.sum().item()
    assert int(flag.item()) == 0


@pytest.mark.parametrize("N", [192, 128])
@pytest.mark.parametrize("hw", [(5, 7), (20, 34)])
def test_h3_deconv_igdn(device, N, hw):
    """deconv + IGDN in the h3 form (csrc/engine_h3.hip: three fp16 part products per MAC on the
    32x32x16 f16 MFMA) against the oracle (synthesis_17.py:15-22, GDN.py:64-94 inverse), on grids
    that are and are not whole 16×16 tiles: the fp32 output at the fp32 bar and as close to the
    x6 engine as two exact-f32 summation orders; its h3 and x6 outputs encode exactly that fp32
    output, in NHWC and chunk-major form; on ŷ the int_in form (hi plane only, two products) is
    bit-identical to the full form, also with a latent beyond fp16's 11 bits. The IGDN
    contraction runs in the h3 form too (per-pixel power-of-two scale of x²)."""
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    dec = net.Decoder
    F = torch.nn.functional
    h, w = hw
    x1, x2 = dec.packed_h3k()[:2]
    d1, d2 = dec.packed()[:2]
    q1, q2 = dec.igdn1.effective_params_x6(), dec.igdn2.effective_params_x6()
    h1, h2 = dec.igdn1.effective_params_h3(), dec.igdn2.effective_params_h3()
    yq = torch.round(torch.from_numpy(synth.uniform(5, (2, N, h, w), -6, 6)))
    act = torch.from_numpy(synth.normal_like(6, (2, N, h, w), 0.7))
    flag = kernels.h3_range_flag(device)
    flag.zero_()
    with torch.no_grad():
        for inp, lay, wx, wp, q, qh, key in ((yq, "deconv1", x1, d1, q1, h1, "igdn1"),
                                             (act, "deconv2", x2, d2, q2, h2, "igdn2")):
            inh = kernels.h3_planes(nhwc(inp).contiguous().to(device), cm=kernels.DECONV_CM)
            bias = getattr(dec, lay).bias
            s, f, s6 = kernels.deconv_igdn_h3(inh, wx, bias, *qh, want_f32=True, want_x6=True)
            r_v = F.conv_transpose2d(inp, sd[f"Decoder.{lay}.weight"], sd[f"Decoder.{lay}.bias"],
                                     stride=2, padding=2, output_padding=1)
            r_s = oracle.gdn(r_v, sd[f"Decoder.{key}.beta"], sd[f"Decoder.{key}.gamma"], True)
            assert f.shape == (2, 2 * h, 2 * w, N)
            assert rel_err(f, nhwc(r_s)) < REL, lay
            assert torch.equal(kernels.merge_planes(s6), f)
            assert torch.equal(s, kernels.h3_planes(f, cm=kernels.DECONV_CM))
            scm, _, s6cm = kernels.deconv_igdn_h3(inh, wx, bias, *qh, want_x6=True,
                                                  chunk_major=True)
            assert scm.shape == (2, 2, N // 32, 2 * h, 2 * w, 32)
            assert s.shape == (2, 2, N // 16, 2 * h, 2 * w, 16)
            assert torch.equal(planes_nhwc(scm), planes_nhwc(s))   # the same planes, two layouts
            assert torch.equal(s6cm, s6)   # the x6 output stays NHWC
            _, f_old, _ = kernels.deconv_igdn_x6(kernels.split_planes(nhwc(inp).contiguous().to(device)),
                                                 wp, bias, *q, want_f32=True)
            assert rel_err(f, f_old) < 2e-6, lay
            if lay == "deconv1":
                si, fi, _ = kernels.deconv_igdn_h3(inh, wx, bias, *qh, want_f32=True, int_in=True)
                assert torch.equal(fi, f) and torch.equal(si, s)
                # a latent beyond fp16's 11 significant bits (3001): the workgroups that see it
                # run the three-product form, and the result still equals the full form's
                big = inp.clone()
                big[1, 7, h // 2, w // 2] = 3001.0
                bs = kernels.h3_planes(nhwc(big).contiguous().to(device), cm=kernels.DECONV_CM)
                _, fb, _ = kernels.deconv_igdn_h3(bs, wx, bias, *qh, want_h3=False, want_f32=True)
                _, fbi, _ = kernels.deconv_igdn_h3(bs, wx, bias, *qh, want_h3=False, want_f32=True,
                                                   int_in=True)
                assert torch.equal(fbi, fb) and not torch.equal(fb, f)
    assert int(flag.item()) == 0


@pytest.mark.parametrize("N", [192, 128])
def test_h3_deconv3(device, N):
    """deconv3 + clamp on the chunk-major h3 input (three fp16 part products per MAC) against the
    oracle's conv_transpose2d + clamp from the same activation, at the fp32 bar, and against the x6
    halo kernel to two-summation-order noise; the SSE partials and the folded bit reduction agree
    with their separate kernels."""
    net, sd = net_for(N, 3, device), sd_for(N, 3)
    dec = net.Decoder
    h = torch.from_numpy(synth.normal_like(7, (2, N, 16, 24), 0.5))
    x = image(9, 2, 64, 96).to(device)
    hh = kernels.h3_planes(nhwc(h).contiguous().to(device))
    hcm = hh.reshape(2, 2, 16, 24, N // 32, 32).permute(0, 1, 4, 2, 3, 5).contiguous()
    w3 = dec.packed_h3k()[2]
    torch.manual_seed(1)
    part = (torch.rand(2, 5, dtype=torch.float64) * 50.0).to(device)
    with torch.no_grad():
        c, r, sse = kernels.deconv3_h3(hcm, w3, dec.deconv3.bias, x_ref=x, want_recon=True)
        c2, r2, sse2, tot = kernels.deconv3_h3(hcm, w3, dec.deconv3.bias, x_ref=x, want_recon=True,
                                               bits=(part, 1.0 / 777.0))
        ref_r = torch.nn.functional.conv_transpose2d(kernels.merge_h3(hh).permute(0, 3, 1, 2).cpu(),
                                                     sd["Decoder.deconv3.weight"], sd["Decoder.deconv3.bias"],
                                                     stride=4, padding=4, output_padding=3)
        s6 = kernels.split_planes(nhwc(h).contiguous().to(device))
        s6cm = s6.reshape(3, 2, 16, 24, N // 32, 32).permute(0, 1, 4, 2, 3, 5).contiguous()
        c6, r6, _ = kernels.deconv3_x6(s6cm, dec.packed_x6(), dec.deconv3.bias, x_ref=x, want_recon=True)
    assert rel_err(r, ref_r) < REL and torch.equal(c.cpu(), ref_r.clamp(0, 1)) or rel_err(c, ref_r.clamp(0, 1)) < REL
    assert rel_err(r, r6) < 2e-6
    assert torch.equal(c, c2) and torch.equal(r, r2) and torch.equal(sse, sse2)
    _, ref_tot = kernels.reduce_partials(part, 1.0 / 777.0, per_image=False)
    assert torch.equal(tot, ref_tot)
    d = (c - x).double()
    assert abs(sse.sum().item() - (d * d).sum().item()) <= 1e-6 * (d * d).sum().item()


@pytest.mark.parametrize("N,B,hw", [(192, 3, (48, 80)), (128, 2, (32, 32)), (192, 40, (32, 32))])
def test_conv3_x6_presplit_weights(device, N, B, hw):
    """x6 conv3 reading its weights pre-split (iclr17_analysis_conv3_quant_rate_x6w, split_packed
    once) equals the per-k-step split bit for bit — ŷ, y, the split ŷ and the bit partials — in
    round mode and in noise mode (48-column tiles below 256 tiles·images, 4 partials per tile;
    B=40 stays on them, N=128 never does); and its y agrees with the oracle's conv3."""
    net = net_for(N, 1, device)
    enc = net.Encoder
    w3, w3s = enc.packed()[2], enc.packed_w3_split()
    rate, rtab = net.bitEstimator.packed(), net.bitEstimator.rate_table()
    h, w = hw
    a2 = torch.from_numpy(synth.normal_like(21, (B, h, w, N), 0.7))
    hs = kernels.split_planes(a2.to(device))
    noise = torch.from_numpy(synth.uniform(22, (B, N, h // 2, w // 2), -0.5, 0.5)).to(device)
    for nz in (None, noise):
        kw = dict(want_y=True, rtab=rtab if nz is None else None)
        a = kernels.conv3_quant_rate_x6(hs, w3, rate, nz, **kw)
        b = kernels.conv3_quant_rate_x6(hs, w3, rate, nz, w_split=w3s, **kw)
        assert all(torch.equal(x, y) for x, y in zip(a, b))
    r_y = torch.nn.functional.conv2d(a2.permute(0, 3, 1, 2), sd_for(N, 1)["Encoder.conv3.weight"], None,
                                     stride=2, padding=2)
    assert rel_err(b[2].permute(0, 3, 1, 2).cpu(), r_y) < REL


@pytest.mark.parametrize("T", [4, 8, 100])
def test_deconv3_bits_fold(device, T):
    """bpp's reduction folded into deconv3 (x6 chunk-major and bf16 kernels, workgroup 0) equals
    the separate reduce_partials kernel bit for bit, for batches of more than 64 images and for
    more than 64 partials per image; the images are the kernels' own outputs, unchanged."""
    N, B = 128, 70
    net = net_for(N, 2, device)
    dec = net.Decoder
    torch.manual_seed(1)
    part = (torch.rand(B, T, dtype=torch.float64) * 50.0).to(device)
    _, ref = kernels.reduce_partials(part, 1.0 / 12345.0, per_image=False)
    h = (torch.randn(B, 4, 4, N) * 0.5).to(device)
    hs = kernels.split_planes(h).reshape(3, B, 4, 4, N // 32, 32).permute(0, 1, 4, 2, 3, 5).contiguous()
    with torch.no_grad():
        c0, _, _ = kernels.deconv3_x6(hs, dec.packed_x6(), dec.deconv3.bias)
        c1, _, _, tot = kernels.deconv3_x6(hs, dec.packed_x6(), dec.deconv3.bias, bits=(part, 1.0 / 12345.0))
        assert torch.equal(c0, c1) and torch.equal(tot, ref)
        hb = kernels.to_bf16(h)
        b3 = dec.packed_bf16()[2]
        c2, _, _ = kernels.deconv3_bf16(hb, b3, dec.deconv3.bias)
        c3, _, _, tot2 = kernels.deconv3_bf16(hb, b3, dec.deconv3.bias, bits=(part, 1.0 / 12345.0))
        assert torch.equal(c2, c3) and torch.equal(tot2, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [192, 128])
def test_conv2_h3_tile_rows_match(device, N):
    """conv2 + GDN2 on the h3 engine takes 8-row tiles when 16-row ones would leave CUs idle (a
    small batch: training's B = 32 at 256²) and 16-row ones otherwise. The same images in a small
    (8-row) and a large (16-row) batch give bit-equal h3, fp32, x6 and pre-activation outputs: a
    pixel's arithmetic does not depend on the tile."""
    h, w = 64, 64                      # conv2 output 32×32: four 16×16 tiles per image
    Bs, Bw = 3, 64                     # 12 tiles·images < 256 CUs (8 rows), 256 (16 rows)
    net = net_for(N, 1, device)
    enc = net.Encoder
    w2h = enc.packed_h3()[0]
    ge2 = enc.gdn2.effective_params_h3()
    a1 = torch.from_numpy(synth.normal_like(33, (Bw, h, w, N), 0.7)).to(device)

    def run(B):
        return kernels.conv2_gdn_h3(kernels.h3_planes(a1[:B].contiguous(), cm=kernels.CONV_CM), w2h,
                                    enc.conv2.bias, *ge2, want_f32=True, want_x6=True, want_pre=True)

    small, wide = run(Bs), run(Bw)
    assert torch.equal(small[0], wide[0][:, :Bs])      # h3 planes [2][B][…]
    assert torch.equal(small[1], wide[1][:Bs])         # fp32
    assert torch.equal(small[2], wide[2][:, :Bs])      # x6 split [3][B][…]
    assert torch.equal(small[3], wide[3][:Bs])         # GDN2's input


@pytest.mark.gpu
@pytest.mark.parametrize("N", [192, 128])
@pytest.mark.parametrize("int_in", [False, True])
def test_deconv_h3_tile_rows_match(device, int_in, N):
    """deconv + IGDN on the h3 engine: 8-row tiles on a small batch (deconv1 at B = 3: 12 workgroups
    of 16 rows would leave CUs idle), 16-row ones on a large one (B = 64); the same images give
    bit-equal outputs, with the integer-input (ŷ) form and without."""
    h, w = 16, 16
    Bs, Bw = 3, 64
    net = net_for(N, 1, device)
    dec = net.Decoder
    x1 = dec.packed_h3k()[0]
    h1 = dec.igdn1.effective_params_h3()
    if int_in:
        y = torch.round(torch.from_numpy(synth.uniform(34, (Bw, h, w, N), -6, 6))).to(device)
    else:
        y = torch.from_numpy(synth.normal_like(34, (Bw, h, w, N), 2.0)).to(device)

    def run(B):
        return kernels.deconv_igdn_h3(kernels.h3_planes(y[:B].contiguous(), cm=kernels.DECONV_CM), x1,
                                      dec.deconv1.bias, *h1, want_f32=True, want_x6=True, want_pre=True,
                                      int_in=int_in)

    small, wide = run(Bs), run(Bw)
    for s_, w_ in zip(small, wide):
        if s_ is None:
            continue
        if s_.dim() == 4:
            assert torch.equal(s_, w_[:Bs])
        else:                       # planes first: [P][B][…]
            assert torch.equal(s_, w_[:, :Bs])


@pytest.mark.parametrize("form", ["h3", "x6"])
def test_conv3_narrow_tiles_match_wide(device, form):
    """Noise-mode conv3 at N=192 on a small and a large batch: x6 takes different tilings (under
    256 tiles·images the 48-column tiles, conv3_narrow, at or above it the 96-column ones), the h3
    engine the same one (8 × 16 tiles × 64-channel slices) at every batch. The same images in both
    batches give bit-equal y, ỹ and its split / h3 form (an output element's summation order does
    not depend on the tiling), and per-image bits that agree to summation order (x6: the partial
    counts differ) or bit for bit (h3)."""
    N, h, w = 192, 32, 32          # conv3 output 16×16: four 8×8 tiles per image
    Bs, Bw = 3, 64                 # 12 tiles·images < 256 (narrow), 256 (wide)
    net = net_for(N, 1, device)
    enc = net.Encoder
    rate = net.bitEstimator.packed()
    a2 = torch.from_numpy(synth.normal_like(31, (Bw, h, w, N), 0.7)).to(device)
    noise = torch.from_numpy(synth.uniform(32, (Bw, N, h // 2, w // 2), -0.5, 0.5)).to(device)

    def run(B):
        if form == "h3":
            r = kernels.conv3_quant_rate_h3(kernels.h3_planes(a2[:B].contiguous(), cm=kernels.CONV_CM), enc.packed_h3()[1],
                                            rate, noise[:B].contiguous(), want_y=True)
        else:
            r = kernels.conv3_quant_rate_x6(kernels.split_planes(a2[:B].contiguous()),
                                            enc.packed()[2], rate, noise[:B].contiguous(), want_y=True,
                                            w_split=enc.packed_w3_split())
        return r

    small, wide = run(Bs), run(Bw)
    if form == "h3":   # one tiling at every batch: the same partials
        assert torch.equal(small[1], wide[1][:Bs])
    else:
        assert small[1].shape[1] == 2 * wide[1].shape[1]   # twice the partials per image
    assert torch.equal(small[0], wide[0][:Bs]) and torch.equal(small[2], wide[2][:Bs])
    assert torch.equal(small[3], wide[3][:, :Bs])
    bs, bw = small[1].sum(1), wide[1][:Bs].sum(1)
    assert ((bs - bw).abs() <= 1e-6 * bw.abs()).all()   # fp32 per-tile sums in another grouping
