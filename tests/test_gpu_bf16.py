"""The bf16 throughput mode (csrc/engine_bf16.hip).

Layer kernels are checked against a plain PyTorch fp32 reference of the SAME op: the reference
layer (oracle/codec_ref.py, itself pinned to the reference) evaluated on bf16-rounded operands
with fp32 arithmetic, its output rounded to bf16 — i.e. what one bf16 product per MAC with fp32
accumulation computes, up to the fp32 summation order. Bar: every element within 2 bf16 ulps
(2^-7 relative) of that reference, plus 1e-3 of the tensor's max (near-zero elements, where the
reference's fp32 sum and ours round to different bf16 neighbours of a tiny value).

End to end the mode has no bit-identity claim; the tests bound and print what SURVEY §8d asks
to report — the latent flip rate, Δbpp and ΔPSNR against the exact reference (the oracle) —
on C1 and on four Kodak-size images (G5 generator).
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from iclr_17_compression_amd import _lib, kernels, synth
from iclr_17_compression_amd.model import ImageCompressor
from oracle import codec_ref as oracle

pytestmark = pytest.mark.gpu


def bf(t: torch.Tensor) -> torch.Tensor:
    """fp32 → nearest bf16 value (round half to even), kept in fp32."""
    return t.float().to(torch.bfloat16).float()


def net_for(N, seed, device):
    net = ImageCompressor(out_channel_N=N)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, seed).items()})
    return net.to(device).eval()


def sd_for(N, seed):
    return oracle.state_dict_to_torch(synth.trained_like_state_dict(N, seed))


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def gdn_bf16_ref(u, beta, gamma, inverse):
    """GDN.py:73-94 with x² and γ_eff rounded to bf16 (the kernel's contraction operands)."""
    be, ge = oracle.gdn_effective_params(beta, gamma)
    C = u.shape[1]
    n = F.conv2d(bf(u * u), bf(ge).view(C, C, 1, 1)) + be.view(1, C, 1, 1)
    return u * torch.sqrt(n) if inverse else u / torch.sqrt(n)


def check_bf16(got_bits, ref, what):
    got = kernels.from_bf16(got_bits).cpu()
    ref = bf(ref)
    tol = 2.0 ** -7 * ref.abs() + 1e-3 * ref.abs().max()
    bad = (got - ref).abs() > tol
    frac_eq = (got == ref).float().mean().item()
    print(f"{what}: {frac_eq:.4f} of elements equal to the bf16 reference, "
          f"max |Δ| {(got - ref).abs().max().item():.3e} (max |ref| {ref.abs().max().item():.3e})")
    assert not bool(bad.any()), (what, int(bad.sum()))
    assert frac_eq > 0.9, (what, frac_eq)


@pytest.fixture
def bf16_mode():
    old = kernels.precision()
    kernels.set_precision("bf16")
    yield
    kernels.set_precision(old)


def test_to_bf16_round_to_nearest_even(device):
    x = torch.from_numpy(synth.normal_like(51, (4096,), 3.0))
    x[:8] = torch.tensor([0.0, -0.0, 1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, -1.0 - 2 ** -8, 3.0e38, 1e-40, 0.1])
    got = kernels.from_bf16(kernels.to_bf16(x.to(device))).cpu()
    assert torch.equal(got, bf(x))


@pytest.mark.parametrize("N", [192, 128])
@pytest.mark.parametrize("shape", [(2, 64, 96), (1, 80, 112), (1, 256, 256)])
def test_bf16_analysis_layers(device, N, shape):
    """conv1+GDN1, conv2+GDN2 and conv3+quantiser+rate in bf16, each from the reference's input
    (bf16-rounded), partial 8×8 / 16×16 / 8×16 tiles at 80×112."""
    B, H, W = shape
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(11, B, H, W)))
    w1b, w2b, w3b = net.Encoder.packed_bf16()
    e1, e2 = net.Encoder.gdn1.effective_params_bf16(), net.Encoder.gdn2.effective_params_bf16()
    with torch.no_grad():
        # conv1 + GDN1
        u1 = F.conv2d(bf(x), bf(sd["Encoder.conv1.weight"]), sd["Encoder.conv1.bias"], stride=4, padding=4)
        r_a1 = gdn_bf16_ref(u1, sd["Encoder.gdn1.beta"], sd["Encoder.gdn1.gamma"], False)
        a1 = kernels.conv1_gdn_bf16(x.to(device), w1b, net.Encoder.conv1.bias, *e1, N)
        check_bf16(a1, nhwc(r_a1), f"conv1+gdn1 N={N} {shape}")
        # conv2 + GDN2 from the reference's a1
        a1r = bf(r_a1)
        u2 = F.conv2d(a1r, bf(sd["Encoder.conv2.weight"]), sd["Encoder.conv2.bias"], stride=2, padding=2)
        r_a2 = gdn_bf16_ref(u2, sd["Encoder.gdn2.beta"], sd["Encoder.gdn2.gamma"], False)
        a2 = kernels.conv2_gdn_bf16(kernels.to_bf16(nhwc(a1r).to(device)), w2b, net.Encoder.conv2.bias, *e2)
        check_bf16(a2, nhwc(r_a2), f"conv2+gdn2 N={N} {shape}")
        # conv3 + round + rate from the reference's a2
        a2r = bf(r_a2)
        r_y = F.conv2d(a2r, bf(sd["Encoder.conv3.weight"]), None, stride=2, padding=2)
        y_hat, partial, y, ybf = kernels.conv3_quant_rate_bf16(kernels.to_bf16(nhwc(a2r).to(device)), w3b,
                                                               net.bitEstimator.packed(), want_y=True)
    err = (y.cpu() - nhwc(r_y)).abs().max().item() / r_y.abs().max().item()
    assert err < 1e-5, err                                  # fp32 accumulation of bf16 products
    assert torch.equal(y_hat.cpu(), torch.round(y.cpu()))   # half-to-even on the kernel's own y
    assert torch.equal(kernels.from_bf16(ybf).cpu(), bf(y_hat.cpu()))
    per, _ = kernels.reduce_partials(partial)
    r_bits = oracle.estimate_bits(y_hat.cpu().permute(0, 3, 1, 2), sd)[0]
    assert per.sum().item() == pytest.approx(float(r_bits), rel=1e-5)


@pytest.mark.parametrize("N", [192, 128])
@pytest.mark.parametrize("hw", [(4, 6), (5, 7), (16, 16), (32, 32)])
def test_bf16_synthesis_layers(device, N, hw):
    """deconv1/deconv2 + IGDN (both tile heights: 8 rows at small grids, 16 at ≥ 512 workgroups)
    and deconv3 + clamp (+ SSE) in bf16, each from the reference's input (bf16-rounded)."""
    h, w = hw
    B = 2 if h * w <= 256 else 4
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    d1b, d2b, d3 = net.Decoder.packed_bf16()
    q1, q2 = net.Decoder.igdn1.effective_params_bf16(), net.Decoder.igdn2.effective_params_bf16()
    y = torch.round(torch.from_numpy(synth.uniform(5, (B, N, h, w), -4, 4)))
    with torch.no_grad():
        v1 = F.conv_transpose2d(bf(y), bf(sd["Decoder.deconv1.weight"]), sd["Decoder.deconv1.bias"],
                                stride=2, padding=2, output_padding=1)
        r_s1 = gdn_bf16_ref(v1, sd["Decoder.igdn1.beta"], sd["Decoder.igdn1.gamma"], True)
        s1 = kernels.deconv_igdn_bf16(kernels.to_bf16(nhwc(y).to(device)), d1b, net.Decoder.deconv1.bias, *q1)
        check_bf16(s1, nhwc(r_s1), f"deconv1+igdn1 N={N} {hw}")
        s1r = bf(r_s1)
        v2 = F.conv_transpose2d(s1r, bf(sd["Decoder.deconv2.weight"]), sd["Decoder.deconv2.bias"],
                                stride=2, padding=2, output_padding=1)
        r_s2 = gdn_bf16_ref(v2, sd["Decoder.igdn2.beta"], sd["Decoder.igdn2.gamma"], True)
        s2 = kernels.deconv_igdn_bf16(kernels.to_bf16(nhwc(s1r).to(device)), d2b, net.Decoder.deconv2.bias, *q2)
        check_bf16(s2, nhwc(r_s2), f"deconv2+igdn2 N={N} {hw}")
        s2r = bf(r_s2)
        r_out = F.conv_transpose2d(s2r, bf(sd["Decoder.deconv3.weight"]), sd["Decoder.deconv3.bias"],
                                   stride=4, padding=4, output_padding=3)
        xr = torch.from_numpy(synth.to_unit_float(synth.image_u8(3, B, 16 * h, 16 * w)))
        clipped, recon, part = kernels.deconv3_bf16(kernels.to_bf16(nhwc(s2r).to(device)), d3,
                                                    net.Decoder.deconv3.bias, x_ref=xr.to(device),
                                                    want_recon=True)
    err = (recon.cpu() - r_out).abs().max().item() / r_out.abs().max().item()
    assert err < 1e-5, err
    assert torch.equal(clipped, recon.clamp(0, 1))
    per, _ = kernels.reduce_partials(part)
    ref_sse = (clipped.cpu().double() - xr.double()).pow(2).sum((1, 2, 3))
    assert torch.allclose(per.cpu(), ref_sse, rtol=1e-5)


def _flip_report(y_hat, r_yhat):
    n = int((y_hat.detach().cpu() != r_yhat).sum())
    return n, n / r_yhat.numel()


def test_bf16_c1_end_to_end(device, bf16_mode, golden_dir):
    """C1 (the reference's 256² plumbing image, G3) through the bf16 mode against the
    reference's own ŷ / bpp / MSE: flip rate and relative Δbpp / ΔPSNR bounded (and printed)."""
    g = np.load(os.path.join(golden_dir, "g3_c1_n192_256px.npz"), allow_pickle=False)
    meta = json.load(open(os.path.join(golden_dir, "g3_c1_n192_256px.json")))
    net = net_for(192, 1, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(0, 1, 256, 256))).to(device)
    with torch.no_grad():
        clipped, y_hat, bpp = net(x)
        ev = net.evaluate(x)
    n, rate = _flip_report(y_hat, torch.from_numpy(g["y_hat"].astype(np.float32)))
    dbpp = (bpp.item() - meta["bpp"]) / meta["bpp"]
    dpsnr = ev["psnr"][0].item() - meta["psnr"]
    print(f"bf16 C1: {n} latent flips ({rate:.4%}), Δbpp {dbpp:+.3e} rel, ΔPSNR {dpsnr:+.4f} dB")
    assert rate < 0.03 and abs(dbpp) < 0.01 and abs(dpsnr) < 0.05
    assert torch.equal(ev["y_hat"], y_hat)


def test_bf16_kodak_flip_rate(device, bf16_mode, golden_dir):
    """Four Kodak-size images (G5 generator, portrait and landscape) in bf16 against the
    reference's bpp / PSNR (G5) and the oracle's latents."""
    meta = json.load(open(os.path.join(golden_dir, "g5_kodak24_synth_n192.json")))
    net, sd = net_for(meta["N"], meta["weight_seed"], device), sd_for(meta["N"], meta["weight_seed"])
    for row in [meta["images"][i] for i in (0, 3, 9, 23)]:
        x = torch.from_numpy(synth.to_unit_float(
            synth.smooth_image_u8(meta["image_seed_base"] + row["index"], row["height"], row["width"])))[None]
        with torch.no_grad():
            ev = net.evaluate(x.to(device), want_msssim=True)
        _, r_yhat, _, _, _ = oracle.codec_forward(x, sd)
        n, rate = _flip_report(ev["y_hat"], r_yhat)
        dbpp = (ev["bpp"][0].item() - row["bpp"]) / row["bpp"]
        dpsnr = ev["psnr"][0].item() - row["psnr"]
        print(f"bf16 kodak-synth[{row['index']}]: {n} latent flips ({rate:.4%}), Δbpp {dbpp:+.3e} rel, "
              f"ΔPSNR {dpsnr:+.4f} dB")
        assert rate < 0.03 and abs(dbpp) < 0.01 and abs(dpsnr) < 0.05


def test_bf16_batch_independence_and_determinism(device, bf16_mode):
    net = net_for(192, 1, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(21, 3, 64, 96))).to(device)
    ev1, ev2 = net.evaluate(x), net.evaluate(x)
    for k in ("clipped", "y_hat", "bpp", "mse"):
        assert torch.equal(ev1[k], ev2[k]), k
    for i in range(3):
        evi = net.evaluate(x[i:i + 1])
        for k in ("y_hat", "bpp", "clipped"):
            assert torch.equal(evi[k][0], ev1[k][i]), k


def test_bf16_weight_packing_layout(device):
    """iclr17_pack_bf16: spot-check the documented layouts against the reference weights."""
    N = 128
    net = net_for(N, 1, device)
    w = net.Encoder.conv2.weight.detach().cpu()
    p = kernels.from_bf16(kernels.pack_bf16(_lib.ICLR17_BF_CONV5, net.Encoder.conv2.weight, N)).cpu()
    p = p.view(N // 16, 13, 4, N, 8)
    for (c, s, kg, co, e) in [(0, 0, 0, 0, 0), (3, 7, 2, 77, 5), (7, 12, 1, 127, 7), (7, 12, 3, 5, 1)]:
        t, ci = 2 * s + (kg >> 1), 16 * c + 8 * (kg & 1) + e
        ref = bf(w[co, ci, t // 5, t % 5]) if t < 25 else torch.tensor(0.0)
        assert p[c, s, kg, co, e] == ref
    wd = net.Decoder.deconv2.weight.detach().cpu()
    pd = kernels.from_bf16(kernels.pack_bf16(_lib.ICLR17_BF_DECONV5, net.Decoder.deconv2.weight, N)).cpu()
    # phase 3 (py = px = 1): taps ky, kx ∈ {1, 3}, 2 steps per chunk, after 5 + 3 + 3 steps of phases 0-2
    off = (N // 16) * (5 + 3 + 3) * 4 * N * 8
    p3 = pd[off:].view(N // 16, 2, 4, N, 8)
    for (c, s, kg, co, e) in [(0, 0, 0, 0, 0), (5, 1, 3, 100, 6)]:
        t, ci = 2 * s + (kg >> 1), 16 * c + 8 * (kg & 1) + e
        assert p3[c, s, kg, co, e] == bf(wd[ci, co, 2 * (t // 2) + 1, 2 * (t % 2) + 1])


def test_rate_table_matches_element_bits(device):
    """iclr17_rate_table: per channel the bits of the integer latents −32..32 (model.py:71-73),
    against the oracle's element_bits (fp32 rounding order of torch-CPU vs the kernel's: 1e-5)."""
    N = 192
    net, sd = net_for(N, 1, device), sd_for(N, 1)
    tab = net.bitEstimator.rate_table().cpu()
    v = torch.arange(-32, 33, dtype=torch.float32).view(1, 1, 1, 65).expand(1, N, 1, 65).contiguous()
    ref = oracle.element_bits(v, sd)[0, :, 0, :]
    assert tab.shape == (N, 65)
    # p = F(v+½) − F(v−½) cancels in fp32: ulp-level differences δF between the device's and
    # torch-CPU's CDFs move bits by ≈ δF / (p ln 2) = δF · 2^bits / ln 2; bound δF by 8 ulps of 1
    tol = 1e-5 * ref + 8 * 2.0 ** -24 * torch.exp2(ref) / 0.6931
    err = (tab - ref).abs()
    print(f"rate table: max |Δbits| {err.max().item():.3e}, max |Δ|/tol {(err / tol).max().item():.3f}")
    assert bool((err <= tol).all())
