"""GPU parity of the training path (train.py:97-112 → rd_loss.backward()): every parameter
gradient of the fused HIP backward against the CPU oracle's autograd (oracle/codec_ref.py,
pinned to the reference's own autograd by tests/test_oracle_golden.py::test_g4_train_grads).

Tolerance: per tensor, max |Δgrad| ≤ 1e-4 · max |grad_ref| (fp32 reductions over up to ~1e5
terms in a different order); the loss terms within 1e-5 relative.
"""
import pytest
import torch

from iclr_17_compression_amd import kernels, synth
from iclr_17_compression_amd.model import ImageCompressor
from oracle import codec_ref as oracle

pytestmark = pytest.mark.gpu

GRAD_REL = 1e-4
LAM = 0.01 * 255.0 ** 2


def grad_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def make(N, seed, device):
    sd = synth.trained_like_state_dict(N, seed)
    net = ImageCompressor(out_channel_N=N)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return net.to(device).train(), oracle.state_dict_to_torch(sd)


@pytest.fixture(params=["h3", "x6", "fp32"])
def precision(request):
    """x6: the input-gradient contractions run in x6 on split-form gradients; h3: the same
    backward after the forward on the codec's h3 kernels; fp32: exact f32."""
    from iclr_17_compression_amd import kernels
    old = kernels.precision()
    kernels.set_precision(request.param)
    yield request.param
    kernels.set_precision(old)


@pytest.mark.parametrize("N,B,H,W", [(192, 2, 64, 64), (128, 2, 48, 80)])
def test_train_step_all_grads(device, precision, N, B, H, W):
    net, sd = make(N, 2, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(3, B, H, W)))
    noise = torch.from_numpy(synth.uniform(4, (B, N, H // 16, W // 16), -0.5, 0.5))
    clipped, mse, bpp = net.forward_train(x.to(device), noise=noise.to(device))
    loss = LAM * mse + bpp
    net.zero_grad()
    loss.backward()
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    r_loss, r_mse, r_bpp = oracle.rd_loss(x, sdp, noise, LAM)
    r_loss.backward()
    assert mse.item() == pytest.approx(r_mse.item(), rel=1e-5)
    assert bpp.item() == pytest.approx(r_bpp.item(), rel=1e-5)
    assert loss.item() == pytest.approx(r_loss.item(), rel=1e-5)
    errs = {k: grad_err(p.grad, sdp[k].grad) for k, p in net.named_parameters()}
    bad = {k: e for k, e in errs.items() if not e < GRAD_REL}
    print("max rel grad err", max(errs.values()))
    assert not bad, bad


def test_forward_tuple_in_training_mode(device):
    """ImageCompressor.forward in train mode returns (clipped, ỹ, bpp) (model.py:80), all
    differentiable; bpp alone back-propagates through the rate model into the encoder."""
    N = 192
    net, sd = make(N, 2, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(5, 1, 32, 32)))
    noise = torch.from_numpy(synth.uniform(6, (1, N, 2, 2), -0.5, 0.5))
    clipped, y_tilde, bpp = net(x.to(device), noise=noise.to(device))
    net.zero_grad()
    bpp.backward()
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    _, r_ytilde, r_bpp, _, _ = oracle.codec_forward(x, sdp, training=True, noise=noise)
    r_bpp.backward()
    assert grad_err(y_tilde, r_ytilde) < 2e-5
    for k, p in net.named_parameters():
        if sdp[k].grad is None or sdp[k].grad.abs().max() == 0:
            assert p.grad is None or p.grad.abs().max() == 0, k
            continue
        assert grad_err(p.grad, sdp[k].grad) < GRAD_REL, k


def test_decoder_alone_backward(device):
    """train_decoder_new.py:66-105 trains a Decoder on its own: gradients w.r.t. its input
    latent and its parameters."""
    N = 192
    net, sd = make(N, 7, device)
    y = torch.from_numpy(synth.uniform(8, (2, N, 4, 4), -3, 3))
    target = torch.from_numpy(synth.to_unit_float(synth.image_u8(9, 2, 64, 64)))
    yd = y.to(device).requires_grad_(True)
    recon = net.Decoder(yd)
    loss = torch.mean((recon - target.to(device)) ** 2)
    loss.backward()
    ry = y.clone().requires_grad_(True)
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    r_loss = torch.mean((oracle.synthesis(ry, sdp) - target) ** 2)
    r_loss.backward()
    assert loss.item() == pytest.approx(r_loss.item(), rel=1e-5)
    assert grad_err(yd.grad, ry.grad) < GRAD_REL
    for k, p in net.Decoder.named_parameters():
        assert grad_err(p.grad, sdp["Decoder." + k].grad) < GRAD_REL, k


def test_encoder_alone_backward(device):
    N = 128
    net, sd = make(N, 11, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(12, 2, 64, 48)))
    R = torch.from_numpy(synth.uniform(13, (2, N, 4, 3), -1, 1))
    y = net.Encoder(x.to(device))
    (y * R.to(device)).sum().backward()
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    (oracle.analysis(x, sdp) * R).sum().backward()
    for k, p in net.Encoder.named_parameters():
        assert grad_err(p.grad, sdp["Encoder." + k].grad) < GRAD_REL, k


def test_backward_is_deterministic(device):
    N = 192
    net, _ = make(N, 2, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(3, 2, 64, 64))).to(device)
    noise = torch.from_numpy(synth.uniform(4, (2, N, 4, 4), -0.5, 0.5)).to(device)
    grads = []
    for _ in range(2):
        net.zero_grad()
        _, mse, bpp = net.forward_train(x, noise=noise)
        (LAM * mse + bpp).backward()
        grads.append({k: p.grad.clone() for k, p in net.named_parameters()})
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


@pytest.mark.parametrize("M,C,B,Ho,Wo", [(192, 192, 2, 16, 16), (192, 192, 3, 8, 12), (128, 128, 2, 32, 32)])
def test_wgrad_k5_x6_matches_fp32(device, M, C, B, Ho, Wo):
    """The x6 weight gradient (split-form operands, ds_read_b64_tr_b16 fragments) against the
    exact-f32 wgrad_k5 on the same values: the split is exact, so only rounding differs.
    Partial last k-step (B·Ho·Wo not a multiple of 32 per split) at 3×8×12."""
    from iclr_17_compression_amd import kernels
    G = torch.from_numpy(synth.normal_like(21, (B, Ho, Wo, M), 1.0)).to(device)
    X = torch.from_numpy(synth.normal_like(22, (B, 2 * Ho, 2 * Wo, C), 1.0)).to(device)
    ref = kernels.wgrad_k5(G, X)
    got = kernels.wgrad_k5_x6(kernels.split_planes(G), kernels.split_planes(X))
    torch.cuda.synchronize()
    assert grad_err(got, ref) < 1e-5


@pytest.mark.parametrize("C,inverse,channels_last,shape", [(192, False, False, (2, 5, 7)),
                                                           (192, True, True, (1, 16, 16)),
                                                           (128, False, True, (3, 9, 4))])
def test_standalone_gdn_backward(device, C, inverse, channels_last, shape):
    """models.GDN used on its own (GDN.py:64-94): ∂x, ∂β, ∂γ against the oracle's autograd (with
    LowerBound's gradient rule, some β/γ entries below their bounds); ragged 64-pixel tiles."""
    from iclr_17_compression_amd.models import GDN
    B, H, W = shape
    sd = synth.trained_like_state_dict(C, 7)
    beta = torch.from_numpy(sd["Encoder.gdn1.beta"].copy())
    gamma = torch.from_numpy(sd["Encoder.gdn1.gamma"].copy())
    beta[:3] = 1e-4    # below the LowerBound of √(1e-6 + 2^-36): gradient only where g < 0
    gamma[0, :5] = 0.0
    m = GDN(C, inverse=inverse)
    m.load_state_dict({"beta": beta, "gamma": gamma})
    m = m.to(device)
    x = torch.from_numpy(synth.normal_like(31, (B, C, H, W), 0.7))
    g = torch.from_numpy(synth.normal_like(32, (B, C, H, W), 1.0))
    xd = x.to(device).requires_grad_(True)
    xin = xd.contiguous(memory_format=torch.channels_last) if channels_last else xd
    y = m(xin)
    y.backward(g.to(device))
    bp, gp = beta.clone().requires_grad_(True), gamma.clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    yr = oracle.gdn(xr, bp, gp, inverse)
    yr.backward(g)
    assert grad_err(y, yr) < 2e-5
    assert grad_err(xd.grad, xr.grad) < 1e-4
    assert grad_err(m.beta.grad, bp.grad) < 1e-4
    assert grad_err(m.gamma.grad, gp.grad) < 1e-4


@pytest.mark.parametrize("channels_last", [False, True])
def test_standalone_bit_estimator_backward(device, channels_last):
    """models.BitEstimator / Bitparm on their own (bitEstimator.py:6-42): ∂x and every ∂h, ∂b,
    ∂a against the oracle's autograd."""
    from iclr_17_compression_amd.models import BitEstimator
    C = 192
    sd = synth.trained_like_state_dict(C, 8)
    be = BitEstimator(C)
    be.load_state_dict({k[len("bitEstimator."):]: torch.from_numpy(v.copy()) for k, v in sd.items()
                        if k.startswith("bitEstimator.")})
    be = be.to(device)
    x = torch.from_numpy(synth.uniform(33, (2, C, 6, 5), -6, 6))
    g = torch.from_numpy(synth.normal_like(34, (2, C, 6, 5), 1.0))
    xd = x.to(device).requires_grad_(True)
    xin = xd.contiguous(memory_format=torch.channels_last) if channels_last else xd
    # the full estimator, then each Bitparm alone (a non-final and the final layer)
    outs = [be(xin), be.f2(xin), be.f4(xin)]
    sum((o * g.to(device)).sum() for o in outs).backward()
    p = {k: torch.from_numpy(v.copy()).requires_grad_(True) for k, v in sd.items()
         if k.startswith("bitEstimator.")}
    xr = x.clone().requires_grad_(True)
    ro = [oracle.bit_estimator(xr, p),
          oracle.bitparm(xr, p["bitEstimator.f2.h"], p["bitEstimator.f2.b"], p["bitEstimator.f2.a"]),
          oracle.bitparm(xr, p["bitEstimator.f4.h"], p["bitEstimator.f4.b"], None)]
    sum((o * g).sum() for o in ro).backward()
    for o, r in zip(outs, ro):
        assert grad_err(o, r) < 1e-5
    assert grad_err(xd.grad, xr.grad) < 1e-4
    for name, prm in be.named_parameters():
        assert grad_err(prm.grad, p["bitEstimator." + name].grad) < 1e-4, name


@pytest.mark.parametrize("M,B,Ho,Wo", [(192, 2, 16, 16), (128, 1, 8, 12), (192, 3, 20, 12)])
def test_wgrad_k9_x6_matches_fp32(device, M, B, Ho, Wo):
    """The x6 conv1/deconv3 weight gradient (split im2col + 1×1 x6 GEMM, tr_b16 fragments)
    against the exact-f32 wgrad_k9 on the same values, incl. ragged last k-steps."""
    from iclr_17_compression_amd import kernels
    G = torch.from_numpy(synth.normal_like(23, (B, Ho, Wo, M), 1.0)).to(device)
    X = torch.from_numpy(synth.uniform(24, (B, 3, 4 * Ho, 4 * Wo), 0.0, 1.0)).to(device)
    ref = kernels.wgrad_k9(G, X)
    got = kernels.wgrad_k9_x6(kernels.split_planes(G), X)
    torch.cuda.synchronize()
    assert grad_err(got, ref) < 1e-5


@pytest.mark.parametrize("C,P", [(192, 131072), (192, 1000 + 17), (128, 4096 + 5), (192, 40)])
def test_gdn_wgrad_x6_matches_fp32(device, C, P):
    """The x6 GDN γ gradient (dn and u² split inside the kernel) against the exact-f32 kernel and a
    float64 reference on the same values: full-size GDN1 pixels, ragged last steps, fewer pixels
    than one split."""
    from iclr_17_compression_amd import kernels
    dn = torch.from_numpy(synth.normal_like(25, (P, C), 1.0))
    u = torch.from_numpy(synth.normal_like(26, (P, C), 1.0))
    ref64 = dn.double().t() @ (u.float() * u.float()).double()
    dd, ud = dn.to(device), u.to(device)
    got = kernels.gdn_wgrad(dd, ud, x6=True)
    f32 = kernels.gdn_wgrad(dd, ud, x6=False)
    torch.cuda.synchronize()
    assert grad_err(got, ref64.float()) < 1e-5
    assert grad_err(got, f32) < 1e-5
    assert torch.equal(kernels.gdn_wgrad(dd, ud, x6=True), got)   # deterministic


@pytest.mark.parametrize("N,B,H,W", [(192, 2, 64, 64), (128, 1, 48, 80)])
def test_input_image_gradient_train_step(device, precision, N, B, H, W):
    """∂(λ·MSE + bpp)/∂x through the fused training step (the reference's autograd through
    analysis_17.py:32-39 and the loss): conv1's input gradient on the deconv3 kernel with
    conv1's weights, against the oracle's autograd; the parameter gradients are unchanged."""
    net, sd = make(N, 2, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(7, B, H, W)))
    noise = torch.from_numpy(synth.uniform(8, (B, N, H // 16, W // 16), -0.5, 0.5))
    xg = x.to(device).requires_grad_(True)
    _, mse, bpp = net.forward_train(xg, noise=noise.to(device))
    net.zero_grad()
    (LAM * mse + bpp).backward()
    xr = x.clone().requires_grad_(True)
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    r_loss, _, _ = oracle.rd_loss(xr, sdp, noise, LAM)
    r_loss.backward()
    assert grad_err(xg.grad, xr.grad) < GRAD_REL, grad_err(xg.grad, xr.grad)
    errs = {k: grad_err(p.grad, sdp[k].grad) for k, p in net.named_parameters()}
    assert max(errs.values()) < GRAD_REL, errs


def test_analysis_module_input_gradient(device):
    """Analysis_net_17 alone (analysis_17.py:32-39) with x.requires_grad: ∂(Σ y·g)/∂x and the
    parameter gradients against the oracle's autograd."""
    N, B, H, W = 192, 2, 64, 48
    net, sd = make(N, 3, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(9, B, H, W)))
    gy = torch.from_numpy(synth.normal_like(10, (B, N, H // 16, W // 16), 1.0))
    xg = x.to(device).requires_grad_(True)
    y = net.Encoder(xg)
    net.zero_grad()
    (y * gy.to(device)).sum().backward()
    xr = x.clone().requires_grad_(True)
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    (oracle.analysis(xr, sdp) * gy).sum().backward()
    assert grad_err(xg.grad, xr.grad) < GRAD_REL
    for k, p in net.Encoder.named_parameters():
        assert grad_err(p.grad, sdp["Encoder." + k].grad) < GRAD_REL, k


def test_eval_mode_autograd(device):
    """ImageCompressor.forward in eval mode with autograd on (model.py:47-80 with torch.round):
    the outputs equal the fused eval path's, and a loss on (clipped, bpp) back-propagates into
    the synthesis and BitEstimator parameters as the oracle's autograd does; round's zero
    gradient leaves the encoder without one."""
    N, B, H, W = 192, 2, 64, 64
    net, sd = make(N, 2, device)
    net.eval()
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(11, B, H, W)))
    clipped, y_hat, bpp = net(x.to(device))
    with torch.no_grad():
        c0, yh0, b0 = net(x.to(device))
    assert torch.equal(y_hat, yh0)
    assert grad_err(clipped, c0) < 2e-5 and bpp.item() == pytest.approx(b0.item(), rel=1e-5)
    net.zero_grad()
    (LAM * torch.mean((clipped - x.to(device)) ** 2) + bpp).backward()
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    r_clipped, r_yhat, r_bpp, _, _ = oracle.codec_forward(x, sdp, training=False)
    (LAM * torch.mean((r_clipped - x) ** 2) + r_bpp).backward()
    assert torch.equal(y_hat.cpu(), r_yhat)
    for k, p in net.named_parameters():
        ref = sdp[k].grad
        if k.startswith("Encoder."):
            assert p.grad is None and (ref is None or ref.abs().max() == 0), k
            continue
        assert grad_err(p.grad, ref) < GRAD_REL, (k, grad_err(p.grad, ref))


def test_h3_training_forward_saved_tensors(device):
    """The h3 training forward (the codec's h3 kernels with their pre-activation and x6 split
    outputs) hands the backward the x6 forward's tensors to the h3 form's accuracy, at a size with
    partial tiles (B=2, 48×80: conv2's 12×20 output, deconv1's 3×5 input)."""
    from iclr_17_compression_amd import autograd, kernels
    N = 192
    net, _ = make(N, 3, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(7, 2, 48, 80))).to(device)
    enc, dec = net.Encoder, net.Decoder
    old = kernels.precision()
    try:
        with torch.no_grad():
            kernels.set_precision("x6")
            _, sx = autograd.analysis_features_train(enc, x)
            y = kernels.conv3_quant_rate_x6(sx["a2s"], enc.packed()[2], net.bitEstimator.packed())[0]
            _, rx, ssex, tx = autograd.synthesis_forward_train(dec, y, x_ref=x)
            kernels.set_precision("h3")
            _, sh = autograd.analysis_features_train(enc, x)
            _, rh, sseh, th = autograd.synthesis_forward_train(dec, y, x_ref=x)
    finally:
        kernels.set_precision(old)
    rel = lambda a, b: ((a - b).abs().max() / b.abs().max()).item()  # noqa: E731
    for k in ("u1", "u2"):
        assert rel(sh[k], sx[k]) < 5e-6, k
    for k in ("a1s", "a2s"):
        assert rel(kernels.merge_planes(sh[k]), kernels.merge_planes(sx[k])) < 5e-6, k
    assert torch.equal(kernels.merge_h3(sh["a2h"]), kernels.merge_h3(kernels.h3_planes(
        kernels.merge_planes(sh["a2s"]))))
    for k in ("v1", "v2"):
        assert rel(th[k], tx[k]) < 5e-6, k
    for k in ("s1s", "s2s"):
        assert rel(kernels.merge_planes(th[k]), kernels.merge_planes(tx[k])) < 5e-6, k
    assert rel(rh, rx) < 5e-6
    assert abs(sseh.double().sum().item() - ssex.double().sum().item()) <= 1e-5 * ssex.double().sum().item()


@pytest.mark.parametrize("T,C", [(1, 3), (37, 192), (4096 + 3, 192), (2048, 128), (513, 300)])
def test_sum_rows_fixed_order(device, T, C):
    """iclr17_sum_rows / _sum_rows2 (the bias and β partials of the backward): the split rows
    added by the last-arriving workgroup (C ≤ 256) or by a second launch (C > 256) give the
    column sums within fp32 summation error, bitwise the same on every call, and the pair entry
    bitwise the single one."""
    g = torch.Generator().manual_seed(T * 1000 + C)
    a = (torch.randn(T, C, generator=g) * torch.exp(torch.randn(T, 1, generator=g))).to(device)
    b = torch.randn(T, C, generator=g).to(device)
    ref = a.double().sum(0)
    s1, s2 = kernels.sum_rows(a), kernels.sum_rows(a)
    torch.cuda.synchronize()
    assert torch.equal(s1, s2)
    tol = 1e-6 * a.double().abs().sum(0).max().item()
    assert (s1.double() - ref).abs().max().item() <= tol
    pa, pb = kernels.sum_rows2(a, b)
    assert torch.equal(pa, s1) and torch.equal(pb, kernels.sum_rows(b))
