"""Full-size configurations on the GPU (BASELINE configs[1] and [2]):

* C3 — one training step at its production size, B = 32 crops of 256×256, N = 192, λ = 0.01
  (train_lambda 650.25), fixed noise: the loss terms and all 30 parameter gradients against the
  oracle's autograd (oracle/codec_ref.py, pinned to the reference's autograd by G4), in the h3
  (the default: h3 forward, x6 backward), x6 and exact-f32 modes. These are the kernels' real launch shapes (split-K partial counts, grid
  sizing, partial-sum trees at 32×64²), which the small-shape tests do not reach.
* Data-parallel semantics (train.py:228 DataParallel → one process per GPU): the
  gradient of the full batch equals the mean of the gradients of its two equal shards, i.e. the
  λ·MSE_r + bpp_r averaging DESIGN §6 uses.
* C2 — all 24 synthetic Kodak images (G5) through ``evaluate``: bpp and PSNR against the
  reference's values at 1e-5, the latents against the oracle (near-tie rule of check_latents),
  the flip count printed per image; and testKodak's own lines (train.py:171-179) run verbatim
  on the build's names (``from model import *``).

Gradient bar as tests/test_gpu_backward.py: per tensor max |Δ| ≤ 1e-4 · max |ref|.
"""
import json
import os

import numpy as np
import pytest
import torch

from iclr_17_compression_amd import kernels, synth
from iclr_17_compression_amd.model import ImageCompressor
from oracle import codec_ref as oracle

pytestmark = pytest.mark.gpu

GRAD_REL = 1e-4
METRIC_REL = 1e-5
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


@pytest.fixture(scope="module")
def c3_case():
    """The C3 inputs (images seed 1, noise seed 2, as SURVEY §8d) and the oracle's loss terms and
    gradients, computed once on the host CPU."""
    N, B, S = 192, 32, 256
    sd = oracle.state_dict_to_torch(synth.trained_like_state_dict(N, 2))
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(1, B, S, S)))
    noise = torch.from_numpy(synth.uniform(2, (B, N, S // 16, S // 16), -0.5, 0.5))
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    r_loss, r_mse, r_bpp = oracle.rd_loss(x, sdp, noise, LAM)
    r_loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in sdp.items()}
    return {"x": x, "noise": noise, "loss": r_loss.item(), "mse": r_mse.item(), "bpp": r_bpp.item(),
            "grads": grads}


@pytest.mark.parametrize("precision", ["h3", "x6", "fp32"])
def test_c3_train_step_full_size(device, c3_case, precision):
    old = kernels.precision()
    kernels.set_precision(precision)
    try:
        net, _ = make(192, 2, device)
        x, noise = c3_case["x"].to(device), c3_case["noise"].to(device)
        _, mse, bpp = net.forward_train(x, noise=noise)
        loss = LAM * mse + bpp
        net.zero_grad()
        loss.backward()
        torch.cuda.synchronize()
    finally:
        kernels.set_precision(old)
    assert mse.item() == pytest.approx(c3_case["mse"], rel=METRIC_REL)
    assert bpp.item() == pytest.approx(c3_case["bpp"], rel=METRIC_REL)
    assert loss.item() == pytest.approx(c3_case["loss"], rel=METRIC_REL)
    errs = {k: grad_err(p.grad, c3_case["grads"][k]) for k, p in net.named_parameters()}
    print(f"C3 {precision}: max rel grad err {max(errs.values()):.3e} "
          f"({max(errs, key=errs.get)}); rel mse {abs(mse.item() / c3_case['mse'] - 1):.2e}, "
          f"rel bpp {abs(bpp.item() / c3_case['bpp'] - 1):.2e}")
    bad = {k: e for k, e in errs.items() if not e < GRAD_REL}
    assert not bad, bad


def test_data_parallel_equals_full_batch(device):
    """Mean of the per-shard gradients (two B=4 shards) == gradient of the B=8 batch, the
    all-reduce-average semantics of dist.GradAllReducer / allreduce_grads."""
    N, B, S = 192, 8, 64
    net, _ = make(N, 3, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(5, B, S, S))).to(device)
    noise = torch.from_numpy(synth.uniform(6, (B, N, S // 16, S // 16), -0.5, 0.5)).to(device)

    def grads(lo, hi):
        net.zero_grad(set_to_none=True)
        _, mse, bpp = net.forward_train(x[lo:hi], noise=noise[lo:hi])
        (LAM * mse + bpp).backward()
        return {k: p.grad.clone() for k, p in net.named_parameters()}

    full = grads(0, B)
    g0, g1 = grads(0, B // 2), grads(B // 2, B)
    errs = {k: grad_err((g0[k] + g1[k]) / 2, full[k]) for k in full}
    print(f"DP shard-mean vs full batch: max rel err {max(errs.values()):.3e}")
    bad = {k: e for k, e in errs.items() if not e < GRAD_REL}
    assert not bad, bad


def test_c4_global_batch_shards_lambda_sweep(device):
    """BASELINE configs[3] (C4) on one GPU: a global batch of 256 crops of 256² sharded 8 × 32 as
    the 8 ranks would hold it, for each λ of the sweep {0.003, 0.01, 0.03, 0.1} (train_lambda =
    λ·255²). The all-reduce average of the 8 shard gradients (what dist.GradAllReducer delivers
    before the clamp + Adam) equals the gradient of the whole 256-crop batch, per tensor at the
    gradient bar. The ranks' collective itself is covered by tests/test_dist_cpu.py (gloo) and
    tests/test_gpu_dp_overlap.py; 8 GPUs are not available to the test suite."""
    N, S, R, PER = 192, 256, 8, 32
    B = R * PER
    net, _ = make(N, 7, device)
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(11, B, S, S))).to(device)
    noise = torch.from_numpy(synth.uniform(12, (B, N, S // 16, S // 16), -0.5, 0.5)).to(device)

    def grads(lam, lo, hi):
        net.zero_grad(set_to_none=True)
        _, mse, bpp = net.forward_train(x[lo:hi], noise=noise[lo:hi])
        loss = lam * mse + bpp
        loss.backward()
        return loss.item(), {k: p.grad.clone() for k, p in net.named_parameters()}

    for lam_rd in (0.003, 0.01, 0.03, 0.1):
        lam = lam_rd * 255.0 ** 2
        full_loss, full = grads(lam, 0, B)
        shard = [grads(lam, r * PER, (r + 1) * PER) for r in range(R)]
        mean_loss = sum(s[0] for s in shard) / R
        errs = {k: grad_err(sum(s[1][k] for s in shard) / R, full[k]) for k in full}
        print(f"C4 λ={lam_rd}: loss {full_loss:.6f} (shard mean {mean_loss:.6f}), "
              f"max rel grad err {max(errs.values()):.3e}")
        assert np.isfinite(full_loss) and mean_loss == pytest.approx(full_loss, rel=METRIC_REL)
        bad = {k: e for k, e in errs.items() if not e < GRAD_REL}
        assert not bad, (lam_rd, bad)


# ------------------------------------------------------------------------------------- C2
def _kodak_meta(golden_dir):
    return json.load(open(os.path.join(golden_dir, "g5_kodak24_synth_n192.json")))


def _kodak_image(meta, row):
    return torch.from_numpy(synth.to_unit_float(
        synth.smooth_image_u8(meta["image_seed_base"] + row["index"], row["height"], row["width"])))[None]


def _check_latents(y_hat, y, r_yhat, r_y, max_rate=1e-4):
    from test_gpu_parity import check_latents   # tests/ is on sys.path (pytest prepend mode)
    return check_latents(y_hat, y, r_yhat, r_y, max_rate)


@pytest.mark.parametrize("precision", ["h3", "x6", "fp32"])
def test_kodak24_all_images(device, golden_dir, precision):
    meta = _kodak_meta(golden_dir)
    old = kernels.precision()
    kernels.set_precision(precision)
    sd = oracle.state_dict_to_torch(synth.trained_like_state_dict(meta["N"], meta["weight_seed"]))
    net, _ = make(meta["N"], meta["weight_seed"], device)
    net.eval()
    total = 0
    try:
        for row in meta["images"]:
            x = _kodak_image(meta, row)
            with torch.no_grad():
                ev = net.evaluate(x.to(device), want_y=True)
            assert ev["bpp"][0].item() == pytest.approx(row["bpp"], rel=METRIC_REL), row["index"]
            assert ev["psnr"][0].item() == pytest.approx(row["psnr"], rel=METRIC_REL), row["index"]
            _, r_yhat, _, _, r_y = oracle.codec_forward(x, sd)
            n = _check_latents(ev["y_hat"], ev["y"], r_yhat, r_y)
            total += n
            print(f"kodak-synth[{row['index']:2d}] {precision}: {n} near-tie latent flips of "
                  f"{r_yhat.numel()}")
    finally:
        kernels.set_precision(old)
    print(f"kodak-synth all 24 {precision}: {total} near-tie flips of "
          f"{24 * 192 * 32 * 48} latents")


def test_testkodak_lines_verbatim(device, golden_dir):
    """train.py:171-179 as written, on names from `from model import *` (ms_ssim with CPU tensors,
    size_average=True), for four G5 images: bpp / PSNR against the reference's values (1e-5),
    MS-SSIM against the oracle on the same pair (1e-5) and against the reference's value at the
    degenerate G5 operating point (1e-3, see test_gpu_parity.test_kodak_synth_subset)."""
    ns = {}
    exec("from iclr_17_compression_amd.model import *", ns)
    ms_ssim, np_, torch_ = ns["ms_ssim"], ns["np"], ns["torch"]
    meta = _kodak_meta(golden_dir)
    net, _ = make(meta["N"], meta["weight_seed"], device)
    net.eval()
    for row in [meta["images"][i] for i in (1, 8, 17, 22)]:
        input = _kodak_image(meta, row).to(device)
        with torch_.no_grad():
            # ---- train.py:171-179 ----
            clipped_recon_image, mse_loss, bpp = net(input)
            mse_loss = torch_.mean((clipped_recon_image - input).pow(2))
            mse_loss, bpp = \
                torch_.mean(mse_loss), torch_.mean(bpp)
            psnr = 10 * (torch_.log(1. / mse_loss) / np_.log(10))
            msssim = ms_ssim(clipped_recon_image.cpu().detach(), input.cpu(), data_range=1.0, size_average=True)
            msssimDB = -10 * (torch_.log(1-msssim) / np_.log(10))
            # ----
        assert msssim.device.type == "cpu" and msssim.dim() == 0
        assert bpp.item() == pytest.approx(row["bpp"], rel=METRIC_REL)
        assert psnr.item() == pytest.approx(row["psnr"], rel=METRIC_REL)
        r_ms = oracle.ms_ssim(clipped_recon_image.cpu(), input.cpu(), 1.0)
        assert msssim.item() == pytest.approx(r_ms.item(), rel=1e-5)
        assert msssim.item() == pytest.approx(row["ms_ssim"], rel=1e-3)
        assert np.isfinite(msssimDB.item())


def test_ssim_single_scale_vs_oracle(device):
    """models.ssim (ms_ssim_torch.py:86-120) on the GPU against the oracle's single-level
    (ssim, cs): per image, batch mean, and `full`."""
    from iclr_17_compression_amd.models import ssim
    B, H, W = 3, 64, 80
    x = torch.from_numpy(synth.uniform(41, (B, 3, H, W)))
    y = (x + torch.from_numpy(synth.normal_like(42, (B, 3, H, W), 0.05))).clamp(0, 1)
    r_s, r_cs = oracle.ssim_and_cs(y, x, oracle.gauss_window(), 1.0)
    s, cs = ssim(y.to(device), x.to(device), data_range=1.0, size_average=False, full=True)
    assert s.cpu().tolist() == pytest.approx(r_s.tolist(), rel=1e-5)
    assert cs.cpu().tolist() == pytest.approx(r_cs.tolist(), rel=1e-5)
    m = ssim(y, x, data_range=1.0)   # CPU in, CPU out, batch mean
    assert m.device.type == "cpu" and m.item() == pytest.approx(float(r_s.mean()), rel=1e-5)
