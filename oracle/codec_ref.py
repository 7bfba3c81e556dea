"""ORACLE — CPU restatement of the reference Ballé-2017 hot path. TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline. The product path
(``iclr_17_compression_amd``) never imports it and fails loudly without its HIP library.

Every function restates, op for op and in the same fp32 evaluation order, the reference
PyTorch code it cites (paths relative to the reference repo root). Because the op
sequence is identical, on the same torch build this restatement is bit-identical to the
reference; ``tests/golden/gen_goldens.py`` checks that by importing the reference in the
build container and committing the reference's own outputs as fixtures, and
``tests/test_oracle_golden.py`` pins this module against those fixtures (parity pinned).

Parameters come in as a dict keyed like the reference ``state_dict``.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

# models/GDN.py:35-38,46-49 — constructor defaults and derived bounds
GDN_BETA_MIN = 1e-6
GDN_REPARAM_OFFSET = 2.0 ** -18
GDN_PEDESTAL = GDN_REPARAM_OFFSET ** 2
GDN_BETA_BOUND = (GDN_BETA_MIN + GDN_PEDESTAL) ** 0.5
GDN_GAMMA_BOUND = GDN_REPARAM_OFFSET


class _LowerBound(torch.autograd.Function):
    """``LowerBound`` of models/GDN.py:10-24.

    forward: max(x, ones_like(x)·bound); backward: pass g where x ≥ bound OR g < 0.
    """

    @staticmethod
    def forward(ctx, x, bound):
        b = torch.ones_like(x) * bound
        ctx.save_for_backward(x, b)
        return torch.max(x, b)

    @staticmethod
    def backward(ctx, g):
        x, b = ctx.saved_tensors
        keep = (x >= b) | (g < 0)
        return keep.type(g.dtype) * g, None


def lower_bound(x: Tensor, bound: float) -> Tensor:
    return _LowerBound.apply(x, bound)


def gdn_effective_params(beta_p: Tensor, gamma_p: Tensor) -> Tuple[Tensor, Tensor]:
    """Re-parametrisation of models/GDN.py:73-79: β = lb(β_p)² − ped, γ = lb(γ_p)² − ped."""
    beta = lower_bound(beta_p, GDN_BETA_BOUND) ** 2 - GDN_PEDESTAL
    gamma = lower_bound(gamma_p, GDN_GAMMA_BOUND) ** 2 - GDN_PEDESTAL
    return beta, gamma


def gdn(x: Tensor, beta_p: Tensor, gamma_p: Tensor, inverse: bool) -> Tensor:
    """GDN / IGDN forward, models/GDN.py:64-94 (4-D input path).

    norm = sqrt(conv2d(x², γ.view(C,C,1,1), β)); y = x / norm (GDN) or x · norm (IGDN).
    """
    c = x.shape[1]
    beta, gamma = gdn_effective_params(beta_p, gamma_p)
    norm = F.conv2d(x ** 2, gamma.view(c, c, 1, 1), beta)     # GDN.py:83
    norm = torch.sqrt(norm)                                    # GDN.py:84
    return x * norm if inverse else x / norm                   # GDN.py:87-90


def analysis(x: Tensor, p: Dict[str, Tensor], prefix: str = "Encoder.") -> Tensor:
    """Analysis_net_17.forward, models/analysis_17.py:32-39 (layers :14-23)."""
    g = lambda k: p[prefix + k]
    h = F.conv2d(x, g("conv1.weight"), g("conv1.bias"), stride=4, padding=4)
    h = gdn(h, g("gdn1.beta"), g("gdn1.gamma"), inverse=False)
    h = F.conv2d(h, g("conv2.weight"), g("conv2.bias"), stride=2, padding=2)
    h = gdn(h, g("gdn2.beta"), g("gdn2.gamma"), inverse=False)
    return F.conv2d(h, g("conv3.weight"), None, stride=2, padding=2)


def synthesis(y: Tensor, p: Dict[str, Tensor], prefix: str = "Decoder.") -> Tensor:
    """Synthesis_net_17.forward, models/synthesis_17.py:27-31 (layers :15-25)."""
    g = lambda k: p[prefix + k]
    h = F.conv_transpose2d(y, g("deconv1.weight"), g("deconv1.bias"), stride=2, padding=2,
                           output_padding=1)
    h = gdn(h, g("igdn1.beta"), g("igdn1.gamma"), inverse=True)
    h = F.conv_transpose2d(h, g("deconv2.weight"), g("deconv2.bias"), stride=2, padding=2,
                           output_padding=1)
    h = gdn(h, g("igdn2.beta"), g("igdn2.gamma"), inverse=True)
    return F.conv_transpose2d(h, g("deconv3.weight"), g("deconv3.bias"), stride=4, padding=4,
                              output_padding=3)


def bitparm(x: Tensor, h: Tensor, b: Tensor, a: Optional[Tensor]) -> Tensor:
    """Bitparm.forward, models/bitEstimator.py:20-25 (final layer when ``a`` is None)."""
    if a is None:
        return torch.sigmoid(x * F.softplus(h) + b)
    x = x * F.softplus(h) + b
    return x + torch.tanh(x) * torch.tanh(a)


def bit_estimator(x: Tensor, p: Dict[str, Tensor], prefix: str = "bitEstimator.") -> Tensor:
    """BitEstimator.forward, models/bitEstimator.py:38-42: f4∘f3∘f2∘f1."""
    for f in ("f1", "f2", "f3"):
        x = bitparm(x, p[f"{prefix}{f}.h"], p[f"{prefix}{f}.b"], p[f"{prefix}{f}.a"])
    return bitparm(x, p[f"{prefix}f4.h"], p[f"{prefix}f4.b"], None)


def estimate_bits(z: Tensor, p: Dict[str, Tensor]) -> Tuple[Tensor, Tensor]:
    """iclr18_estimate_bits_z, model.py:71-74: Σ clamp(−ln(p + 1e-10)/ln 2, 0, 50)."""
    prob = bit_estimator(z + 0.5, p) - bit_estimator(z - 0.5, p)
    total_bits = torch.sum(torch.clamp(-1.0 * torch.log(prob + 1e-10) / math.log(2.0), 0, 50))
    return total_bits, prob


def element_bits(z: Tensor, p: Dict[str, Tensor]) -> Tensor:
    """Per-element bits before the sum of model.py:73 (used for per-image sums)."""
    prob = bit_estimator(z + 0.5, p) - bit_estimator(z - 0.5, p)
    return torch.clamp(-1.0 * torch.log(prob + 1e-10) / math.log(2.0), 0, 50)


def codec_forward(x: Tensor, p: Dict[str, Tensor], training: bool = False,
                  noise: Optional[Tensor] = None):
    """ImageCompressor.forward, model.py:47-80.

    Returns ``(clipped_recon, y_hat, bpp, recon, y)``: the reference's return tuple
    (model.py:80) plus the unclipped reconstruction (whose MSE model.py:61 computes for the
    intended training loss) and the pre-quantisation latent.
    ``noise`` replaces the device RNG draw of model.py:48-49 in training mode.
    """
    y = analysis(x, p)
    if training:
        if noise is None:
            noise = torch.empty_like(y).uniform_(-0.5, 0.5)
        y_hat = y + noise                                       # model.py:54
    else:
        y_hat = torch.round(y)                                  # model.py:56
    recon = synthesis(y_hat, p)
    clipped = recon.clamp(0.0, 1.0)                             # model.py:59
    total_bits, _ = estimate_bits(y_hat, p)
    bpp = total_bits / (x.shape[0] * x.shape[2] * x.shape[3])  # model.py:78
    return clipped, y_hat, bpp, recon, y


def rd_loss(x: Tensor, p: Dict[str, Tensor], noise: Tensor, train_lambda: float):
    """The intended training objective of train.py:97-102 (defect D2 resolved as
    model.py:61,81 intend): λ·mean((recon − x)²) + bpp, recon unclipped."""
    clipped, y_hat, bpp, recon, _ = codec_forward(x, p, training=True, noise=noise)
    mse = torch.mean((recon - x).pow(2))
    return train_lambda * mse + bpp, mse, bpp


def psnr(clipped: Tensor, x: Tensor) -> Tensor:
    """testKodak PSNR, train.py:172-175: 10·log10(1 / mean((clipped − x)²))."""
    mse = torch.mean((clipped - x).pow(2))
    return 10 * (torch.log(1.0 / mse) / math.log(10))


# ------------------------------------------------------------------------------ MS-SSIM
# models/ms_ssim_torch.py as train.py:178 calls it: ms_ssim(clipped, x, data_range=1.0,
# size_average=True) with the default 11-tap, σ = 1.5 window and the 5 default level weights.
MSSSIM_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)   # ms_ssim_torch.py:153-154


def gauss_window(size: int = 11, sigma: float = 1.5) -> Tensor:
    """ms_ssim_torch.py:5-18: normalised 1-D Gaussian, fp32, centred at size // 2."""
    t = torch.arange(size).to(dtype=torch.float) - size // 2
    g = torch.exp(-(t ** 2) / (2 * sigma ** 2))
    return g / g.sum()


def _blur(z: Tensor, g: Tensor) -> Tensor:
    """ms_ssim_torch.py:21-34: depthwise 'valid' filtering, first along W, then along H."""
    C = z.shape[1]
    kw = g.reshape(1, 1, 1, -1).repeat(C, 1, 1, 1)
    z = F.conv2d(z, kw, groups=C)
    return F.conv2d(z, kw.transpose(2, 3), groups=C)


def ssim_and_cs(X: Tensor, Y: Tensor, g: Tensor, data_range: float) -> Tuple[Tensor, Tensor]:
    """ms_ssim_torch.py:37-80 (size_average=False, full=True): per-image means over C,H,W of
    the SSIM map and the contrast-structure map."""
    c1, c2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    mx, my = _blur(X, g), _blur(Y, g)
    mxx, myy, mxy = mx.pow(2), my.pow(2), mx * my
    vx = 1.0 * (_blur(X * X, g) - mxx)
    vy = 1.0 * (_blur(Y * Y, g) - myy)
    cxy = 1.0 * (_blur(X * Y, g) - mxy)
    cs_map = (2 * cxy + c2) / (vx + vy + c2)
    ssim_map = ((2 * mxy + c1) / (mxx + myy + c1)) * cs_map
    per_image = lambda m: m.mean(-1).mean(-1).mean(-1)  # noqa: E731
    return per_image(ssim_map), per_image(cs_map)


def ms_ssim(X: Tensor, Y: Tensor, data_range: float = 1.0) -> Tensor:
    """ms_ssim_torch.py:123-196 → per-image MS-SSIM [B]. Five levels, 2×2 average pooling with
    one padding row/column on odd sizes (counted in the average, avg_pool2d's default). Like the
    reference, the final product multiplies the LAST level's SSIM term into every one of the
    first four levels (ms_ssim_torch.py:189-190), so it enters as ssim_5^(4·w_5), and the last
    level's cs is not used."""
    w = torch.tensor(MSSSIM_WEIGHTS, dtype=X.dtype)
    g = gauss_window()
    mcs = []
    s = None
    for _ in range(len(MSSSIM_WEIGHTS)):
        s, cs = ssim_and_cs(X, Y, g, data_range)
        mcs.append(cs)
        pad = (X.shape[2] % 2, X.shape[3] % 2)
        X = F.avg_pool2d(X, kernel_size=2, padding=pad)
        Y = F.avg_pool2d(Y, kernel_size=2, padding=pad)
    mcs = torch.stack(mcs, dim=0)
    return torch.prod((mcs[:-1] ** w[:-1].unsqueeze(1)) * (s ** w[-1]), dim=0)


def state_dict_to_torch(sd) -> Dict[str, Tensor]:
    return {k: torch.as_tensor(v).float().contiguous() for k, v in sd.items()}
