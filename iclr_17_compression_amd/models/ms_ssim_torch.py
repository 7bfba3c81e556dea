"""MS-SSIM / SSIM — surface of the reference models/ms_ssim_torch.py:86-241 on the GPU kernels
(``csrc/msssim.hip``: separable 11-tap σ=1.5 Gaussian, 'valid' filtering, 2×2 average pooling,
the reference's level weights and final product).

``ms_ssim(X, Y, ...)`` and ``ssim(X, Y, ...)`` keep the reference signatures, argument checks
(``ValueError`` messages of :102-112 / :140-150) and return shapes (a 0-dim mean with
``size_average``, else a per-image vector). train.py:178 calls

    ms_ssim(clipped_recon_image.cpu().detach(), input.cpu(), data_range=1.0, size_average=True)

with CPU tensors: the inputs are copied to the current GPU, computed there and the result is
returned on the inputs' device. There is no CPU implementation: without a GPU this raises
``Iclr17Error``. The kernels implement the reference's default window and weights only; a
custom ``win`` / ``win_size`` / ``win_sigma`` / ``weights`` raises instead of silently computing
something else.
"""
from __future__ import annotations

import torch

from .. import kernels
from .._lib import Iclr17Error

_DEFAULT_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)   # ms_ssim_torch.py:162-163


def _check_inputs(X, Y, win_size):
    """ms_ssim_torch.py:102-112 / :140-150, in the reference's order."""
    if len(X.shape) != 4:
        raise ValueError('Input images must 4-d tensor.')
    if not X.type() == Y.type():
        raise ValueError('Input images must have the same dtype.')
    if not X.shape == Y.shape:
        raise ValueError('Input images must have the same dimensions.')
    if not (win_size % 2 == 1):
        raise ValueError('Window size must be odd.')


def _check_window(win_size, win_sigma, win):
    if win is not None or win_size != 11 or float(win_sigma) != 1.5:
        raise Iclr17Error("iclr17: the GPU SSIM kernels implement the reference's default window "
                          "(win_size=11, win_sigma=1.5, win=None) only")


def _to_gpu(X, Y):
    """(X, Y) on a GPU as contiguous fp32, plus the device to return results on. The kernels have
    no backward: with autograd on and an input that requires grad this raises rather than
    return a value a loss such as 1 − ms_ssim(...) would silently not differentiate."""
    if torch.is_grad_enabled() and (X.requires_grad or Y.requires_grad):
        raise Iclr17Error("iclr17: ms_ssim/ssim have no backward on the GPU kernels; call them on "
                          "detached tensors or under torch.no_grad()")
    if X.dtype != torch.float32:
        raise Iclr17Error(f"iclr17: ssim/ms_ssim take float32 images (got {X.dtype})")
    home = X.device
    if X.is_cuda:
        return X.detach().contiguous(), Y.detach().to(X.device).contiguous(), home
    if not torch.cuda.is_available():
        raise Iclr17Error("iclr17: ms_ssim/ssim run only on a ROCm GPU (MI355X / gfx950) — there "
                          "is no CPU implementation")
    dev = torch.device("cuda", torch.cuda.current_device())
    return (X.detach().to(dev, non_blocking=True).contiguous(),
            Y.detach().to(dev, non_blocking=True).contiguous(), home)


def ssim(X, Y, win_size=11, win_sigma=1.5, win=None, data_range=255, size_average=True, full=False):
    """ms_ssim_torch.py:86-120: per-image SSIM (mean over C·Ho·Wo of the ssim map); with
    ``size_average`` the batch mean; with ``full`` also the cs means."""
    _check_inputs(X, Y, win_size)
    _check_window(win_size, win_sigma, win)
    x, y, home = _to_gpu(X, Y)
    s, cs = kernels.ssim(x, y, float(data_range))
    if size_average:
        s, cs = s.mean(), cs.mean()
    s, cs = s.to(home), cs.to(home)
    return (s, cs) if full else s


def ms_ssim(X, Y, win_size=11, win_sigma=1.5, win=None, data_range=255, size_average=True,
            full=False, weights=None):
    """ms_ssim_torch.py:123-196: per-image MS-SSIM over 5 levels; with ``size_average`` the
    batch mean (0-dim). ``full`` is accepted and, as in the reference, has no effect."""
    _check_inputs(X, Y, win_size)
    _check_window(win_size, win_sigma, win)
    if weights is not None:
        w = torch.as_tensor(weights, dtype=torch.float32).reshape(-1).cpu()
        if w.numel() != 5 or not torch.equal(w, torch.tensor(_DEFAULT_WEIGHTS, dtype=torch.float32)):
            raise Iclr17Error("iclr17: the GPU MS-SSIM kernel implements the reference's default "
                              "5-level weights only")
    x, y, home = _to_gpu(X, Y)
    v = kernels.ms_ssim(x, y, float(data_range))
    if size_average:
        v = v.mean()
    return v.to(home)


class SSIM(torch.nn.Module):
    """ms_ssim_torch.py:200-219."""

    def __init__(self, win_size=11, win_sigma=1.5, data_range=None, size_average=True, channel=3):
        super().__init__()
        _check_window(win_size, win_sigma, None)
        if channel != 3:
            raise Iclr17Error("iclr17: the GPU SSIM kernels take 3-channel images")
        self.win = None
        self.size_average = size_average
        self.data_range = data_range

    def forward(self, X, Y):
        return ssim(X, Y, win=self.win, data_range=self.data_range, size_average=self.size_average)


class MS_SSIM(torch.nn.Module):
    """ms_ssim_torch.py:222-241."""

    def __init__(self, win_size=11, win_sigma=1.5, data_range=None, size_average=True, channel=3,
                 weights=None):
        super().__init__()
        _check_window(win_size, win_sigma, None)
        if channel != 3:
            raise Iclr17Error("iclr17: the GPU MS-SSIM kernel takes 3-channel images")
        self.win = None
        self.size_average = size_average
        self.data_range = data_range
        self.weights = weights

    def forward(self, X, Y):
        return ms_ssim(X, Y, win=self.win, size_average=self.size_average,
                       data_range=self.data_range, weights=self.weights)
