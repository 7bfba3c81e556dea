"""GDN / IGDN module — surface of the reference models/GDN.py:10-94.

Same constructor, parameters (``beta`` [C], ``gamma`` [C, C]) and re-parametrisation. The module
called on its own runs the stand-alone gfx950 kernel (per-pixel channel contraction β + γ·x² on
the exact-f32 MFMA, then x/√n or x·√n) through libiclr17.so; inside the codec's chain the same
contraction is fused into the producing convolution's epilogue and runs in the chain's precision
mode (h3 by default: three fp16 part products per MAC; kernels.precision). Effective (bounded,
squared) parameters are computed by a packing kernel and cached until the parameters change.
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn
from torch.autograd import Function

from .. import kernels
from ..packcache import PackCache


class LowerBound(Function):
    """models/GDN.py:10-24: forward max(x, bound); backward passes g where x ≥ bound or g < 0.
    (Parameter-sized; the GDN hot path applies the bound inside its packing kernel.)"""

    @staticmethod
    def forward(ctx, inputs, bound):
        b = torch.ones_like(inputs) * bound
        ctx.save_for_backward(inputs, b)
        return torch.max(inputs, b)

    @staticmethod
    def backward(ctx, grad_output):
        inputs, b = ctx.saved_tensors
        pass_through = (inputs >= b) | (grad_output < 0)
        return pass_through.type(grad_output.dtype) * grad_output, None


class GDN(nn.Module):
    """Generalized divisive normalization: y[i] = x[i] / sqrt(beta[i] + sum_j gamma[i, j] x[j]^2)
    (the conv2d semantics of the reference, GDN.py:80-83; ``inverse`` multiplies instead)."""

    def __init__(self, ch, inverse=False, beta_min=1e-6, gamma_init=0.1, reparam_offset=2 ** -18):
        super().__init__()
        self.inverse = inverse
        self.beta_min = beta_min
        self.gamma_init = gamma_init
        self.reparam_offset = reparam_offset
        self.build(ch)
        self._pack = PackCache()

    def build(self, ch):
        # GDN.py:46-62
        self.pedestal = self.reparam_offset ** 2
        self.beta_bound = (self.beta_min + self.reparam_offset ** 2) ** 0.5
        self.gamma_bound = self.reparam_offset
        self.beta = nn.Parameter(torch.sqrt(torch.ones(ch) + self.pedestal))
        self.gamma = nn.Parameter(torch.sqrt(self.gamma_init * torch.eye(ch) + self.pedestal))

    def bounds_f32(self):
        """The fp32 values ones_like(x) * bound evaluates to in the reference."""
        return (float(np.float32(self.beta_bound)), float(np.float32(self.gamma_bound)),
                float(np.float32(self.pedestal)))

    def _packed_all(self, force: bool = False):
        """(beta_eff, gamma_packed, gamma_packed_transposed), one packing launch, cached until
        beta or gamma change (their version counters move on every in-place update)."""
        bb, gb, ped = self.bounds_f32()
        return self._pack.get("gdn", (self.beta, self.gamma),
                              lambda: kernels.pack_gdn(self.beta, self.gamma, bb, gb, ped,
                                                       transposed=True), force=force)

    def effective_params(self, force: bool = False):
        """(beta_eff [C], gamma_packed [C*C]) on the parameters' device."""
        be, gp, _ = self._packed_all(force)
        return be, gp

    def effective_params_x6(self, force: bool = False):
        """(beta_eff, gamma_packed, gamma split planes) for the x6 inference kernels."""
        be, gp = self.effective_params(force)
        C = self.beta.shape[0]
        g6 = self._pack.get("gdn6", (self.beta, self.gamma),
                            lambda: kernels.split_packed(gp, 1, C, C), force=force)
        return be, gp, g6

    def effective_params_h3(self, force: bool = False):
        """(beta_eff, γ_eff in the h3 form: two fp16 planes + trailer, kernels.split_packed_h3 of
        the [C/4][C][4] packing) for the h3 inference kernels."""
        be, gp = self.effective_params(force)
        C = self.beta.shape[0]
        gh = self._pack.get("gdnh3", (self.beta, self.gamma),
                            lambda: kernels.split_packed_h3(gp, 1, C, C), force=force)
        return be, gh

    def effective_params_bf16(self, force: bool = False):
        """(beta_eff, γ_eff rounded to bf16 in the 16x16x32 fragment layout) for the bf16
        throughput kernels."""
        be, gp = self.effective_params(force)
        C = self.beta.shape[0]
        gb = self._pack.get("gdnbf", (self.beta, self.gamma),
                            lambda: kernels.round_packed(gp, 1, C, C), force=force)
        return be, gb

    def effective_params_bwd(self):
        """(beta_eff, gamma_packed, gamma_packed_transposed) for the backward kernels."""
        return self._packed_all()

    def effective_params_bwd_x6(self):
        """effective_params_bwd plus γ and γᵀ split for the x6 backward contractions:
        (beta_eff, gamma_packed, gamma_packed_t, gamma_split, gamma_t_split)."""
        be, gp, gpt = self._packed_all()
        C = self.beta.shape[0]
        g6 = self.effective_params_x6()[2]
        g6t = self._pack.get("gdn6t", (self.beta, self.gamma),
                             lambda: kernels.split_packed(gpt, 1, C, C))
        return be, gp, gpt, g6, g6t

    def forward(self, inputs):
        unfold = inputs.dim() == 5
        if unfold:  # GDN.py:65-69
            bs, ch, d, w, h = inputs.size()
            inputs = inputs.reshape(bs, ch, d * w, h)
        from ..autograd import gdn_apply
        outputs = gdn_apply(inputs, self)
        if unfold:
            outputs = outputs.reshape(bs, ch, d, w, h)
        return outputs
