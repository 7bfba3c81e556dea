"""Autograd glue for the HIP kernels.

Forward passes always run on libiclr17.so. Where a backward kernel is not wired yet the output
carries a grad_fn that raises a clear error instead of silently producing wrong gradients.
"""
from __future__ import annotations

from typing import Sequence

import torch

from . import kernels


class _NoBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, name, out, *inputs):
        ctx.name = name
        return out.view_as(out)

    @staticmethod
    def backward(ctx, *grads):
        raise NotImplementedError(f"iclr17: backward of {ctx.name} is not implemented by the HIP path yet")


def no_backward(out: torch.Tensor, name: str, params: Sequence[torch.Tensor], x: torch.Tensor):
    needs = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
    if not needs:
        return out
    return _NoBackward.apply(name, out, x, *params)


def gdn_apply(x: torch.Tensor, module) -> torch.Tensor:
    beta_eff, gp = module.effective_params()
    out = kernels.gdn(x, beta_eff, gp, module.inverse)
    return no_backward(out, "GDN", (module.beta, module.gamma), x)
