"""Factorised entropy model — surface of the reference models/bitEstimator.py:6-42.

``Bitparm`` / ``BitEstimator`` keep the reference parameters (h, b, a of shape (1, C, 1, 1);
the final layer has no ``a``) and init; forwards run gfx950 elementwise kernels.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import kernels
from ..packcache import PackCache


class Bitparm(nn.Module):
    def __init__(self, channel, final=False):
        super().__init__()
        self.final = final
        self.h = nn.Parameter(torch.nn.init.normal_(torch.empty(channel).view(1, -1, 1, 1), 0, 0.01))
        self.b = nn.Parameter(torch.nn.init.normal_(torch.empty(channel).view(1, -1, 1, 1), 0, 0.01))
        if not final:
            self.a = nn.Parameter(torch.nn.init.normal_(torch.empty(channel).view(1, -1, 1, 1), 0, 0.01))
        else:
            self.a = None

    def forward(self, x):
        # bitEstimator.py:20-25
        from ..autograd import BitparmFn, needs_grad
        ps = [p for p in (self.h, self.b, self.a) if p is not None]
        if needs_grad(x, ps):
            return BitparmFn.apply(x, self, *ps)
        return kernels.bitparm(x, self.h, self.b, self.a)


class BitEstimator(nn.Module):
    def __init__(self, channel):
        super().__init__()
        self.f1 = Bitparm(channel)
        self.f2 = Bitparm(channel)
        self.f3 = Bitparm(channel)
        self.f4 = Bitparm(channel, True)
        self.channel = channel
        self._pack = PackCache()

    def params_in_order(self):
        return [self.f1.h, self.f1.b, self.f1.a, self.f2.h, self.f2.b, self.f2.a,
                self.f3.h, self.f3.b, self.f3.a, self.f4.h, self.f4.b]

    def packed(self, force: bool = False):
        """Per-channel table [11][C]: softplus(h_k), b_k, tanh(a_k) (k=1..3), softplus(h4), b4."""
        ps = self.params_in_order()
        return self._pack.get("rate", ps, lambda: kernels.pack_rate(ps), force=force)

    def rate_table(self, force: bool = False):
        """element_bits for the integer latents −32..32 per channel ([C, 65]; the round-mode
        quantiser epilogue looks them up), cached like the packed parameters."""
        ps = self.params_in_order()
        return self._pack.get("rtab", ps, lambda: kernels.rate_table(self.packed(force), self.channel),
                              force=force)

    def entropy_tables(self, K: int = kernels.ENTROPY_K):
        """Quantised CDFs for the entropy coder (cached like the packed parameters)."""
        ps = self.params_in_order()
        return self._pack.get(f"cdf{K}", ps,
                              lambda: kernels.entropy_tables(self.packed(), self.channel, K),
                              )

    def forward(self, x):
        # bitEstimator.py:38-42
        from ..autograd import BitEstimatorFn, needs_grad
        if needs_grad(x, self.params_in_order()):
            return BitEstimatorFn.apply(x, self, *self.params_in_order())
        return kernels.bit_estimator(x, self.packed(), self.channel)
