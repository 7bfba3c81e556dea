"""Synthesis transform g_s — surface of the reference models/synthesis_17.py:8-31.

Layers and init (synthesis_17.py:15-25): deconv5×5/s2 → IGDN → deconv5×5/s2 → IGDN →
deconv9×9/s4 → 3 channels. ``forward`` runs two fused deconv+IGDN kernels (stride-phase
decomposed, no zero insertion) and the all-phase deconv3 kernel; returns the UNclipped
reconstruction, NCHW, exactly like the reference module.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import _lib, kernels
from ..packcache import PackCache
from .GDN import GDN


class Synthesis_net_17(nn.Module):
    """Decode synthesis"""

    def __init__(self, out_channel_N=192):
        super().__init__()
        N = out_channel_N
        self.deconv1 = nn.ConvTranspose2d(N, N, 5, stride=2, padding=2, output_padding=1)
        torch.nn.init.xavier_normal_(self.deconv1.weight.data, math.sqrt(2 * 1))
        torch.nn.init.constant_(self.deconv1.bias.data, 0.01)
        self.igdn1 = GDN(N, inverse=True)
        self.deconv2 = nn.ConvTranspose2d(N, N, 5, stride=2, padding=2, output_padding=1)
        torch.nn.init.xavier_normal_(self.deconv2.weight.data, math.sqrt(2 * 1))
        torch.nn.init.constant_(self.deconv2.bias.data, 0.01)
        self.igdn2 = GDN(N, inverse=True)
        self.deconv3 = nn.ConvTranspose2d(N, 3, 9, stride=4, padding=4, output_padding=3)
        torch.nn.init.xavier_normal_(self.deconv3.weight.data, math.sqrt(2 * 1))
        torch.nn.init.constant_(self.deconv3.bias.data, 0.01)
        self.out_channel_N = N
        self._pack = PackCache()

    def packed(self, force: bool = False):
        N, f = self.out_channel_N, force
        d1 = self._pack.get("d1", (self.deconv1.weight,),
                            lambda: kernels.pack_weight(_lib.ICLR17_W_DECONV5, self.deconv1.weight, N), f)
        d2 = self._pack.get("d2", (self.deconv2.weight,),
                            lambda: kernels.pack_weight(_lib.ICLR17_W_DECONV5, self.deconv2.weight, N), f)
        return d1, d2, self.packed_d3(f), self.igdn1.effective_params(force), self.igdn2.effective_params(force)

    def packed_d3(self, force: bool = False):
        """deconv3's fp32 packing alone (the h3 layouts split it; the h3 training step needs no
        other fp32 weight packing of this module), cached with ``packed``'s entry."""
        N = self.out_channel_N
        return self._pack.get("d3", (self.deconv3.weight,),
                              lambda: kernels.pack_weight(_lib.ICLR17_W_DECONV9, self.deconv3.weight, N),
                              force)

    def packed_x6(self, force: bool = False):
        """deconv3's packed weights split into the x6 planes the halo kernel stages, cached."""
        d3 = self.packed_d3(force)
        return self._pack.get("d3x6", (self.deconv3.weight,),
                              lambda: kernels.split_deconv3(d3, self.out_channel_N), force)

    def packed_h3k(self, force: bool = False):
        """deconv1 / deconv2 in the h3 engine's two fp16 weight planes (4 stride phases, per-tensor
        power-of-two scale in the trailer) and deconv3's all-phase packing split the same way,
        cached until the weights change."""
        N, f = self.out_channel_N, force
        d1 = self._pack.get("d1h3", (self.deconv1.weight,),
                            lambda: kernels.pack_h3k(_lib.ICLR17_H3K_DECONV5, self.deconv1.weight, N), f)
        d2 = self._pack.get("d2h3", (self.deconv2.weight,),
                            lambda: kernels.pack_h3k(_lib.ICLR17_H3K_DECONV5, self.deconv2.weight, N), f)
        d3 = self.packed_d3(force)
        d3h = self._pack.get("d3h3", (self.deconv3.weight,),
                             lambda: kernels.split_packed_h3(d3, 9, N, 48), f)
        return d1, d2, d3h

    def packed_bf16(self, force: bool = False):
        """deconv1 / deconv2 in the bf16 engine's step layout (4 stride phases) and deconv3's
        all-phase packing rounded to bf16 fragments, cached."""
        N, f = self.out_channel_N, force
        d1 = self._pack.get("d1bf", (self.deconv1.weight,),
                            lambda: kernels.pack_bf16(_lib.ICLR17_BF_DECONV5, self.deconv1.weight, N), f)
        d2 = self._pack.get("d2bf", (self.deconv2.weight,),
                            lambda: kernels.pack_bf16(_lib.ICLR17_BF_DECONV5, self.deconv2.weight, N), f)
        d3 = self.packed_d3(force)
        d3b = self._pack.get("d3bf", (self.deconv3.weight,),
                             lambda: kernels.round_packed(d3, 9, N, 48), f)
        return d1, d2, d3b

    def packed_bwd(self, x6: bool):
        """The deconv weights packed as the convolutions of their input gradients: (deconv3 in
        the conv1 layout — x6 split form when ``x6`` —, deconv2, deconv1 in the conv5 layout),
        cached until the weights change."""
        N = self.out_channel_N
        if x6:
            d3 = self._pack.get("d3cx6", (self.deconv3.weight,),
                                lambda: kernels.pack_conv1_x6(self.deconv3.weight, N))
        else:
            d3 = self._pack.get("d3c", (self.deconv3.weight,),
                                lambda: kernels.pack_weight(_lib.ICLR17_W_CONV1, self.deconv3.weight, N))
        d2c = self._pack.get("d2c", (self.deconv2.weight,),
                             lambda: kernels.pack_weight(_lib.ICLR17_W_CONV5, self.deconv2.weight, N))
        d1c = self._pack.get("d1c", (self.deconv1.weight,),
                             lambda: kernels.pack_weight(_lib.ICLR17_W_CONV5, self.deconv1.weight, N))
        return d3, d2c, d1c

    @staticmethod
    def to_nhwc(y):
        """NCHW-shaped latent (any memory format) → contiguous NHWC [B, h, w, N] (no copy when
        the latent is already channels-last, e.g. the Encoder's own output)."""
        return y.permute(0, 2, 3, 1).contiguous()

    def decode(self, y_nhwc, x_ref=None, want_recon=True, y_split=None, y_bf16=None,
               y_integral=False, bits=None, y_h3=None, bits_per_image=False):
        """NHWC latent → (clipped NCHW, unclipped NCHW | None, SSE partials | None).
        With ``y_split`` (the latent in x6 split form) the three layers run in the x6 mode, with
        ``y_h3`` (the h3 form) the three layers run in the h3 form, with
        ``y_bf16`` (bf16 bit patterns) in the bf16 throughput mode. ``y_integral``: the latent
        is ŷ = round(y) (model.py:56), so the h3 deconv1 takes its integer-input form.
        ``bits`` = (conv3's bit partials, scale): a fourth output, ``reduce_partials``' 0-dim total,
        computed inside deconv3's kernel in the h3, x6 and bf16 modes (one launch fewer); h3 with
        ``bits_per_image``: a fifth, the per-image sums. In the h3 mode every output is NaN when a
        value of the chain (since the last kernels.h3_chain_begin) did not fit the h3 form."""
        d1, d2, d3, g1, g2 = self.packed()
        if y_bf16 is not None:
            b1, b2, b3 = self.packed_bf16()
            q1, q2 = self.igdn1.effective_params_bf16(), self.igdn2.effective_params_bf16()
            h = kernels.deconv_igdn_bf16(y_bf16, b1, self.deconv1.bias, *q1)
            h = kernels.deconv_igdn_bf16(h, b2, self.deconv2.bias, *q2)
            return kernels.deconv3_bf16(h, b3, self.deconv3.bias, x_ref=x_ref, want_recon=want_recon,
                                        bits=bits)
        if y_h3 is not None:
            q1, q2 = self.igdn1.effective_params_h3(), self.igdn2.effective_params_h3()
            w1, w2, w3 = self.packed_h3k()
            # on ŷ the integer-input form skips the lo products (the same bits: Decoder(round(y))
            # reproduces the codec's reconstruction without knowing its input is ŷ)
            hs, _, _ = kernels.deconv_igdn_h3(y_h3, w1, self.deconv1.bias, *q1, int_in=y_integral)
            hs, _, _ = kernels.deconv_igdn_h3(hs, w2, self.deconv2.bias, *q2, chunk_major=True)
            return kernels.deconv3_h3(hs, w3, self.deconv3.bias, x_ref=x_ref, want_recon=want_recon,
                                      bits=bits, bits_per_image=bits_per_image)
        if y_split is not None:
            q1, q2 = self.igdn1.effective_params_x6(), self.igdn2.effective_params_x6()
            hs, _, _ = kernels.deconv_igdn_x6(y_split, d1, self.deconv1.bias, *q1)
            hs, _, _ = kernels.deconv_igdn_x6(hs, d2, self.deconv2.bias, *q2, chunk_major=True)
            return kernels.deconv3_x6(hs, self.packed_x6(), self.deconv3.bias, x_ref=x_ref,
                                      want_recon=want_recon, bits=bits)
        else:
            h = kernels.deconv_igdn(y_nhwc, d1, self.deconv1.bias, g1[0], g1[1])
            h = kernels.deconv_igdn(h, d2, self.deconv2.bias, g2[0], g2[1])
        out = kernels.deconv3(h, d3, self.deconv3.bias, x_ref=x_ref, want_recon=want_recon)
        if bits is None:
            return out
        return (*out, kernels.reduce_partials(bits[0], bits[1], per_image=False)[1])

    def forward(self, x):
        from ..autograd import SynthesisFn, needs_grad
        kernels._check(x, "latent", 4)
        if x.shape[1] != self.out_channel_N:
            raise kernels.Iclr17Error(f"iclr17: Synthesis_net_17 expects {self.out_channel_N} channels")
        params = list(self.parameters())
        if needs_grad(x, params):
            return SynthesisFn.apply(x, self, *params)
        y = self.to_nhwc(x)
        split = kernels.split_planes(y) if kernels.precision() == "x6" else None
        if kernels.precision() == "h3":
            kernels.h3_chain_begin(y.device)
        yh3 = kernels.h3_planes(y, cm=kernels.DECONV_CM) if kernels.precision() == "h3" else None
        ybf = kernels.to_bf16(y) if kernels.precision() == "bf16" else None
        _, recon, _ = self.decode(y, want_recon=True, y_split=split, y_bf16=ybf, y_h3=yh3)
        return recon
