"""Analysis transform g_a — surface of the reference models/analysis_17.py:8-39.

Layers (and their init, analysis_17.py:14-23) are the reference's: conv9×9/s4 → GDN →
conv5×5/s2 → GDN → conv5×5/s2 (no bias). ``forward`` runs three fused gfx950 kernels
(conv1+GDN, conv2+GDN, conv3) on NHWC activations and returns y as a contiguous NCHW
tensor, like the reference.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import _lib, kernels
from ..packcache import PackCache
from .GDN import GDN


class Analysis_net_17(nn.Module):
    """Analysis net"""

    def __init__(self, out_channel_N=192):
        super().__init__()
        N = out_channel_N
        self.conv1 = nn.Conv2d(3, N, 9, stride=4, padding=4)
        torch.nn.init.xavier_normal_(self.conv1.weight.data, math.sqrt(2 * (3 + N) / 6))
        torch.nn.init.constant_(self.conv1.bias.data, 0.01)
        self.gdn1 = GDN(N)
        self.conv2 = nn.Conv2d(N, N, 5, stride=2, padding=2)
        torch.nn.init.xavier_normal_(self.conv2.weight.data, math.sqrt(2))
        torch.nn.init.constant_(self.conv2.bias.data, 0.01)
        self.gdn2 = GDN(N)
        self.conv3 = nn.Conv2d(N, N, 5, stride=2, padding=2, bias=False)
        torch.nn.init.xavier_normal_(self.conv3.weight.data, math.sqrt(2))
        self.out_channel_N = N
        self._pack = PackCache()

    def packed(self, force: bool = False):
        N, f = self.out_channel_N, force
        w1 = self._pack.get("w1", (self.conv1.weight,),
                            lambda: kernels.pack_weight(_lib.ICLR17_W_CONV1, self.conv1.weight, N), f)
        w2 = self._pack.get("w2", (self.conv2.weight,),
                            lambda: kernels.pack_weight(_lib.ICLR17_W_CONV5, self.conv2.weight, N), f)
        g1 = self.gdn1.effective_params(force)
        g2 = self.gdn2.effective_params(force)
        return w1, w2, self.packed_w3(f), g1, g2

    def packed_w3(self, force: bool = False):
        """conv3's fp32 packing alone (the h3 layouts split it; the h3 training step needs no
        other fp32 weight packing of this module), cached with ``packed``'s entry."""
        N = self.out_channel_N
        return self._pack.get("w3", (self.conv3.weight,),
                              lambda: kernels.pack_weight(_lib.ICLR17_W_CONV5, self.conv3.weight, N),
                              force)

    def packed_w3_split(self, force: bool = False):
        """conv3's packed weights pre-split into the x6 planes (kernels.split_packed), cached:
        the x6 conv3 then reads its B operand as it is instead of splitting it per k-step."""
        N = self.out_channel_N
        w3 = self.packed_w3(force)
        return self._pack.get("w3x6", (self.conv3.weight,),
                              lambda: kernels.split_packed(w3, 25, N, N), force)

    def packed_h3(self, force: bool = False):
        """conv2 / conv3 weights in the h3 engine's packing (kernels.pack_h3k, ICLR17_H3K_CONV5:
        two fp16 planes, per-tensor power-of-two scales), cached."""
        N = self.out_channel_N
        w2h = self._pack.get("w2h3", (self.conv2.weight,),
                             lambda: kernels.pack_h3k(_lib.ICLR17_H3K_CONV5, self.conv2.weight, N), force)
        w3h = self._pack.get("w3h3", (self.conv3.weight,),
                             lambda: kernels.pack_h3k(_lib.ICLR17_H3K_CONV5, self.conv3.weight, N), force)
        return w2h, w3h

    def packed_conv1_h3(self, force: bool = False):
        """conv1's weights in the h3 form (kernels.pack_conv1_h3), cached."""
        N = self.out_channel_N
        return self._pack.get("w1h3", (self.conv1.weight,),
                              lambda: kernels.pack_conv1_h3(self.conv1.weight, N), force)

    def packed_conv1_x6(self, force: bool = False):
        """conv1's weights in the x6 kernel's split layout (kernels.pack_conv1_x6), cached."""
        N = self.out_channel_N
        return self._pack.get("w1x6", (self.conv1.weight,),
                              lambda: kernels.pack_conv1_x6(self.conv1.weight, N),
                              force)

    def packed_bf16(self, force: bool = False):
        """The bf16 throughput-mode weights (conv1 in the reordered-K fragment layout, conv2 and
        conv3 in the bf16 engine's step layout), cached until the weights change."""
        N, f = self.out_channel_N, force
        w1 = self._pack.get("w1bf", (self.conv1.weight,),
                            lambda: kernels.round_packed(
                                kernels.pack_weight(_lib.ICLR17_W_CONV1_X6, self.conv1.weight, N),
                                1, 256, N), f)
        w2 = self._pack.get("w2bf", (self.conv2.weight,),
                            lambda: kernels.pack_bf16(_lib.ICLR17_BF_CONV5, self.conv2.weight, N), f)
        w3 = self._pack.get("w3bf", (self.conv3.weight,),
                            lambda: kernels.pack_bf16(_lib.ICLR17_BF_CONV5, self.conv3.weight, N), f)
        return w1, w2, w3

    def packed_bwd(self):
        """conv3 / conv2 weights packed as the transposed convolutions of their input gradients
        (the engine's deconv layout), cached until the weights change."""
        N = self.out_channel_N
        w3t = self._pack.get("w3t", (self.conv3.weight,),
                             lambda: kernels.pack_weight(_lib.ICLR17_W_DECONV5, self.conv3.weight, N))
        w2t = self._pack.get("w2t", (self.conv2.weight,),
                             lambda: kernels.pack_weight(_lib.ICLR17_W_DECONV5, self.conv2.weight, N))
        return w3t, w2t

    def packed_conv1_t(self):
        """conv1.weight in deconv3's packing: the transposed convolution of conv1's input
        gradient (autograd.conv1_input_grad), cached until the weight changes."""
        return self._pack.get("w1t", (self.conv1.weight,),
                              lambda: kernels.pack_weight(_lib.ICLR17_W_DECONV9, self.conv1.weight,
                                                          self.out_channel_N))

    def forward(self, x):
        """analysis_17.py:31-36 → y, contiguous NCHW like the reference's. With or without
        autograd it runs the very kernels of ``ImageCompressor.forward``'s analysis half in the
        current precision (conv3 with its quantiser epilogue, y taken before the rounding), so
        ``torch.round(Encoder(x))`` is bitwise the codec's ŷ (NewTests/testReconSeperateEandD.py:67,
        which runs with autograd on)."""
        from ..autograd import AnalysisFn, needs_grad
        kernels._check(x, "image", 4)
        params = list(self.parameters())
        if needs_grad(x, params):
            return AnalysisFn.apply(x.contiguous(), self, *params)
        return self.y_nhwc(x.contiguous()).permute(0, 3, 1, 2).contiguous()

    def y_nhwc(self, x, feats=None):
        """y (NHWC) through the codec's analysis kernels. ``feats``: the training forward's
        conv2+GDN2 output (autograd.analysis_features_train), reused for conv3 where it is the
        codec's own operand (x6: its split form; fp32: the fp32 activation; h3: its h3 form — the
        training forward runs the codec's h3 kernels). In the bf16 mode the codec's own chain runs
        again (its y is what the codec rounds) while the gradient is the training kernels' x6
        one, a different function at bf16 precision (≈0.3 % of the rounded latents, §3 of
        DESIGN.md)."""
        N = self.out_channel_N
        w1, w2, w3, g1, g2 = self.packed()
        # the rate epilogue needs a model: a zero one (its bits are discarded, y is all we keep)
        z = torch.zeros(11 * N, device=x.device)
        ztab = torch.zeros(N, 65, device=x.device)
        if feats is not None and kernels.precision() == "h3" and feats.get("a2h") is not None:
            return kernels.conv3_quant_rate_h3(feats["a2h"], self.packed_h3()[1], z, want_y=True,
                                               rtab=ztab, want_h3=False)[2]
        if feats is not None and kernels.precision() == "x6" and feats.get("a2s") is not None:
            return kernels.conv3_quant_rate_x6(feats["a2s"], w3, z, want_y=True, rtab=ztab,
                                               w_split=self.packed_w3_split())[2]
        if feats is not None and kernels.precision() == "fp32":
            return kernels.conv3_quant_rate(feats["a2"], w3, z, want_y=True, rtab=ztab)[2]
        if kernels.precision() == "bf16":
            w1b, w2b, w3b = self.packed_bf16()
            e1, e2 = self.gdn1.effective_params_bf16(), self.gdn2.effective_params_bf16()
            h = kernels.conv1_gdn_bf16(x, w1b, self.conv1.bias, *e1, N)
            h = kernels.conv2_gdn_bf16(h, w2b, self.conv2.bias, *e2)
            y = kernels.conv3_quant_rate_bf16(h, w3b, z, ztab, want_y=True)[2]
        elif kernels.precision() == "h3":
            kernels.h3_chain_begin(x.device)
            e1, e2 = self.gdn1.effective_params_h3(), self.gdn2.effective_params_h3()
            w2h, w3h = self.packed_h3()
            hs, _ = kernels.conv1_gdn_h3(x, self.packed_conv1_h3(), self.conv1.bias, *e1, N)
            hs, _, _ = kernels.conv2_gdn_h3(hs, w2h, self.conv2.bias, *e2)
            y = kernels.conv3_quant_rate_h3(hs, w3h, z, want_y=True, rtab=ztab, want_h3=False)[2]
        elif kernels.precision() == "x6":
            e1, e2 = self.gdn1.effective_params_x6(), self.gdn2.effective_params_x6()
            hs, _, _ = kernels.conv1x6_gdn(x, self.packed_conv1_x6(), self.conv1.bias, e1[0], e1[2], N)
            hs, _, _ = kernels.conv2_gdn_x6(hs, w2, self.conv2.bias, *e2)
            y = kernels.conv3_quant_rate_x6(hs, w3, z, want_y=True, rtab=ztab,
                                            w_split=self.packed_w3_split())[2]
        else:
            h = kernels.conv1_gdn(x, w1, self.conv1.bias, g1[0], g1[1], N)
            h = kernels.conv2_gdn(h, w2, self.conv2.bias, g2[0], g2[1])
            y = kernels.conv3_quant_rate(h, w3, z, want_y=True, rtab=ztab)[2]
        return y
