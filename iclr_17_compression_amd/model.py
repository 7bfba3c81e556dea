"""Top-level codec — surface of the reference model.py:1-81.

``ImageCompressor(out_channel_N=128)`` owns ``Encoder`` (Analysis_net_17), ``Decoder``
(Synthesis_net_17) and ``bitEstimator`` (BitEstimator) with the reference's state_dict keys,
and ``forward(x) -> (clipped_recon, y_hat, bpp)`` (model.py:47-80). The forward is one chain
of fused gfx950 kernels:

    conv1+GDN → conv2+GDN → conv3+quantise+rate → deconv1+IGDN → deconv2+IGDN →
    deconv3+bias+clamp → deterministic bit reduction

``save_model`` / ``load_model`` keep the reference's file naming and merge semantics
(model.py:18-35).
"""
from __future__ import annotations

import logging  # noqa: F401  (re-exported: train.py uses it via `from model import *`)
import math  # noqa: F401
import os
from typing import Dict, Optional

import numpy as np  # noqa: F401  (re-exported, train.py:117)
import torch
import torch.nn as nn

from . import kernels
from .models import *  # noqa: F401,F403
from .models import Analysis_net_17, BitEstimator, Synthesis_net_17


def save_model(model, iter, name):
    """model.py:18-19"""
    torch.save(model.state_dict(), os.path.join(name, "iter_{}.pth.tar".format(iter)))


def load_model(model, f):
    """model.py:22-35: merge the checkpoint's matching keys; always returns step 0 (D7)."""
    with open(f, "rb") as fh:
        pretrained_dict = torch.load(fh, map_location="cpu", weights_only=True)
        model_dict = model.state_dict()
        pretrained_dict = {k: v for k, v in pretrained_dict.items() if k in model_dict}
        model_dict.update(pretrained_dict)
        model.load_state_dict(model_dict)
    return 0


class ImageCompressor(nn.Module):
    def __init__(self, out_channel_N=128):
        super().__init__()
        self.Encoder = Analysis_net_17(out_channel_N=out_channel_N)
        self.Decoder = Synthesis_net_17(out_channel_N=out_channel_N)
        self.bitEstimator = BitEstimator(channel=out_channel_N)
        self.out_channel_N = out_channel_N

    # -------------------------------------------------------------------------------------
    def _latent_noise(self, x: torch.Tensor) -> torch.Tensor:
        # model.py:48-49: U(-0.5, 0.5) of shape [B, N, H//16, W//16] on the device RNG
        B, _, H, W = x.shape
        return torch.empty(B, self.out_channel_N, H // 16, W // 16, device=x.device,
                           dtype=torch.float32).uniform_(-0.5, 0.5)

    def run(self, x: torch.Tensor, noise: Optional[torch.Tensor] = None, training: Optional[bool] = None,
            x_ref_sse: bool = False, want_recon: bool = False,
            want_y: bool = False) -> Dict[str, torch.Tensor]:
        """The fused forward. Returns a dict with ``clipped`` (NCHW), ``y_hat`` (NHWC), bits
        partials and, on request, per-image SSE partials (vs x) and the unclipped recon."""
        training = self.training if training is None else training
        x = x.contiguous()
        q = self.encode_latents(x, noise, training, want_y)
        y_hat, bits_partial, y_split = q["y_hat"], q["bits_partial"], q["y_split"]
        out = {"y_hat": y_hat, "bits_partial": bits_partial, "y": q["y"]}
        if q.get("y_h3") is not None:
            # h3: the per-image bit sums folded into deconv3's kernel, which writes them (and every
            # other result) as NaN when a value of the chain did not fit the h3 form
            B, _, H, W = x.shape
            clipped, recon, sse_partial, _, out["bits_per_image"] = self.Decoder.decode(
                y_hat, x_ref=x if x_ref_sse else None, want_recon=want_recon,
                y_integral=not training, y_h3=q["y_h3"], bits=(bits_partial, 1.0 / (B * H * W)),
                bits_per_image=True)
        else:
            clipped, recon, sse_partial = self.Decoder.decode(y_hat, x_ref=x if x_ref_sse else None,
                                                              want_recon=want_recon, y_split=y_split,
                                                              y_bf16=q.get("y_bf16"),
                                                              y_integral=not training)
        out.update({"clipped": clipped, "sse_partial": sse_partial, "recon": recon})
        return out

    def encode_latents(self, x: torch.Tensor, noise: Optional[torch.Tensor] = None,
                       training: bool = False, want_y: bool = False) -> Dict[str, torch.Tensor]:
        """The analysis half of ``run``: conv1+GDN → conv2+GDN → conv3+quantise+rate. Returns
        ``y_hat`` (NHWC), the bits partials, ``y_split`` (x6 split form, or None), ``y_h3`` (the
        h3 form in the h3 mode, or None) and ``y``."""
        kernels._check(x, "image", 4)
        if training and noise is None:
            noise = self._latent_noise(x)
        if not training:
            noise = None
        x = x.contiguous()
        w1, w2, w3, g1, g2 = self.Encoder.packed()
        N = self.out_channel_N
        if kernels.precision() == "bf16" and noise is None:
            # the throughput mode: bf16 activations and weights, one bf16 product per MAC
            w1b, w2b, w3b = self.Encoder.packed_bf16()
            e1 = self.Encoder.gdn1.effective_params_bf16()
            e2 = self.Encoder.gdn2.effective_params_bf16()
            h = kernels.conv1_gdn_bf16(x, w1b, self.Encoder.conv1.bias, *e1, N)
            h = kernels.conv2_gdn_bf16(h, w2b, self.Encoder.conv2.bias, *e2)
            y_hat, bits, y, ybf = kernels.conv3_quant_rate_bf16(h, w3b, self.bitEstimator.packed(),
                                                                self.bitEstimator.rate_table(),
                                                                want_y=want_y)
            return {"y_hat": y_hat, "bits_partial": bits, "y_split": None, "y_bf16": ybf, "y": y}
        if kernels.precision() == "h3":
            # the parity mode on the f16 MFMA: conv1, conv2 and conv3 (and the GDN contractions)
            # in the h3 form (three fp16 part products per MAC), ŷ handed on in the h3 form
            kernels.h3_chain_begin(x.device)
            e1 = self.Encoder.gdn1.effective_params_h3()
            e2 = self.Encoder.gdn2.effective_params_h3()
            w2h, w3h = self.Encoder.packed_h3()
            hs, _ = kernels.conv1_gdn_h3(x, self.Encoder.packed_conv1_h3(), self.Encoder.conv1.bias,
                                         *e1, N)
            hs, _, _ = kernels.conv2_gdn_h3(hs, w2h, self.Encoder.conv2.bias, *e2)
            rt = self.bitEstimator.rate_table() if noise is None else None
            q = kernels.conv3_quant_rate_h3(hs, w3h, self.bitEstimator.packed(), noise, want_y=want_y,
                                            rtab=rt)
            return {"y_hat": q[0], "bits_partial": q[1], "y_split": None, "y_h3": q[3],
                    "y": q[2] if want_y else None}
        if kernels.precision() != "fp32":
            e1 = self.Encoder.gdn1.effective_params_x6()
            e2 = self.Encoder.gdn2.effective_params_x6()
            hs, _, _ = kernels.conv1x6_gdn(x, self.Encoder.packed_conv1_x6(), self.Encoder.conv1.bias,
                                           e1[0], e1[2], N)
            hs, _, _ = kernels.conv2_gdn_x6(hs, w2, self.Encoder.conv2.bias, *e2)
            rt = self.bitEstimator.rate_table() if noise is None else None
            q = kernels.conv3_quant_rate_x6(hs, w3, self.bitEstimator.packed(), noise, want_y=want_y,
                                            rtab=rt, w_split=self.Encoder.packed_w3_split())
            y_split = q[3]
        else:
            h = kernels.conv1_gdn(x, w1, self.Encoder.conv1.bias, g1[0], g1[1], N)
            h = kernels.conv2_gdn(h, w2, self.Encoder.conv2.bias, g2[0], g2[1])
            rt = self.bitEstimator.rate_table() if noise is None else None
            q = kernels.conv3_quant_rate(h, w3, self.bitEstimator.packed(), noise, want_y=want_y,
                                         rtab=rt)
            y_split = None
        return {"y_hat": q[0], "bits_partial": q[1], "y_split": y_split,
                "y": q[2] if want_y else None}

    def forward(self, input_image, noise: Optional[torch.Tensor] = None):
        """model.py:47-80 → (clipped_recon, ŷ or ỹ, bpp). In training mode with autograd on, the
        fused training kernels run and every output is differentiable."""
        from .autograd import CodecTrainFn, needs_grad, no_backward
        params = list(self.parameters())
        if self.training and needs_grad(input_image, params):
            clipped, y_tilde, bpp, _ = self._train_outputs(input_image, noise, params)
            return clipped, y_tilde, bpp
        B, _, H, W = input_image.shape
        if not self.training and needs_grad(input_image, params):
            return self._eval_autograd(input_image)
        # run() with bpp's reduction (model.py:71-78) folded into deconv3's kernel
        q = self.encode_latents(input_image.contiguous(), noise, self.training)
        clipped, _, _, bpp = self.Decoder.decode(q["y_hat"], want_recon=False, y_split=q["y_split"],
                                                 y_bf16=q.get("y_bf16"), y_integral=not self.training,
                                                 bits=(q["bits_partial"], 1.0 / (B * H * W)),
                                                 y_h3=q.get("y_h3"))
        out = {"clipped": clipped, "y_hat": q["y_hat"]}
        y_hat = out["y_hat"].permute(0, 3, 1, 2).contiguous()   # NCHW like model.py:56
        clipped = no_backward(out["clipped"], "ImageCompressor (training mode, no grad)", params,
                              input_image)
        return clipped, y_hat, bpp

    def _eval_autograd(self, x):
        """model.py:47-80 in eval mode with autograd on. torch.round (model.py:56) has a zero
        gradient, so nothing flows back into the encoder or the image; the reconstruction is
        differentiable in the synthesis parameters (the fused synthesis forward/backward,
        autograd.SynthesisFn) and the rate in the BitEstimator parameters (model.py:71-78 on
        the module's autograd kernels). The encoder's parameters and the image get no gradient
        where torch would give zeros."""
        B, _, H, W = x.shape
        with torch.no_grad():
            y_hat = self.encode_latents(x)["y_hat"].permute(0, 3, 1, 2).contiguous()
        recon = self.Decoder(y_hat)
        clipped = recon.clamp(0., 1.)                                        # model.py:59
        prob = self.bitEstimator(y_hat + 0.5) - self.bitEstimator(y_hat - 0.5)   # model.py:71-72
        total_bits = torch.sum(torch.clamp(-1.0 * torch.log(prob + 1e-10) / math.log(2.0), 0, 50))
        bpp = total_bits / (B * H * W)                                       # model.py:76-78
        return clipped, y_hat, bpp

    def _train_outputs(self, x, noise, params):
        from .autograd import CodecTrainFn
        kernels._check(x, "image", 4)
        if noise is None:
            noise = self._latent_noise(x)
        self._warm_packs(backward=True)   # one batched pack per parameter update
        return CodecTrainFn.apply(x.contiguous(), noise.contiguous(), self, *params)

    def forward_train(self, input_image, noise: Optional[torch.Tensor] = None):
        """The tuple train.py:97 unpacks, as model.py:81 intends:
        (clipped_recon, mse of the UNclipped recon (model.py:61), bpp), all differentiable."""
        clipped, _, bpp, mse = self._train_outputs(input_image, noise, list(self.parameters()))
        return clipped, mse, bpp

    # ------------------------------------------------------------- entropy coding (§8 f4)
    @torch.no_grad()
    def compress(self, x: torch.Tensor, streams_per_image: int = kernels.STREAMS_PER_IMAGE,
                 K: int = kernels.ENTROPY_K) -> Dict[str, object]:
        """Encode images to byte strings: the analysis transform, rounding, then rANS over the
        factorised BitEstimator (the model the reference uses only to estimate bpp). Per image:
        P little-endian uint32 stream word counts, then the stream words (uint16 LE).
        Returns {"strings": [bytes] * B, "shape": (h, w), "streams_per_image": P, "K": K}."""
        y_hat = self.encode_latents(x)["y_hat"]
        if kernels.precision() == "h3" and kernels.h3_range_overflowed(x.device):
            # an activation did not fit the h3 form (conv3 wrote ŷ as NaN): encode from the x6
            # chain's ŷ instead (full fp32 operands). The flag read is one synchronisation, and
            # the stream sizes below synchronise anyway.
            kernels.set_precision("x6")
            try:
                y_hat = self.encode_latents(x)["y_hat"]
            finally:
                kernels.set_precision("h3")
        B, h, w, N = y_hat.shape
        P = streams_per_image
        words, offsets = kernels.rans_encode(y_hat, self.bitEstimator.entropy_tables(K), K, P)
        off = offsets.cpu().numpy()
        wv = words.cpu().numpy().view("<u2")
        strings = []
        for b in range(B):
            o = off[b * P:(b + 1) * P + 1]
            strings.append(np.diff(o).astype("<u4").tobytes() + wv[o[0]:o[-1]].tobytes())
        return {"strings": strings, "shape": (h, w), "streams_per_image": P, "K": K}

    @torch.no_grad()
    def decompress(self, strings, shape, streams_per_image: int = kernels.STREAMS_PER_IMAGE,
                   K: int = kernels.ENTROPY_K, device=None) -> Dict[str, torch.Tensor]:
        """Inverse of ``compress``: byte strings → {"y_hat": NCHW latents, "x_hat": the clipped
        reconstruction} (bit-identical latents; the synthesis as in ``forward``)."""
        P, N = streams_per_image, self.out_channel_N
        h, w = shape
        device = device or next(self.parameters()).device
        counts, payload = [], []
        for sbytes in strings:
            head = np.frombuffer(sbytes[:4 * P], dtype="<u4")
            if head.size != P:
                raise kernels.Iclr17Error("iclr17: decompress: truncated stream header")
            body = np.frombuffer(sbytes[4 * P:], dtype="<u2")
            if body.size != int(head.sum()):
                raise kernels.Iclr17Error("iclr17: decompress: stream lengths do not match the payload")
            counts.append(head.astype(np.int64))
            payload.append(body)
        B = len(strings)
        off = np.concatenate([[0], np.cumsum(np.concatenate(counts))]).astype(np.int64)
        words = torch.from_numpy(np.concatenate(payload).view(np.int16).copy()).to(device)
        offsets = torch.from_numpy(off).to(device)
        y_hat = kernels.rans_decode(words, offsets, self.bitEstimator.entropy_tables(K), B, h, w, N,
                                    K, P)
        split = kernels.split_planes(y_hat) if kernels.precision() == "x6" else None
        if kernels.precision() == "h3":
            kernels.h3_chain_begin(y_hat.device)
        yh3 = kernels.h3_planes(y_hat, cm=kernels.DECONV_CM) if kernels.precision() == "h3" else None
        ybf = kernels.to_bf16(y_hat) if kernels.precision() == "bf16" else None
        clipped, _, _ = self.Decoder.decode(y_hat, want_recon=False, y_split=split, y_bf16=ybf,
                                            y_integral=True, y_h3=yh3)
        return {"y_hat": y_hat.permute(0, 3, 1, 2).contiguous(), "x_hat": clipped}

    @torch.no_grad()
    def evaluate(self, x: torch.Tensor, want_y: bool = False,
                 want_msssim: bool = False, h3_overflow: str = "nan") -> Dict[str, torch.Tensor]:
        """testKodak-style per-image metrics (train.py:157-190): bpp, MSE of the clipped
        reconstruction and PSNR per image, all from deterministic on-device reductions; with
        ``want_msssim`` also MS-SSIM (train.py:178, on the GPU) and MS-SSIM-DB (train.py:179).

        ``h3_overflow`` (the h3 mode: an activation of magnitude ≥ 2^22 does not fit the form):
        "nan" (default, no host synchronisation) — the reconstruction, bpp, MSE and PSNR of the
        batch come back NaN; "raise" — read the range flag (one synchronisation) and raise
        Iclr17Error; "x6" — read it and, when set, evaluate the batch again in the x6 mode (full
        fp32 operands) and return those results."""
        if h3_overflow not in ("nan", "raise", "x6"):
            raise kernels.Iclr17Error(f"iclr17: h3_overflow must be 'nan', 'raise' or 'x6' "
                                      f"(got {h3_overflow!r})")
        res = self._evaluate(x, want_y, want_msssim)
        if h3_overflow != "nan" and kernels.precision() == "h3" and \
                kernels.h3_range_overflowed(x.device):
            if h3_overflow == "raise":
                raise kernels.Iclr17Error(kernels.H3_RANGE_MESSAGE)
            kernels.set_precision("x6")
            try:
                res = self._evaluate(x, want_y, want_msssim)
            finally:
                kernels.set_precision("h3")
        return res

    def _evaluate(self, x, want_y, want_msssim):
        B, _, H, W = x.shape
        out = self.run(x, training=False, x_ref_sse=True, want_y=want_y)
        bits = out.get("bits_per_image")
        if bits is None:
            bits, _ = kernels.reduce_partials(out["bits_partial"])
        sse, _ = kernels.reduce_partials(out["sse_partial"])
        bpp = bits / (H * W)
        mse = sse / (3 * H * W)
        psnr = 10.0 * torch.log10(1.0 / mse)
        res = {"clipped": out["clipped"], "y_hat": out["y_hat"].permute(0, 3, 1, 2).contiguous(),
               "bpp": bpp, "mse": mse, "psnr": psnr}
        if want_y:
            res["y"] = out["y"].permute(0, 3, 1, 2).contiguous()
        if want_msssim:
            ms = kernels.ms_ssim(out["clipped"], x, data_range=1.0)
            res["ms_ssim"] = ms
            res["ms_ssim_db"] = -10 * (torch.log(1 - ms) / math.log(10))
        return res

    def _warm_packs(self, backward: bool = False) -> None:
        """Build (or refresh) every derived parameter layout ``run`` reads (with ``backward``
        also those of the training backward) on the current stream, the stale ones as one
        batched packing launch pair (kernels.batched_packs)."""
        x6 = kernels.precision() != "fp32"
        gdns = (self.Encoder.gdn1, self.Encoder.gdn2, self.Decoder.igdn1, self.Decoder.igdn2)
        h3 = kernels.precision() == "h3"
        with kernels.batched_packs():
            if h3 and backward:   # an h3 training step reads only these fp32 packings
                self.Encoder.packed_w3()
                self.Decoder.packed_d3()
                for g in gdns:
                    g.effective_params()
            else:
                self.Encoder.packed()
                self.Decoder.packed()
            self.bitEstimator.packed()
            if x6:
                if not (h3 and backward):   # the x6 forward's (an h3 training step has none)
                    self.Encoder.packed_conv1_x6()
                    self.Encoder.packed_w3_split()
                    self.Decoder.packed_x6()
                    for g in gdns:
                        g.effective_params_x6()
            if backward:
                self.Encoder.packed_bwd()
                self.Decoder.packed_bwd(x6)
                for g in gdns:
                    if x6:
                        g.effective_params_bwd_x6()
                    else:
                        g.effective_params_bwd()
        if h3:
            # the h3 layouts (the codec's, and the training forward's in this mode) split the
            # packs above, which the batch writes only at its exit; they form a batch of their own
            with kernels.batched_h3_packs():
                self.Decoder.packed_h3k()
                self.Encoder.packed_h3()
                self.Encoder.packed_conv1_h3()
                for g in gdns:
                    g.effective_params_h3()
        if not backward:   # eval: the rate table of the round quantiser (+ the bf16 layouts)
            self.bitEstimator.rate_table()
            if kernels.precision() == "bf16":
                self.Encoder.packed_bf16()
                self.Decoder.packed_bf16()
                for g in gdns:
                    g.effective_params_bf16()

    def evaluate_many(self, batches, want_y: bool = False,
                      want_msssim: bool = False):
        """``evaluate`` of several batches (e.g. Kodak's landscape and portrait images, which
        cannot share one batch) on concurrent HIP streams: the first on the current stream, each
        other on a side stream, so one batch's partly filled last round of workgroups in every
        layer overlaps the other's work. Same kernels and inputs per batch, so the results are
        bitwise those of sequential ``evaluate`` calls."""
        batches = list(batches)
        if len(batches) <= 1 or not batches[0].is_cuda:
            return [self.evaluate(b, want_y=want_y, want_msssim=want_msssim) for b in batches]
        cur = torch.cuda.current_stream(batches[0].device)
        streams = getattr(self, "_side_streams", [])
        while len(streams) < len(batches) - 1:
            streams.append(torch.cuda.Stream(device=batches[0].device))
        self._side_streams = streams
        self._warm_packs()   # packs are written on cur before any side stream reads them
        outs = [None] * len(batches)
        for i, b in enumerate(batches):
            if i == 0:
                continue
            s = streams[i - 1]
            s.wait_stream(cur)
            b.record_stream(s)
            with torch.cuda.stream(s):
                outs[i] = self.evaluate(b, want_y=want_y, want_msssim=want_msssim)
        outs[0] = self.evaluate(batches[0], want_y=want_y, want_msssim=want_msssim)
        for i in range(1, len(batches)):
            cur.wait_stream(streams[i - 1])
            for t in outs[i].values():
                if isinstance(t, torch.Tensor):
                    t.record_stream(cur)
        return outs
