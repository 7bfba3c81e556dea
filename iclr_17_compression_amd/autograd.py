"""Autograd glue for the HIP kernels (forward and backward both run in libiclr17.so).

* ``CodecTrainFn`` — the fused training step of ImageCompressor (model.py:47-80 with the loss
  terms train.py:97-102 intends): outputs (clipped, ỹ, bpp, mse_unclipped); its backward is the
  reference autograd graph of ``rd_loss.backward()`` (train.py:105) as fused kernels.
* ``AnalysisFn`` / ``SynthesisFn`` — Encoder / Decoder used on their own (NewTests-style
  callers, train_decoder_new.py:66-105 trains a Decoder alone).
* ``GDNFn`` / ``BitEstimatorFn`` / ``BitparmFn`` — the stand-alone modules with their own
  backward kernels.
* Where no backward is wired (ImageCompressor.forward in eval mode with autograd on), outputs
  carry a grad_fn that raises instead of silently producing wrong gradients.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

from . import kernels

Tensor = torch.Tensor


class _NoBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, name, out, *inputs):
        ctx.name = name
        return out.view_as(out)

    @staticmethod
    def backward(ctx, *grads):
        raise NotImplementedError(f"iclr17: backward of {ctx.name} is not implemented by the HIP path yet")


def no_backward(out: Tensor, name: str, params: Sequence[Tensor], x: Tensor):
    needs = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
    if not needs:
        return out
    return _NoBackward.apply(name, out, x, *params)


def gdn_apply(x: Tensor, module) -> Tensor:
    if needs_grad(x, (module.beta, module.gamma)):
        return GDNFn.apply(x, module, module.beta, module.gamma)
    beta_eff, gp = module.effective_params()
    return kernels.gdn(x, beta_eff, gp, module.inverse)


class GDNFn(torch.autograd.Function):
    """Stand-alone GDN / IGDN (GDN.py:64-94) with its autograd: ∂x from the fused backward
    kernel, ∂β / ∂γ through GDN.py:73-79 (LowerBound's gradient rule included)."""

    @staticmethod
    def forward(ctx, x, module, beta, gamma):
        beta_eff, gp = module.effective_params()
        ctx.module = module
        ctx.save_for_backward(x)
        return kernels.gdn(x, beta_eff, gp, module.inverse)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        m = ctx.module
        be, gp, gpt = m.effective_params_bwd()
        dx, dn, u = kernels.gdn_backward(x, g, be, gp, gpt, m.inverse)
        bb, gb, _ = m.bounds_f32()
        dbeta, dgamma = kernels.gdn_param_grads(dn, u, kernels.bias_grad_nhwc(dn), m.beta, m.gamma,
                                                bb, gb)
        return dx, None, dbeta.view_as(m.beta), dgamma.view_as(m.gamma)


class BitEstimatorFn(torch.autograd.Function):
    """BitEstimator.forward (bitEstimator.py:38-42) with its autograd."""

    @staticmethod
    def forward(ctx, x, module, *params):
        ctx.module = module
        ctx.save_for_backward(x)
        return kernels.bit_estimator(x, module.packed(), module.channel)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        m = ctx.module
        dx, part = kernels.bit_estimator_backward(x, g, m.packed(), m.channel)
        grads = kernels.rate_param_grads(part, m.params_in_order())
        return (dx.view_as(x), None, *[gr.view_as(p) for gr, p in zip(grads, m.params_in_order())])


class BitparmFn(torch.autograd.Function):
    """One Bitparm layer (bitEstimator.py:20-25) with its autograd."""

    @staticmethod
    def forward(ctx, x, module, *params):
        ctx.module = module
        ctx.save_for_backward(x)
        return kernels.bitparm(x, module.h, module.b, module.a)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        m = ctx.module
        dx, part = kernels.bitparm_backward(x, g, m.h, m.b, m.a)
        if m.a is not None:   # slots 0-2 of the rate table: (h, b, a) as BitEstimator's f1
            grads = kernels.rate_param_grads(part, [m.h, m.b, m.a] * 3 + [m.h, m.b])[:3]
        else:                 # slots 9-10: the final layer's (h, b)
            grads = kernels.rate_param_grads(part, [m.h, m.b, m.h] * 3 + [m.h, m.b])[9:]
        ps = [p for p in (m.h, m.b, m.a) if p is not None]
        return (dx.view_as(x), None, *[gr.view_as(p) for gr, p in zip(grads, ps)])


def needs_grad(x: Optional[Tensor], params: Sequence[Tensor]) -> bool:
    return torch.is_grad_enabled() and ((x is not None and x.requires_grad) or
                                        any(p.requires_grad for p in params))


def _split_of(saved: Dict[str, Tensor], key: str) -> Tensor:
    """The split form of a saved activation (kept from the x6 forward, or split now)."""
    s = saved.get(key + "s")
    return s if s is not None else kernels.split_planes(saved[key])


# ------------------------------------------------------------------------------ analysis
def analysis_features_train(enc, x: Tensor):
    """conv1+GDN1, conv2+GDN2 keeping the pre-activations the backward needs. In the x6 mode the
    kernels also hand conv2 (and conv3) their input in split form; "a2s" is then set. In the h3
    mode the forward runs the codec's own h3 kernels, which also write the split forms (the x6
    weight-gradient operands) and the pre-activations; "a2h" (conv3's h3 input) is then set."""
    N = enc.out_channel_N
    if kernels.precision() == "h3":
        kernels.h3_chain_begin(x.device)
        ge1, ge2 = enc.gdn1.effective_params_h3(), enc.gdn2.effective_params_h3()
        w2h, _ = enc.packed_h3()
        a1h, _, a1s, u1 = kernels.conv1_gdn_h3(x, enc.packed_conv1_h3(), enc.conv1.bias, *ge1, N,
                                               want_x6=True, want_pre=True)
        a2h, _, a2s, u2 = kernels.conv2_gdn_h3(a1h, w2h, enc.conv2.bias, *ge2, want_x6=True,
                                               want_pre=True)
        return None, {"x": x, "u1": u1, "u2": u2, "a1s": a1s, "a2s": a2s, "a2h": a2h}
    w1, w2, _, g1, g2 = enc.packed()
    if kernels.precision() != "fp32":
        e1, e2 = enc.gdn1.effective_params_x6(), enc.gdn2.effective_params_x6()
        a1s, a1, u1 = kernels.conv1x6_gdn(x, enc.packed_conv1_x6(), enc.conv1.bias, e1[0], e1[2],
                                          N, want_f32=True, want_pre=True)
        a2s, a2, u2 = kernels.conv2_gdn_x6(a1s, w2, enc.conv2.bias, *e2, want_f32=True,
                                           want_pre=True)
        return a2, {"x": x, "u1": u1, "a1": a1, "u2": u2, "a2": a2, "a2s": a2s, "a1s": a1s}
    a1, u1 = kernels.conv1_gdn(x, w1, enc.conv1.bias, g1[0], g1[1], N, want_pre=True)
    a2, u2 = kernels.conv2_gdn(a1, w2, enc.conv2.bias, g2[0], g2[1], want_pre=True)
    return a2, {"x": x, "u1": u1, "a1": a1, "u2": u2, "a2": a2, "a2s": None, "a1s": None}


def conv1_input_grad(enc, g_u1: Tensor) -> Tensor:
    """∂L/∂x of conv1 (analysis_17.py:32, k9 s4 p4): the transposed convolution of ∂L/∂u1
    (NHWC) with conv1's own weights — the shape and arithmetic of deconv3 (k9 s4 p4 op3, N → 3),
    so it runs on the exact-f32 deconv3 kernel with conv1.weight in deconv3's packing, a zero
    bias and the unclipped output."""
    w = enc.packed_conv1_t()
    zero = torch.zeros(3, device=g_u1.device, dtype=torch.float32)
    _, dx, _ = kernels.deconv3(g_u1.contiguous(), w, zero, want_recon=True)
    return dx


def analysis_backward(enc, saved: Dict[str, Tensor], g_y: Tensor,
                      g_y_split: Optional[Tensor] = None, want_dx: bool = False) -> Dict[str, Tensor]:
    """∂L/∂y (NHWC) → parameter gradients of Analysis_net_17 (analysis_17.py:14-39). In the x6
    mode the input-gradient contractions run on split-form gradients (g_y_split, or split here)."""
    bb1, gb1, _ = enc.gdn1.bounds_f32()
    bb2, gb2, _ = enc.gdn2.bounds_f32()
    w3t, w2t = enc.packed_bwd()
    x6 = kernels.precision() != "fp32"
    p2 = None if x6 else enc.gdn2.effective_params_bwd()
    p1 = None if x6 else enc.gdn1.effective_params_bwd()
    if kernels.precision() != "fp32":
        if g_y_split is None:
            g_y_split = kernels.split_planes(g_y)
        x2, x1 = enc.gdn2.effective_params_bwd_x6(), enc.gdn1.effective_params_bwd_x6()
        a2s, a1s = _split_of(saved, "a2"), _split_of(saved, "a1")
        dW3 = kernels.wgrad_k5_x6(g_y_split, a2s)
        g_u2, dn2, db2, dbe2, g_u2s = kernels.bwd_conv_gdn(g_y, w3t, saved["u2"], *x2[:3],
                                                           g_split=g_y_split, want_split=True,
                                                           g6=x2[3], g6t=x2[4], want_f32=False)
        dW2 = kernels.wgrad_k5_x6(g_u2s, a1s)
        dg2 = kernels.gdn_param_grads(dn2, saved["u2"], dbe2, enc.gdn2.beta,
                                                     enc.gdn2.gamma, bb2, gb2)
        g_u1, dn1, db1, dbe1, g_u1s = kernels.bwd_conv_gdn(g_u2, w2t, saved["u1"], *x1[:3],
                                                           g_split=g_u2s, want_split=True,
                                                           g6=x1[3], g6t=x1[4], want_f32=want_dx)
        dW1 = kernels.wgrad_k9_x6(g_u1s, saved["x"])
    else:
        dW3 = kernels.wgrad_k5(g_y, saved["a2"])
        g_u2, dn2, db2, dbe2 = kernels.bwd_conv_gdn(g_y, w3t, saved["u2"], *p2)
        dW2 = kernels.wgrad_k5(g_u2, saved["a1"])
        dg2 = kernels.gdn_param_grads(dn2, saved["u2"], dbe2, enc.gdn2.beta,
                                                     enc.gdn2.gamma, bb2, gb2)
        g_u1, dn1, db1, dbe1 = kernels.bwd_conv_gdn(g_u2, w2t, saved["u1"], *p1)
        dW1 = kernels.wgrad_k9(g_u1, saved["x"])
    dbeta2, dgamma2 = dg2
    dbeta1, dgamma1 = kernels.gdn_param_grads(dn1, saved["u1"], dbe1, enc.gdn1.beta,
                                                             enc.gdn1.gamma, bb1, gb1)
    grads = {"conv1.weight": dW1, "conv1.bias": db1, "gdn1.beta": dbeta1, "gdn1.gamma": dgamma1,
             "conv2.weight": dW2, "conv2.bias": db2, "gdn2.beta": dbeta2, "gdn2.gamma": dgamma2,
             "conv3.weight": dW3}
    if want_dx:
        grads["x"] = conv1_input_grad(enc, g_u1)
    return grads


# ----------------------------------------------------------------------------- synthesis
def synthesis_forward_train(dec, y_nhwc: Tensor, x_ref: Optional[Tensor] = None,
                            y_split: Optional[Tensor] = None, y_h3: Optional[Tensor] = None):
    if kernels.precision() == "h3":
        # the codec's h3 kernels; their x6 outputs are the weight-gradient operands and the
        # pre-activations the IGDN backward's
        if y_h3 is None:   # the Decoder on its own: its chain starts here
            kernels.h3_chain_begin(y_nhwc.device)
            y_h3 = kernels.h3_planes(y_nhwc, cm=kernels.DECONV_CM)
        h1, h2 = dec.igdn1.effective_params_h3(), dec.igdn2.effective_params_h3()
        x1, x2, x3 = dec.packed_h3k()
        s1h, _, s1s, v1 = kernels.deconv_igdn_h3(y_h3, x1, dec.deconv1.bias, *h1, want_x6=True,
                                                 want_pre=True)
        s2h, _, s2s, v2 = kernels.deconv_igdn_h3(s1h, x2, dec.deconv2.bias, *h2, want_x6=True,
                                                 want_pre=True, chunk_major=True)
        clipped, recon, sse = kernels.deconv3_h3(s2h, x3, dec.deconv3.bias, x_ref=x_ref,
                                                 want_recon=True, sse_unclipped=x_ref is not None)
        return clipped, recon, sse, {"y": y_nhwc, "v1": v1, "v2": v2, "s1s": s1s, "s2s": s2s}
    d1, d2, d3, q1, q2 = dec.packed()
    if kernels.precision() != "fp32":
        if y_split is None:
            y_split = kernels.split_planes(y_nhwc)
        e1, e2 = dec.igdn1.effective_params_x6(), dec.igdn2.effective_params_x6()
        s1s, s1, v1 = kernels.deconv_igdn_x6(y_split, d1, dec.deconv1.bias, *e1, want_f32=True,
                                             want_pre=True)
        # NHWC split (not chunk-major): s2s is also deconv3's x6 weight-gradient operand
        s2s, s2, v2 = kernels.deconv_igdn_x6(s1s, d2, dec.deconv2.bias, *e2, want_f32=True,
                                             want_pre=True)
        clipped, recon, sse = kernels.deconv3_x6(s2s, dec.packed_x6(), dec.deconv3.bias, x_ref=x_ref,
                                                 want_recon=True, sse_unclipped=x_ref is not None)
        # the split forms of y and s1 are the x6 weight-gradient operands
        return clipped, recon, sse, {"y": y_nhwc, "v1": v1, "s1": s1, "v2": v2, "s2": s2,
                                     "ys": y_split, "s1s": s1s, "s2s": s2s}
    s1, v1 = kernels.deconv_igdn(y_nhwc, d1, dec.deconv1.bias, q1[0], q1[1], want_pre=True)
    s2, v2 = kernels.deconv_igdn(s1, d2, dec.deconv2.bias, q2[0], q2[1], want_pre=True)
    clipped, recon, sse = kernels.deconv3(s2, d3, dec.deconv3.bias, x_ref=x_ref,
                                          want_recon=True, sse_unclipped=x_ref is not None)
    return clipped, recon, sse, {"y": y_nhwc, "v1": v1, "s1": s1, "v2": v2, "s2": s2}


def synthesis_backward(dec, saved: Dict[str, Tensor], g_recon: Tensor, g_bpp: Optional[Tensor] = None,
                       rate_packed: Optional[Tensor] = None, count: float = 0.0,
                       want_split: bool = False):
    """∂L/∂recon (NCHW) → (∂L/∂ỹ NHWC incl. the rate term when g_bpp is given, parameter
    gradients of Synthesis_net_17, rate-parameter partials[, ∂L/∂ỹ in split form (x6 mode,
    else None)]). In the x6 mode the input-gradient contractions run in x6, each kernel handing
    the next its gradient in split form."""
    x6 = kernels.precision() != "fp32"
    N = dec.out_channel_N
    bq1, gq1, _ = dec.igdn1.bounds_f32()
    bq2, gq2, _ = dec.igdn2.bounds_f32()
    d3p, d2c, d1c = dec.packed_bwd(x6)
    d3c, d3x = (None, d3p) if x6 else (d3p, None)
    q2 = dec.igdn2.effective_params_bwd_x6() if x6 else dec.igdn2.effective_params_bwd()
    q1 = dec.igdn1.effective_params_bwd_x6() if x6 else dec.igdn1.effective_params_bwd()
    y = saved["y"]
    B, h, w, _ = y.shape
    g_ys = None
    gdn_q2 = lambda: kernels.gdn_param_grads(dnq2, saved["v2"], dbeq2, dec.igdn2.beta,  # noqa: E731
                                             dec.igdn2.gamma, bq2, gq2)
    gdn_q1 = lambda: kernels.gdn_param_grads(dnq1, saved["v1"], dbeq1, dec.igdn1.beta,  # noqa: E731
                                             dec.igdn1.gamma, bq1, gq1)
    if x6:
        s2s, s1s = _split_of(saved, "s2"), _split_of(saved, "s1")
        ys = saved.get("ys") if saved.get("ys") is not None else kernels.split_planes(y)
        dWd3 = kernels.wgrad_k9_x6(s2s, g_recon)
        dbd3 = kernels.bias_grad_nchw(g_recon)
        g_v2, dnq2, dbd2, dbeq2, g_v2s = kernels.bwd_deconv3_igdn(g_recon, None, saved["v2"], *q2[:3],
                                                                  w_split=d3x, want_split=True,
                                                                  g6=q2[3], g6t=q2[4], want_f32=False)
        dWd2 = kernels.wgrad_k5_x6(s1s, g_v2s)
        dq2 = gdn_q2()
        g_v1, dnq1, dbd1, dbeq1, g_v1s = kernels.bwd_deconv_igdn(g_v2, d2c, saved["v1"], *q1[:3],
                                                                 g_split=g_v2s, want_split=True,
                                                                 g6=q1[3], g6t=q1[4], want_f32=False)
        dWd1 = kernels.wgrad_k5_x6(ys, g_v1s)
        dq1 = gdn_q1()
        r = kernels.bwd_deconv_rate(g_v1, d1c, y if g_bpp is not None else None, rate_packed,
                                    g_bpp, count, h, w, g_split=g_v1s, want_split=want_split)
        g_y, rpart, g_ys = r if want_split else (*r, None)
    else:
        dWd3 = kernels.wgrad_k9(saved["s2"], g_recon)
        dbd3 = kernels.bias_grad_nchw(g_recon)
        g_v2, dnq2, dbd2, dbeq2 = kernels.bwd_deconv3_igdn(g_recon, d3c, saved["v2"], *q2)
        dWd2 = kernels.wgrad_k5(saved["s1"], g_v2)
        dq2 = gdn_q2()
        g_v1, dnq1, dbd1, dbeq1 = kernels.bwd_deconv_igdn(g_v2, d2c, saved["v1"], *q1)
        dWd1 = kernels.wgrad_k5(y, g_v1)
        dq1 = gdn_q1()
        g_y, rpart = kernels.bwd_deconv_rate(g_v1, d1c, y if g_bpp is not None else None,
                                             rate_packed, g_bpp, count, h, w)
    dbq2, dgq2 = dq2
    dbq1, dgq1 = dq1
    grads = {"deconv1.weight": dWd1, "deconv1.bias": dbd1, "igdn1.beta": dbq1, "igdn1.gamma": dgq1,
             "deconv2.weight": dWd2, "deconv2.bias": dbd2, "igdn2.beta": dbq2, "igdn2.gamma": dgq2,
             "deconv3.weight": dWd3, "deconv3.bias": dbd3}
    return (g_y, grads, rpart, g_ys) if want_split else (g_y, grads, rpart)


def _ordered(module, prefix: str, grads: Dict[str, Tensor]) -> List[Optional[Tensor]]:
    return [grads.get(name) for name, _ in module.named_parameters()]


# --------------------------------------------------------------------------- Functions
class CodecTrainFn(torch.autograd.Function):
    """ImageCompressor training forward: (clipped, ỹ NCHW-view, bpp, mse of unclipped recon)."""

    @staticmethod
    def forward(ctx, x, noise, net, *params):
        ctx.set_materialize_grads(False)
        enc, dec, be = net.Encoder, net.Decoder, net.bitEstimator
        B, _, H, W = x.shape
        a2, saved_a = analysis_features_train(enc, x)
        w3 = enc.packed_w3()
        rate = be.packed()
        a2s, a2h, y_h3 = saved_a.get("a2s"), saved_a.get("a2h"), None
        if a2h is not None:   # h3: conv3 + quantiser on the codec's h3 kernel, ỹ also in h3
            y_tilde, bits_part, _, y_h3 = kernels.conv3_quant_rate_h3(a2h, enc.packed_h3()[1], rate,
                                                                      noise)
            y_split = None
        elif a2s is not None:
            y_tilde, bits_part, _, y_split = kernels.conv3_quant_rate_x6(a2s, w3, rate, noise)
        else:
            (y_tilde, bits_part), y_split = kernels.conv3_quant_rate(a2, w3, rate, noise), None
        clipped, recon, sse_part, saved_s = synthesis_forward_train(dec, y_tilde, x_ref=x,
                                                                    y_split=y_split, y_h3=y_h3)
        _, bpp = kernels.reduce_partials(bits_part, 1.0 / (B * H * W), per_image=False)
        _, mse = kernels.reduce_partials(sse_part, 1.0 / (B * 3 * H * W), per_image=False)
        ctx.net = net
        ctx.saved_a, ctx.saved_s = saved_a, saved_s
        ctx.recon, ctx.x, ctx.rate, ctx.count = recon, x, rate, float(B * H * W)
        return clipped, y_tilde.permute(0, 3, 1, 2), bpp, mse

    @staticmethod
    def backward(ctx, g_clipped, g_ytilde, g_bpp, g_mse):
        net = ctx.net
        enc, dec, be = net.Encoder, net.Decoder, net.bitEstimator
        grads: List[Optional[Tensor]] = []
        if g_clipped is None and g_mse is None:
            g_recon = torch.zeros_like(ctx.recon)
        else:
            g_recon = kernels.grad_recon(ctx.recon, ctx.x, g_mse, g_clipped)
        g_y, gs, rpart, g_ys = synthesis_backward(dec, ctx.saved_s, g_recon, g_bpp, ctx.rate,
                                                  ctx.count, want_split=g_ytilde is None)
        red = getattr(net, "_grad_reducer", None)
        red = red if red is not None and red.active else None
        if red is not None:   # the synthesis gradients all-reduce during the analysis backward
            red.launch(list(dec.parameters()), _ordered(dec, "", gs))
        if g_ytilde is not None:
            g_y = g_y + g_ytilde.permute(0, 2, 3, 1)
        want_dx = ctx.needs_input_grad[0]
        rg = (kernels.rate_param_grads(rpart, be.params_in_order())
              if g_bpp is not None else [None] * 11)
        ga = analysis_backward(enc, ctx.saved_a, g_y.contiguous(), g_ys, want_dx=want_dx)
        grads += _ordered(enc, "Encoder.", ga)
        grads += _ordered(dec, "Decoder.", gs)
        names = [n for n, _ in be.named_parameters()]
        order = ["f1.h", "f1.b", "f1.a", "f2.h", "f2.b", "f2.a", "f3.h", "f3.b", "f3.a", "f4.h", "f4.b"]
        rmap = dict(zip(order, rg))
        grads += [rmap[n] for n in names]
        if red is not None:
            red.launch(list(enc.parameters()) + list(be.parameters()),
                       _ordered(enc, "", ga) + [rmap[n] for n in names])
        dx = ga.get("x")
        if dx is not None and g_mse is not None:   # the loss's own x: ∂mse/∂x = −∂mse/∂recon
            dx = dx - kernels.grad_recon(ctx.recon, ctx.x, g_mse, None)
        ctx.saved_a = ctx.saved_s = ctx.recon = None
        return (dx, None, None, *grads)


class AnalysisFn(torch.autograd.Function):
    """Analysis_net_17.forward with autograd: y, contiguous NCHW, from the codec's own analysis
    kernels (``Analysis_net_17.y_nhwc``), so round(y) is the codec's ŷ with grad on or off."""

    @staticmethod
    def forward(ctx, x, enc, *params):
        ctx.set_materialize_grads(False)
        _, saved = analysis_features_train(enc, x)   # a2s stays: conv3's x6 weight gradient
        ctx.enc, ctx.saved = enc, saved
        return enc.y_nhwc(x, feats=saved).permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def backward(ctx, g_y):
        if g_y is None:
            return (None, None) + (None,) * len(list(ctx.enc.parameters()))
        ga = analysis_backward(ctx.enc, ctx.saved, g_y.permute(0, 2, 3, 1).contiguous(),
                               want_dx=ctx.needs_input_grad[0])
        ctx.saved = None
        return (ga.get("x"), None, *_ordered(ctx.enc, "", ga))


class SynthesisFn(torch.autograd.Function):
    """Synthesis_net_17.forward with autograd: unclipped reconstruction (NCHW)."""

    @staticmethod
    def forward(ctx, y, dec, *params):
        ctx.set_materialize_grads(False)
        _, recon, _, saved = synthesis_forward_train(dec, dec.to_nhwc(y))
        ctx.dec, ctx.saved = dec, saved
        return recon

    @staticmethod
    def backward(ctx, g_recon):
        n_params = len(list(ctx.dec.parameters()))
        if g_recon is None:
            return (None, None) + (None,) * n_params
        g_y, gs, _ = synthesis_backward(ctx.dec, ctx.saved, g_recon.contiguous())
        ctx.saved = None
        return (g_y.permute(0, 3, 1, 2), None, *_ordered(ctx.dec, "", gs))
