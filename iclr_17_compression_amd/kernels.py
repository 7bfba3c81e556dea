"""Tensor-level wrappers over the C ABI (include/iclr17.h).

Each function validates shapes / dtypes / devices, allocates outputs with PyTorch's caching
allocator, and enqueues the HIP kernel on the current stream of the tensors' device. There
is no CPU path: a non-GPU tensor raises.

Activations between layers are NHWC tensors (shape [B, h, w, N], contiguous); the image and
the reconstruction are NCHW. Parameters stay in their reference (NCHW / PyTorch) layout and
are packed into kernel layouts by the ``pack_*`` helpers (derived caches).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import Iclr17Error, call, query

Tensor = torch.Tensor

# models/GDN.py:46-49 default bounds as the fp32 values ones_like(x) * bound produces
DEFAULT_BETA_BOUND = float(np.float32((1e-6 + 2.0 ** -36) ** 0.5))
DEFAULT_GAMMA_BOUND = float(np.float32(2.0 ** -18))
DEFAULT_PEDESTAL = float(np.float32(2.0 ** -36))


def _check(t: Tensor, name: str, ndim: Optional[int] = None) -> None:
    if not isinstance(t, torch.Tensor):
        raise Iclr17Error(f"iclr17: {name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise Iclr17Error(
            f"iclr17: {name} is on {t.device}; this framework runs only on a ROCm GPU "
            "(MI355X / gfx950) — there is no CPU implementation")
    if t.dtype != torch.float32:
        raise Iclr17Error(f"iclr17: {name} must be float32 (got {t.dtype})")
    if ndim is not None and t.dim() != ndim:
        raise Iclr17Error(f"iclr17: {name} must be {ndim}-D (got shape {tuple(t.shape)})")


def _p(t: Optional[Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(t: Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check_image_dims(H: int, W: int) -> None:
    if H <= 0 or W <= 0 or H % 16 or W % 16:
        raise Iclr17Error(f"iclr17: image height/width must be positive multiples of 16, got {H}x{W} "
                          "(model.py:48 builds the latent grid with //16; crop first)")


def _check_channels(N: int) -> None:
    if N not in (128, 192):
        raise Iclr17Error(f"iclr17: channel count N={N} unsupported (kernels are built for 128 and 192)")


# ------------------------------------------------------------------------------ packing
class _PackJob(ctypes.Structure):
    """iclr17_pack_job (include/iclr17.h)."""
    _fields_ = [("kind", ctypes.c_int), ("N", ctypes.c_int), ("taps", ctypes.c_int),
                ("K", ctypes.c_int), ("src0", ctypes.c_void_p), ("src1", ctypes.c_void_p),
                ("dst0", ctypes.c_void_p), ("dst1", ctypes.c_void_p), ("dst2", ctypes.c_void_p),
                ("f0", ctypes.c_float), ("f1", ctypes.c_float), ("f2", ctypes.c_float)]


_deferred: Optional[list] = None   # queued pack jobs inside batched_packs()


def _ptr(t: Optional[Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


@contextlib.contextmanager
def batched_packs():
    """Inside the block, pack_weight / pack_gdn / pack_rate / split_packed allocate their
    outputs and queue the work; on exit it runs as one iclr17_pack_batch (two launches instead of
    one per pack). Nothing may read the outputs inside the block. Re-entrant (inner blocks join
    the outer batch)."""
    global _deferred
    if _deferred is not None:
        yield
        return
    _deferred = []
    try:
        yield
        jobs = _deferred
    finally:
        _deferred = None
    if not jobs:
        return
    arr = (_PackJob * len(jobs))(*[j[0] for j in jobs])
    rate = [j[2] for j in jobs if j[2] is not None]
    rate_arr = (ctypes.c_void_p * 11)(*rate[0]) if rate else None
    call("iclr17_pack_batch", ctypes.cast(arr, ctypes.c_void_p), len(jobs),
         None if rate_arr is None else ctypes.cast(rate_arr, ctypes.c_void_p), jobs[0][3])
    del jobs   # sources stay alive until here; the stream orders their reuse after the launch


def pack_weight(which: int, w: Tensor, N: int) -> Tensor:
    _check(w, "weight", 4)
    w = w.detach().contiguous()
    size = query("iclr17_packed_weight_size", which, N)
    out = torch.empty(size, device=w.device, dtype=torch.float32)
    if _deferred is not None:
        _deferred.append((_PackJob(which, N, 0, 0, _ptr(w), None, _ptr(out), None, None),
                          (w, out), None, _stream(w)))
        return out
    call("iclr17_pack_weight", which, _p(w), _p(out), N, _stream(w))
    return out


def pack_gdn(beta: Tensor, gamma: Tensor, beta_bound: float = DEFAULT_BETA_BOUND,
             gamma_bound: float = DEFAULT_GAMMA_BOUND, pedestal: float = DEFAULT_PEDESTAL,
             transposed: bool = False):
    """(beta_eff, gamma_packed[, gamma_packed_t]) — GDN.py:73-79 effective parameters."""
    _check(beta, "beta", 1)
    _check(gamma, "gamma", 2)
    C = beta.shape[0]
    if tuple(gamma.shape) != (C, C):
        raise Iclr17Error(f"iclr17: gamma must be [{C},{C}] (got {tuple(gamma.shape)})")
    beta = beta.detach().contiguous()
    gamma = gamma.detach().contiguous()
    beta_eff = torch.empty(C, device=beta.device, dtype=torch.float32)
    gp = torch.empty(C * C, device=beta.device, dtype=torch.float32)
    gpt = torch.empty(C * C, device=beta.device, dtype=torch.float32) if transposed else None
    if _deferred is not None:
        _deferred.append((_PackJob(_lib.ICLR17_PACK_GDN, C, 0, 0, _ptr(beta), _ptr(gamma),
                                   _ptr(beta_eff), _ptr(gp), _ptr(gpt), beta_bound, gamma_bound,
                                   pedestal), (beta, gamma, beta_eff, gp, gpt), None, _stream(beta)))
        return (beta_eff, gp, gpt) if transposed else (beta_eff, gp)
    call("iclr17_pack_gdn", _p(beta), _p(gamma), _p(beta_eff), _p(gp), _p(gpt), C,
         ctypes.c_float(beta_bound), ctypes.c_float(gamma_bound), ctypes.c_float(pedestal),
         _stream(beta))
    return (beta_eff, gp, gpt) if transposed else (beta_eff, gp)


def pack_rate(params: Sequence[Tensor]) -> Tensor:
    """params: h1 b1 a1 h2 b2 a2 h3 b3 a3 h4 b4 (each (1,C,1,1) or (C,))."""
    if len(params) != 11:
        raise Iclr17Error("iclr17: pack_rate needs 11 parameter tensors")
    ps = [p.detach().reshape(-1).contiguous() for p in params]
    for i, p in enumerate(ps):
        _check(p, f"rate param {i}")
    C = ps[0].numel()
    out = torch.empty(11 * C, device=ps[0].device, dtype=torch.float32)
    if _deferred is not None:
        if any(j[2] is not None for j in _deferred):
            raise Iclr17Error("iclr17: one rate pack per batched_packs() block")
        _deferred.append((_PackJob(_lib.ICLR17_PACK_RATE, C, 0, 0, None, None, _ptr(out), None, None),
                          (ps, out), [p.data_ptr() for p in ps], _stream(ps[0])))
        return out
    call("iclr17_pack_rate", *[_p(p) for p in ps], _p(out), C, _stream(ps[0]))
    return out


# ------------------------------------------------------------------------------ layers
def conv1_gdn(x: Tensor, wp: Tensor, bias: Tensor, beta_eff: Tensor, gp: Tensor, N: int,
              want_pre: bool = False):
    """analysis_17.py:14-17,33: x NCHW [B,3,H,W] → NHWC [B,H/4,W/4,N] (+ pre-GDN)."""
    _check(x, "image", 4)
    B, C, H, W = x.shape
    if C != 3:
        raise Iclr17Error(f"iclr17: the analysis transform takes 3-channel images (got {C})")
    _check_image_dims(H, W)
    _check_channels(N)
    x = x.contiguous()
    out = torch.empty(B, H // 4, W // 4, N, device=x.device, dtype=torch.float32)
    pre = torch.empty_like(out) if want_pre else None
    call("iclr17_analysis_conv1_gdn", _p(x), B, H, W, N, _p(wp), _p(bias), _p(beta_eff), _p(gp),
         _p(out), _p(pre), _stream(x))
    return (out, pre) if want_pre else out


def conv2_gdn(h: Tensor, wp: Tensor, bias: Tensor, beta_eff: Tensor, gp: Tensor,
              want_pre: bool = False):
    """analysis_17.py:18-21,34: NHWC [B,H/4,W/4,N] → [B,H/8,W/8,N]."""
    _check(h, "activation", 4)
    B, h4, w4, N = h.shape
    _check_channels(N)
    H, W = 4 * h4, 4 * w4
    _check_image_dims(H, W)
    out = torch.empty(B, h4 // 2, w4 // 2, N, device=h.device, dtype=torch.float32)
    pre = torch.empty_like(out) if want_pre else None
    call("iclr17_analysis_conv2_gdn", _p(h.contiguous()), B, H, W, N, _p(wp), _p(bias),
         _p(beta_eff), _p(gp), _p(out), _p(pre), _stream(h))
    return (out, pre) if want_pre else out


def conv3(h: Tensor, wp: Tensor) -> Tensor:
    """analysis_17.py:22,35 (no quantiser): NHWC [B,H/8,W/8,N] → y NHWC [B,H/16,W/16,N]."""
    _check(h, "activation", 4)
    B, h8, w8, N = h.shape
    _check_channels(N)
    H, W = 8 * h8, 8 * w8
    _check_image_dims(H, W)
    y = torch.empty(B, h8 // 2, w8 // 2, N, device=h.device, dtype=torch.float32)
    call("iclr17_analysis_conv3", _p(h.contiguous()), B, H, W, N, _p(wp), _p(y), _stream(h))
    return y


def rate_partials_per_image(H: int, W: int, N: int) -> int:
    return query("iclr17_rate_partials_per_image", H, W, N)


def conv3_quant_rate(h: Tensor, wp: Tensor, rate_packed: Tensor, noise: Optional[Tensor] = None,
                     want_y: bool = False, rtab: Optional[Tensor] = None):
    """analysis_17.py:22 + model.py:48-56,71-73. Returns (y_hat NHWC, bits_partial [B,T], y?).

    noise (training) is NCHW [B,N,H/16,W/16], the shape model.py:48 draws. rtab (``rate_table``
    of rate_packed, round mode): bits of the integer latents by lookup."""
    _check(h, "activation", 4)
    B, h8, w8, N = h.shape
    _check_channels(N)
    H, W = 8 * h8, 8 * w8
    _check_image_dims(H, W)
    mode = _lib.ICLR17_QUANT_ROUND
    if noise is not None:
        _check(noise, "noise", 4)
        if tuple(noise.shape) != (B, N, h8 // 2, w8 // 2):
            raise Iclr17Error(f"iclr17: noise must be {(B, N, h8 // 2, w8 // 2)} (got {tuple(noise.shape)})")
        noise = noise.contiguous()
        mode = _lib.ICLR17_QUANT_NOISE
    y_hat = torch.empty(B, h8 // 2, w8 // 2, N, device=h.device, dtype=torch.float32)
    y = torch.empty_like(y_hat) if want_y else None
    T = rate_partials_per_image(H, W, N)
    partial = torch.empty(B, T, device=h.device, dtype=torch.float64)
    call("iclr17_analysis_conv3_quant_rate", _p(h.contiguous()), B, H, W, N, _p(wp), mode,
         _p(noise), _p(rate_packed), _p(rtab), _p(y), _p(y_hat), _p(partial), _stream(h))
    return (y_hat, partial, y) if want_y else (y_hat, partial)


def deconv_igdn(h: Tensor, wp: Tensor, bias: Tensor, beta_eff: Tensor, gp: Tensor,
                want_pre: bool = False):
    """synthesis_17.py:15-22: NHWC [B,h,w,N] → [B,2h,2w,N]."""
    _check(h, "activation", 4)
    B, hh, ww, N = h.shape
    _check_channels(N)
    out = torch.empty(B, 2 * hh, 2 * ww, N, device=h.device, dtype=torch.float32)
    pre = torch.empty_like(out) if want_pre else None
    call("iclr17_synthesis_deconv_igdn", _p(h.contiguous()), B, hh, ww, N, _p(wp), _p(bias),
         _p(beta_eff), _p(gp), _p(out), _p(pre), _stream(h))
    return (out, pre) if want_pre else out


# ------------------------------------------------------------- x6 (bf16x6) precision mode
PRECISIONS = ("x6", "h3", "fp32", "bf16")
_precision = os.environ.get("ICLR17_PRECISION", "h3")


def precision() -> str:
    """Inference contraction mode: "h3" (the parity default: fp32 operands as two fp16 parts —
    22 significant bits, power-of-two scaled — three part products per MAC on the f16 MFMA with
    fp32 accumulation for every contraction of the chain: the six convolutions and the four GDN /
    IGDN channel contractions; |x| ≥ 2^22 does not fit and makes the chain's results NaN, see
    h3_chain_begin), "x6" (bf16x6 split products on the bf16 MFMA everywhere, full fp32 operands),
    "fp32" (exact-f32 MFMA products) or "bf16" (the throughput mode: bf16 activations and weights,
    one bf16 product per MAC, fp32 accumulation — no parity claim). Training: in the h3 mode the
    forward runs the h3 kernels and the backward the x6 ones; the x6 and bf16 modes train on the
    x6 kernels, the fp32 mode on the exact-f32 ones."""
    if _precision not in PRECISIONS:
        raise Iclr17Error(f"iclr17: ICLR17_PRECISION must be one of {PRECISIONS} (got {_precision!r})")
    return _precision


def set_precision(mode: str) -> None:
    global _precision
    if mode not in PRECISIONS:
        raise Iclr17Error(f"iclr17: precision must be one of {PRECISIONS} (got {mode!r})")
    _precision = mode


# A split-form activation is an int16 tensor [3, B, h, w, N]: the bf16 bit patterns of the exact
# parts hi, mid, lo (x = hi + mid + lo) of an NHWC fp32 activation.
def _check_split(s: Tensor, what: str):
    if not isinstance(s, Tensor) or s.dtype != torch.int16 or s.dim() != 5 or s.shape[0] != 3:
        raise Iclr17Error(f"iclr17: {what} must be a split-form int16 tensor [3,B,h,w,N]")
    if not s.is_cuda:
        raise Iclr17Error(f"iclr17: {what} must be a device tensor (there is no CPU path)")
    if not s.is_contiguous():
        raise Iclr17Error(f"iclr17: {what} must be contiguous")


def split_planes(x: Tensor) -> Tensor:
    """fp32 tensor → split form [3, *x.shape] (exact: hi + mid + lo == x)."""
    _check(x, "tensor", x.dim())
    x = x.contiguous()
    out = torch.empty((3,) + tuple(x.shape), device=x.device, dtype=torch.int16)
    call("iclr17_split_planes", _p(x), x.numel(), _p(out), _stream(x))
    return out


def split_packed(packed: Tensor, taps: int, K: int, N: int) -> Tensor:
    """Packed operand [taps][K/4][N][4] fp32 → split planes [3, taps·K·N] int16 (the x6
    B-fragment layout); used for the GDN γ (taps = 1, K = N = C)."""
    _check(packed, "packed operand", packed.dim())
    if packed.numel() != taps * K * N:
        raise Iclr17Error(f"iclr17: split_packed: {packed.numel()} != {taps}*{K}*{N}")
    out = torch.empty(3, taps * K * N, device=packed.device, dtype=torch.int16)
    if _deferred is not None:
        _deferred.append((_PackJob(_lib.ICLR17_PACK_SPLIT, N, taps, K, _ptr(packed), None,
                                   _ptr(out), None, None), (packed, out), None, _stream(packed)))
        return out
    call("iclr17_split_packed", _p(packed), taps, K, N, _p(out), _stream(packed))
    return out


def merge_planes(s: Tensor) -> Tensor:
    """Split form → fp32 (hi + mid + lo, exact); a chunk-major split [3,B,N/32,h,w,32] comes back
    as NHWC. Test/debug helper (torch ops)."""
    if s.dim() == 6:
        s = s.permute(0, 1, 3, 4, 2, 5).reshape(3, s.shape[1], s.shape[3], s.shape[4], -1)
    u = s.to(torch.int32) & 0xFFFF
    parts = (u << 16).view(torch.float32)
    return parts[0] + parts[1] + parts[2]


def conv1_gdn_x6(x: Tensor, wp: Tensor, bias: Tensor, beta_eff: Tensor, gp: Tensor, N: int,
                 want_f32: bool = False, want_pre: bool = False, g6: Optional[Tensor] = None):
    """conv1_gdn with the output in split form (+ fp32 / pre-GDN on request); with g6
    (split_packed of gp) the GDN contraction runs in x6 too."""
    _check(x, "image", 4)
    B, C, H, W = x.shape
    if C != 3:
        raise Iclr17Error(f"iclr17: the analysis transform takes 3-channel images (got {C})")
    _check_image_dims(H, W)
    _check_channels(N)
    x = x.contiguous()
    split = torch.empty(3, B, H // 4, W // 4, N, device=x.device, dtype=torch.int16)
    out = torch.empty(B, H // 4, W // 4, N, device=x.device) if want_f32 else None
    pre = torch.empty(B, H // 4, W // 4, N, device=x.device) if want_pre else None
    call("iclr17_analysis_conv1_gdn_x6", _p(x), B, H, W, N, _p(wp), _p(bias), _p(beta_eff),
         _p(gp), _p(g6), _p(out), _p(split), _p(pre), _stream(x))
    return split, out, pre


def conv1x6_gdn(x: Tensor, w_split: Tensor, bias: Tensor, beta_eff: Tensor, g6: Tensor, N: int,
                want_f32: bool = False, want_pre: bool = False):
    """analysis_17.py:14-17 with both contractions in x6 (w_split: ``pack_conv1_x6``).
    Returns (split, fp32 | None, pre | None) like ``conv1_gdn_x6``."""
    _check(x, "image", 4)
    B, C, H, W = x.shape
    if C != 3:
        raise Iclr17Error(f"iclr17: the analysis transform takes 3-channel images (got {C})")
    _check_image_dims(H, W)
    _check_channels(N)
    if w_split.dtype != torch.int16 or w_split.numel() != 3 * 256 * N:
        raise Iclr17Error("iclr17: conv1x6_gdn needs the split ICLR17_W_CONV1_X6 packing")
    x = x.contiguous()
    split = torch.empty(3, B, H // 4, W // 4, N, device=x.device, dtype=torch.int16)
    out = torch.empty(B, H // 4, W // 4, N, device=x.device) if want_f32 else None
    pre = torch.empty(B, H // 4, W // 4, N, device=x.device) if want_pre else None
    call("iclr17_analysis_conv1x6_gdn", _p(x), B, H, W, N, _p(w_split), _p(bias), _p(beta_eff),
         _p(g6), _p(out), _p(split), _p(pre), _stream(x))
    return split, out, pre


def pack_conv1_x6(w: Tensor, N: int) -> Tensor:
    """conv1 weight [N,3,9,9] → the split planes conv1x6_gdn reads ([3, 256·N] int16)."""
    return split_packed(pack_weight(_lib.ICLR17_W_CONV1_X6, w, N), 1, 256, N)


def conv2_gdn_x6(hs: Tensor, wp: Tensor, bias: Tensor, beta_eff: Tensor, gp: Tensor,
                 g6: Tensor, want_f32: bool = False, want_pre: bool = False):
    """conv2_gdn on a split-form input (g6: split_packed γ); returns (split, fp32 | None,
    pre | None)."""
    _check_split(hs, "activation")
    _, B, h4, w4, N = hs.shape
    _check_channels(N)
    H, W = 4 * h4, 4 * w4
    _check_image_dims(H, W)
    split = torch.empty(3, B, h4 // 2, w4 // 2, N, device=hs.device, dtype=torch.int16)
    out = torch.empty(B, h4 // 2, w4 // 2, N, device=hs.device) if want_f32 else None
    pre = torch.empty(B, h4 // 2, w4 // 2, N, device=hs.device) if want_pre else None
    call("iclr17_analysis_conv2_gdn_x6", _p(hs), B, H, W, N, _p(wp), _p(bias), _p(beta_eff),
         _p(gp), _p(g6), _p(out), _p(split), _p(pre), _stream(hs))
    return split, out, pre


def conv3_quant_rate_x6(hs: Tensor, wp: Tensor, rate_packed: Tensor,
                        noise: Optional[Tensor] = None, want_y: bool = False,
                        rtab: Optional[Tensor] = None, w_split: Optional[Tensor] = None):
    """conv3_quant_rate on a split-form input. Returns (y_hat, bits_partial, y | None,
    y_hat_split). rtab as ``conv3_quant_rate``. w_split (``split_packed(wp, 25, N, N)``, cached by
    ``Analysis_net_17.packed_w3_split``): the weights pre-split, bit-identical results."""
    _check_split(hs, "activation")
    _, B, h8, w8, N = hs.shape
    _check_channels(N)
    H, W = 8 * h8, 8 * w8
    _check_image_dims(H, W)
    mode = _lib.ICLR17_QUANT_ROUND
    if noise is not None:
        _check(noise, "noise", 4)
        if tuple(noise.shape) != (B, N, h8 // 2, w8 // 2):
            raise Iclr17Error(f"iclr17: noise must be {(B, N, h8 // 2, w8 // 2)} (got {tuple(noise.shape)})")
        noise = noise.contiguous()
        mode = _lib.ICLR17_QUANT_NOISE
    y_hat = torch.empty(B, h8 // 2, w8 // 2, N, device=hs.device, dtype=torch.float32)
    y_hat_split = torch.empty(3, B, h8 // 2, w8 // 2, N, device=hs.device, dtype=torch.int16)
    y = torch.empty_like(y_hat) if want_y else None
    T = query("iclr17_conv3_x6_partials_per_image", B, H, W, N, mode)
    partial = torch.empty(B, T, device=hs.device, dtype=torch.float64)
    if w_split is not None:
        call("iclr17_analysis_conv3_quant_rate_x6w", _p(hs), B, H, W, N, _p(wp), _p(w_split), mode,
             _p(noise), _p(rate_packed), _p(rtab), _p(y), _p(y_hat), _p(y_hat_split), _p(partial),
             _stream(hs))
    else:
        call("iclr17_analysis_conv3_quant_rate_x6", _p(hs), B, H, W, N, _p(wp), mode, _p(noise),
             _p(rate_packed), _p(rtab), _p(y), _p(y_hat), _p(y_hat_split), _p(partial), _stream(hs))
    return y_hat, partial, y, y_hat_split


def deconv_igdn_x6(hs: Tensor, wp: Tensor, bias: Tensor, beta_eff: Tensor, gp: Tensor,
                   g6: Tensor, want_split: bool = True, want_f32: bool = False,
                   want_pre: bool = False, chunk_major: bool = False):
    """deconv_igdn on a split-form input; returns (split | None, fp32 | None, pre | None). With
    ``chunk_major`` the split output is [3, B, N/32, 2h, 2w, 32] — the input form of
    ``deconv3_x6`` that keeps its 32-channel chunks on separate cache lines."""
    _check_split(hs, "activation")
    _, B, hh, ww, N = hs.shape
    _check_channels(N)
    if not (want_split or want_f32):
        raise Iclr17Error("iclr17: deconv_igdn_x6 needs an output")
    shape = (3, B, N // 32, 2 * hh, 2 * ww, 32) if chunk_major else (3, B, 2 * hh, 2 * ww, N)
    split = torch.empty(shape, device=hs.device, dtype=torch.int16) if want_split else None
    out = torch.empty(B, 2 * hh, 2 * ww, N, device=hs.device) if want_f32 else None
    pre = torch.empty(B, 2 * hh, 2 * ww, N, device=hs.device) if want_pre else None
    call("iclr17_synthesis_deconv_igdn_x6_cm" if chunk_major else "iclr17_synthesis_deconv_igdn_x6",
         _p(hs), B, hh, ww, N, _p(wp), _p(bias), _p(beta_eff),
         _p(gp), _p(g6), _p(out), _p(split), _p(pre), _stream(hs))
    return split, out, pre


# ------------------------------------------------------------------ h3 form (csrc/engine_h3.hip)
# An h3 activation is an int16 tensor [2, B, h, w, N] (or chunk-major [2, B, N/32, h, w, 32]): the
# fp16 bit patterns of hi = rne16(x·2^-6) and lo = rne16((x·2^-6 − hi)·2^11) (common.h "h3 form").
H3_SIGMA_A = 2.0 ** -6
_range_flags = {}
H3_RANGE_MESSAGE = ("iclr17: an activation of magnitude >= 2^22 does not fit the h3 form (the "
                    "chain's results are NaN); run this input with kernels.set_precision('x6')")


def h3_range_flag(device) -> Tensor:
    """The h3 range flag of the current stream on ``device`` (int32, 0 = every value of the
    current chain fitted the h3 form). One flag per (device, stream), so chains running
    concurrently on side streams (ImageCompressor.evaluate_many) do not clear each other's."""
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    f = _range_flags.get(key)
    if f is None:
        f = torch.zeros(1, device=dev, dtype=torch.int32)
        _range_flags[key] = f
    return f


def h3_chain_begin(device) -> None:
    """Clear the current stream's h3 range flag at the start of a chain of h3 kernels (one fill
    on the stream; no synchronisation). Every producer sets the flag when a value does not fit;
    the chain's last kernel (deconv3_h3) reads it and writes NaN results when it is set."""
    h3_range_flag(device).zero_()


def h3_range_overflowed(device) -> bool:
    """Whether the current stream's last h3 chain met a value of magnitude ≥ 2^22.
    Synchronises with the device."""
    return int(h3_range_flag(device).item()) != 0


def check_h3_range(device) -> None:
    """Raise Iclr17Error when the current stream's last h3 chain met a value of magnitude
    ≥ 2^22, which the h3 form cannot hold. Synchronises with the device."""
    if h3_range_overflowed(device):
        raise Iclr17Error(H3_RANGE_MESSAGE)


def check_finite(what: str, *values) -> None:
    """For callers that read results anyway (the training driver's log, testKodak, bench): raise
    Iclr17Error when a result is not finite — in the h3 mode the mark of an activation that did
    not fit the form (the chain's last kernel writes NaN then), or of a non-finite input."""
    for v in values:
        t = torch.as_tensor(v)
        if not bool(torch.isfinite(t).all()):
            if precision() == "h3":
                raise Iclr17Error(f"{H3_RANGE_MESSAGE} [{what}]")
            raise Iclr17Error(f"iclr17: non-finite {what}")


# The h3 layers read their input chunk-major: [2, B, N/cm, h, w, cm] with cm the chunk the layer
# stages (conv2 / conv3: 8; deconv1 / deconv2: 16; deconv3: 32), so that a patch piece is 16
# contiguous bytes; each layer writes the layout its consumer reads (out_cm).
CONV_CM, DECONV_CM, DECONV3_CM = 8, 16, 32


def _check_h3(s: Tensor, what: str, cm: int):
    """An h3 activation in the chunk-major layout cm; returns (B, h, w, N)."""
    if (not isinstance(s, Tensor) or s.dtype != torch.int16 or s.dim() != 6 or s.shape[0] != 2
            or s.shape[5] != cm):
        raise Iclr17Error(f"iclr17: {what} must be an h3-form int16 tensor in the chunk-major layout "
                          f"[2,B,N/{cm},h,w,{cm}] (kernels.h3_planes(x, cm={cm}))")
    if not s.is_cuda:
        raise Iclr17Error(f"iclr17: {what} must be a device tensor (there is no CPU path)")
    if not s.is_contiguous():
        raise Iclr17Error(f"iclr17: {what} must be contiguous")
    return s.shape[1], s.shape[3], s.shape[4], s.shape[2] * cm


def _h3_out(B: int, h: int, w: int, N: int, cm: int, device) -> Tensor:
    if cm not in (0, 8, 16, 32) or (cm and N % cm):
        raise Iclr17Error(f"iclr17: h3 output layout must be 0 (NHWC), 8, 16 or 32 (got {cm})")
    shape = (2, B, N // cm, h, w, cm) if cm else (2, B, h, w, N)
    return torch.empty(shape, device=device, dtype=torch.int16)


def h3_planes(x: Tensor, cm: int = 0) -> Tensor:
    """fp32 tensor (numel % 4 == 0) → h3 form [2, *x.shape]; with ``cm`` (8, 16, 32) an NHWC
    [B, h, w, N] tensor → the chunk-major [2, B, N/cm, h, w, cm] the h3 layers read."""
    _check(x, "tensor", x.dim())
    x = x.contiguous()
    if x.numel() % 4:
        raise Iclr17Error("iclr17: h3_planes needs a multiple of 4 elements")
    if cm:
        if x.dim() != 4:
            raise Iclr17Error("iclr17: h3_planes(cm=...) takes an NHWC [B,h,w,N] tensor")
        B, h, w, N = x.shape
        out = _h3_out(B, h, w, N, cm, x.device)
        call("iclr17_h3_planes_cm", _p(x), B, h, w, N, cm, _p(out), _p(h3_range_flag(x.device)),
             _stream(x))
        return out
    out = torch.empty((2,) + tuple(x.shape), device=x.device, dtype=torch.int16)
    call("iclr17_h3_planes", _p(x), x.numel(), _p(out), _p(h3_range_flag(x.device)), _stream(x))
    return out


def merge_h3(s: Tensor) -> Tensor:
    """h3 form → fp32 (hi + lo·2^-11)/σ_a; a chunk-major [2,B,N/cm,h,w,cm] comes back as NHWC.
    Test/debug helper (torch ops, exact in fp32)."""
    if s.dim() == 6:
        s = s.permute(0, 1, 3, 4, 2, 5).reshape(2, s.shape[1], s.shape[3], s.shape[4], -1)
    h = s.view(torch.float16).to(torch.float32)
    return (h[0] + h[1] * (2.0 ** -11)) / H3_SIGMA_A


_deferred_h3: Optional[list] = None   # queued h3 pack jobs inside batched_h3_packs()


@contextlib.contextmanager
def batched_h3_packs():
    """Inside the block, pack_h3k / split_packed_h3 allocate their outputs and queue the work; on
    exit it runs as iclr17_pack_h3_batch (two launches instead of two per pack). Nothing may read
    the outputs inside the block. Re-entrant."""
    global _deferred_h3
    if _deferred_h3 is not None:
        yield
        return
    _deferred_h3 = []
    try:
        yield
        jobs = _deferred_h3
    finally:
        _deferred_h3 = None
    for i in range(0, len(jobs), _lib.ICLR17_PACK_H3_MAXJ):
        part = jobs[i:i + _lib.ICLR17_PACK_H3_MAXJ]
        arr = (_PackJob * len(part))(*[j[0] for j in part])
        call("iclr17_pack_h3_batch", ctypes.cast(arr, ctypes.c_void_p), len(part), part[0][2])
    del jobs   # sources stay alive until here; the stream orders their reuse after the launches


def pack_h3k(which: int, w: Tensor, N: int) -> Tensor:
    """conv / deconv weights → the h3 engine's two fp16 planes (per-tensor power-of-two scale) +
    trailer (ICLR17_H3K_CONV1 / ICLR17_H3K_CONV5 / ICLR17_H3K_DECONV5)."""
    _check(w, "weight", 4)
    size = query("iclr17_h3k_weight_size", which, N)
    if size == 0:
        raise Iclr17Error(f"iclr17: pack_h3k: kind {which}, N={N} unsupported")
    out = torch.empty(size, device=w.device, dtype=torch.int16)
    w = w.detach().contiguous()
    if _deferred_h3 is not None:
        _deferred_h3.append((_PackJob(_lib.ICLR17_PACK_H3K, N, 0, which, _ptr(w), None, _ptr(out),
                                      None, None), (w, out), _stream(w)))
        return out
    call("iclr17_pack_h3k", which, _p(w), _p(out), N, _stream(w))
    return out


def split_packed_h3(packed: Tensor, taps: int, K: int, N: int) -> Tensor:
    """Packed operand [taps][K/4][N][4] fp32 → the h3 engine's two fp16 planes + trailer (int16,
    ``iclr17_split_packed_h3_size`` elements): conv2 / conv3 weights of the h3 form."""
    _check(packed, "packed operand", packed.dim())
    if packed.numel() != taps * K * N:
        raise Iclr17Error(f"iclr17: split_packed_h3: {packed.numel()} != {taps}*{K}*{N}")
    size = query("iclr17_split_packed_h3_size", taps, K, N)
    if size == 0:
        raise Iclr17Error("iclr17: split_packed_h3: bad shape")
    out = torch.empty(size, device=packed.device, dtype=torch.int16)
    packed = packed.contiguous()
    if _deferred_h3 is not None:
        _deferred_h3.append((_PackJob(_lib.ICLR17_PACK_SPLIT_H3, N, taps, K, _ptr(packed), None,
                                      _ptr(out), None, None), (packed, out), _stream(packed)))
        return out
    call("iclr17_split_packed_h3", _p(packed), taps, K, N, _p(out), _stream(packed))
    return out


def pack_conv1_h3(w: Tensor, N: int) -> Tensor:
    """conv1 weight [N,3,9,9] → the h3 engine's conv1 packing (pack_h3k, ICLR17_H3K_CONV1)."""
    return pack_h3k(_lib.ICLR17_H3K_CONV1, w, N)


def conv1_gdn_h3(x: Tensor, w_h3: Tensor, bias: Tensor, beta_eff: Tensor, gh3: Tensor, N: int,
                 want_f32: bool = False, want_h3: bool = True, want_x6: bool = False,
                 want_pre: bool = False, out_cm: int = CONV_CM):
    """analysis_17.py:14-17 conv1 + GDN1 in the h3 form on the h3 engine (three f16 part products
    per MAC for the convolution and the GDN contraction; w_h3: ``pack_conv1_h3``, gh3:
    GDN.effective_params_h3's γ). Returns (h3 | None — chunk-major [2,B,N/out_cm,H/4,W/4,out_cm],
    conv2's input —, fp32 | None), and with ``want_x6`` / ``want_pre`` (training) also (x6 split |
    None, GDN1 input conv1 + bias | None)."""
    _check(x, "image", 4)
    B, C, H, W = x.shape
    if C != 3:
        raise Iclr17Error(f"iclr17: the analysis transform takes 3-channel images (got {C})")
    _check_image_dims(H, W)
    _check_channels(N)
    if w_h3.dtype != torch.int16 or w_h3.numel() != query("iclr17_h3k_weight_size", _lib.ICLR17_H3K_CONV1, N):
        raise Iclr17Error("iclr17: conv1_gdn_h3 needs pack_conv1_h3 weights")
    if gh3.dtype != torch.int16 or gh3.numel() != query("iclr17_split_packed_h3_size", 1, N, N):
        raise Iclr17Error("iclr17: conv1_gdn_h3 needs γ in the h3 form (effective_params_h3)")
    if not (want_h3 or want_f32 or want_x6):
        raise Iclr17Error("iclr17: conv1_gdn_h3 needs an output")
    x = x.contiguous()
    h3 = _h3_out(B, H // 4, W // 4, N, out_cm, x.device) if want_h3 else None
    x6 = torch.empty(3, B, H // 4, W // 4, N, device=x.device, dtype=torch.int16) if want_x6 else None
    out = torch.empty(B, H // 4, W // 4, N, device=x.device) if want_f32 else None
    pre = torch.empty(B, H // 4, W // 4, N, device=x.device) if want_pre else None
    call("iclr17_analysis_conv1_gdn_h3", _p(x), B, H, W, N, _p(w_h3), _p(bias), _p(beta_eff),
         _p(gh3), _p(out), _p(pre), _p(h3), out_cm, _p(x6), _p(h3_range_flag(x.device)), _stream(x))
    if want_x6 or want_pre:
        return h3, out, x6, pre
    return h3, out


def conv2_gdn_h3(hs: Tensor, wk: Tensor, bias: Tensor, beta_eff: Tensor, gh3: Tensor,
                 want_h3: bool = True, want_f32: bool = False, want_x6: bool = False,
                 want_pre: bool = False, out_cm: int = CONV_CM):
    """analysis_17.py:18-21 conv2 + GDN2 in the h3 form on the h3 engine (csrc/engine_h3.hip):
    h3 input chunk-major 8 [2,B,N/8,H/4,W/4,8] → (h3 | None — layout out_cm, conv3's input —,
    fp32 | None, x6 split | None). wk:
    ``pack_h3k(ICLR17_H3K_CONV5, w)``; gh3: GDN.effective_params_h3's γ. With ``want_pre``
    (training) a fourth result: GDN2's input conv2 + bias (fp32 NHWC)."""
    B, h4, w4, N = _check_h3(hs, "activation", CONV_CM)
    _check_channels(N)
    H, W = 4 * h4, 4 * w4
    _check_image_dims(H, W)
    if wk.numel() != query("iclr17_h3k_weight_size", _lib.ICLR17_H3K_CONV5, N):
        raise Iclr17Error("iclr17: conv2_gdn_h3 needs pack_h3k(ICLR17_H3K_CONV5) weights")
    if gh3.dtype != torch.int16 or gh3.numel() != query("iclr17_split_packed_h3_size", 1, N, N):
        raise Iclr17Error("iclr17: conv2_gdn_h3 needs γ in the h3 form (effective_params_h3)")
    if not (want_h3 or want_f32 or want_x6):
        raise Iclr17Error("iclr17: conv2_gdn_h3 needs an output")
    h3 = _h3_out(B, h4 // 2, w4 // 2, N, out_cm, hs.device) if want_h3 else None
    x6 = torch.empty(3, B, h4 // 2, w4 // 2, N, device=hs.device, dtype=torch.int16) if want_x6 else None
    out = torch.empty(B, h4 // 2, w4 // 2, N, device=hs.device) if want_f32 else None
    pre = torch.empty(B, h4 // 2, w4 // 2, N, device=hs.device) if want_pre else None
    call("iclr17_analysis_conv2_gdn_h3", _p(hs), B, H, W, N, _p(wk), _p(bias), _p(beta_eff), _p(gh3),
         _p(out), _p(pre), _p(h3), out_cm, _p(x6), _p(h3_range_flag(hs.device)), _stream(hs))
    if want_pre:
        return h3, out, x6, pre
    return h3, out, x6


def conv3_quant_rate_h3(hs: Tensor, wh: Tensor, rate_packed: Tensor,
                        noise: Optional[Tensor] = None, want_y: bool = False,
                        rtab: Optional[Tensor] = None, want_h3: bool = True,
                        out_cm: int = DECONV_CM):
    """analysis_17.py:22 + model.py:48-56,71-73 in the h3 form on the h3 engine (wh:
    ``pack_h3k(ICLR17_H3K_CONV5, conv3.weight)``), input chunk-major 8. Returns (y_hat NHWC,
    bits_partial [B, iclr17_conv3_h3_partials_per_image], y | None, y_hat h3 | None — layout
    out_cm, deconv1's input)."""
    B, h8, w8, N = _check_h3(hs, "activation", CONV_CM)
    _check_channels(N)
    H, W = 8 * h8, 8 * w8
    _check_image_dims(H, W)
    if wh.dtype != torch.int16 or wh.numel() != query("iclr17_h3k_weight_size", _lib.ICLR17_H3K_CONV5, N):
        raise Iclr17Error("iclr17: conv3_quant_rate_h3 needs pack_h3k(ICLR17_H3K_CONV5) weights")
    mode = _lib.ICLR17_QUANT_ROUND
    if noise is not None:
        _check(noise, "noise", 4)
        if tuple(noise.shape) != (B, N, h8 // 2, w8 // 2):
            raise Iclr17Error(f"iclr17: noise must be {(B, N, h8 // 2, w8 // 2)} (got {tuple(noise.shape)})")
        noise = noise.contiguous()
        mode = _lib.ICLR17_QUANT_NOISE
    y_hat = torch.empty(B, h8 // 2, w8 // 2, N, device=hs.device, dtype=torch.float32)
    y_hat_h3 = _h3_out(B, h8 // 2, w8 // 2, N, out_cm, hs.device) if want_h3 else None
    y = torch.empty_like(y_hat) if want_y else None
    T = query("iclr17_conv3_h3_partials_per_image", B, H, W, N, mode)
    partial = torch.empty(B, T, device=hs.device, dtype=torch.float64)
    call("iclr17_analysis_conv3_quant_rate_h3", _p(hs), B, H, W, N, _p(wh), mode, _p(noise),
         _p(rate_packed), _p(rtab), _p(y), _p(y_hat), _p(y_hat_h3), out_cm, _p(partial),
         _p(h3_range_flag(hs.device)), _stream(hs))
    return y_hat, partial, y, y_hat_h3


def deconv_igdn_h3(hs: Tensor, wh: Tensor, bias: Tensor, beta_eff: Tensor, gh3: Tensor,
                   want_h3: bool = True, want_f32: bool = False, want_x6: bool = False,
                   chunk_major: bool = False, int_in: bool = False, want_pre: bool = False,
                   out_cm: Optional[int] = None):
    """synthesis_17.py:15-22 in the h3 form (csrc/engine_h3.hip): h3 input chunk-major 16
    [2,B,N/16,h,w,16] → (h3 | None, fp32 | None, x6 split | None). wh: ``pack_h3k(ICLR17_H3K_DECONV5,
    …)``; gh3: the IGDN's γ in the h3 form (GDN.effective_params_h3). ``int_in``: the input is ŷ
    (a workgroup whose window has a zero lo plane skips the lo products; same result). The h3
    output's layout: ``out_cm`` (default 16, deconv2's input), or 32 with ``chunk_major`` (deconv3's
    input); the x6 output is NHWC. With ``want_pre`` (training) a fourth result: the IGDN input
    deconv + bias (fp32 NHWC)."""
    B, hh, ww, N = _check_h3(hs, "activation", DECONV_CM)
    if out_cm is None:
        out_cm = DECONV3_CM if chunk_major else DECONV_CM
    _check_channels(N)
    if gh3.dtype != torch.int16 or gh3.numel() != query("iclr17_split_packed_h3_size", 1, N, N):
        raise Iclr17Error("iclr17: deconv_igdn_h3 needs the IGDN's h3 γ (split_packed_h3, taps 1)")
    if not (want_h3 or want_f32 or want_x6):
        raise Iclr17Error("iclr17: deconv_igdn_h3 needs an output")
    if wh.numel() != query("iclr17_h3k_weight_size", _lib.ICLR17_H3K_DECONV5, N):
        raise Iclr17Error("iclr17: deconv_igdn_h3 needs the ICLR17_H3K_DECONV5 packing")
    h3 = _h3_out(B, 2 * hh, 2 * ww, N, out_cm, hs.device) if want_h3 else None
    x6 = torch.empty(3, B, 2 * hh, 2 * ww, N, device=hs.device, dtype=torch.int16) if want_x6 else None
    out = torch.empty(B, 2 * hh, 2 * ww, N, device=hs.device) if want_f32 else None
    pre = torch.empty(B, 2 * hh, 2 * ww, N, device=hs.device) if want_pre else None
    call("iclr17_synthesis_deconv_igdn_h3", _p(hs), B, hh, ww, N, _p(wh), _p(bias),
         _p(beta_eff), _p(gh3), _p(out), _p(pre), _p(h3), _p(x6), out_cm, int(int_in),
         _p(h3_range_flag(hs.device)), _stream(hs))
    if want_pre:
        return h3, out, x6, pre
    return h3, out, x6


def ms_ssim(x: Tensor, y: Tensor, data_range: float = 1.0) -> Tensor:
    """Per-image MS-SSIM [B] of NCHW fp32 image batches (models/ms_ssim_torch.py:123-196 as
    train.py:178 calls it), on the GPU."""
    _check(x, "image", 4)
    _check(y, "image", 4)
    if x.shape != y.shape or x.shape[1] != 3:
        raise Iclr17Error(f"iclr17: ms_ssim needs two [B,3,H,W] batches of one shape "
                          f"(got {tuple(x.shape)} and {tuple(y.shape)})")
    B, _, H, W = x.shape
    nbytes = query("iclr17_ms_ssim_workspace_size", B, H, W)
    if nbytes == 0:
        raise Iclr17Error(f"iclr17: ms_ssim: {H}x{W} is too small for 5 levels of an 11-tap window")
    ws = torch.empty(nbytes, device=x.device, dtype=torch.uint8)
    out = torch.empty(B, device=x.device, dtype=torch.float32)
    call("iclr17_ms_ssim", _p(x.contiguous()), _p(y.contiguous()), B, H, W, float(data_range),
         _p(ws), nbytes, _p(out), _stream(x))
    return out


def ssim(x: Tensor, y: Tensor, data_range: float = 1.0):
    """Per-image single-scale SSIM and cs means ([B], [B]) of NCHW fp32 batches
    (models/ms_ssim_torch.py:36-83 with size_average=False, full=True), on the GPU."""
    _check(x, "image", 4)
    _check(y, "image", 4)
    if x.shape != y.shape or x.shape[1] != 3:
        raise Iclr17Error(f"iclr17: ssim needs two [B,3,H,W] batches of one shape "
                          f"(got {tuple(x.shape)} and {tuple(y.shape)})")
    B, _, H, W = x.shape
    nbytes = query("iclr17_ssim_workspace_size", B, H, W)
    if nbytes == 0:
        raise Iclr17Error(f"iclr17: ssim: {H}x{W} is smaller than the 11-tap window")
    ws = torch.empty(nbytes, device=x.device, dtype=torch.uint8)
    s = torch.empty(B, device=x.device, dtype=torch.float32)
    cs = torch.empty(B, device=x.device, dtype=torch.float32)
    call("iclr17_ssim", _p(x.contiguous()), _p(y.contiguous()), B, H, W, float(data_range),
         _p(ws), nbytes, _p(s), _p(cs), _stream(x))
    return s, cs


def output_partials_per_image(H: int, W: int) -> int:
    return query("iclr17_output_partials_per_image", H, W)


def deconv3(h: Tensor, wp: Tensor, bias: Tensor, x_ref: Optional[Tensor] = None,
            want_recon: bool = False, sse_unclipped: bool = False):
    """synthesis_17.py:23-25 + model.py:59: NHWC [B,H/4,W/4,N] → clipped NCHW [B,3,H,W].

    Returns (clipped, recon_unclipped | None, sse_partial [B,T] | None)."""
    _check(h, "activation", 4)
    B, h4, w4, N = h.shape
    _check_channels(N)
    H, W = 4 * h4, 4 * w4
    _check_image_dims(H, W)
    clipped = torch.empty(B, 3, H, W, device=h.device, dtype=torch.float32)
    recon = torch.empty_like(clipped) if want_recon else None
    partial = None
    if x_ref is not None:
        _check(x_ref, "reference image", 4)
        if tuple(x_ref.shape) != (B, 3, H, W):
            raise Iclr17Error("iclr17: reference image shape mismatch")
        x_ref = x_ref.contiguous()
        partial = torch.empty(B, output_partials_per_image(H, W), device=h.device, dtype=torch.float64)
    call("iclr17_synthesis_deconv3", _p(h.contiguous()), B, H, W, N, _p(wp), _p(bias), _p(x_ref),
         _p(clipped), _p(recon), _p(partial), int(sse_unclipped), _stream(h))
    return clipped, recon, partial


def split_deconv3(wp: Tensor, N: int) -> Tensor:
    """The ICLR17_W_DECONV9 packing of deconv3 split into the x6 weight planes
    [3][9][N/8][48][8] that ``deconv3_x6`` reads (iclr17_split_packed, taps 9, K N, N 48)."""
    return split_packed(wp, 9, N, 48)


def deconv3_x6(hs: Tensor, w_split: Tensor, bias: Tensor, x_ref: Optional[Tensor] = None,
               want_recon: bool = False, sse_unclipped: bool = False,
               bits: Optional[Tuple[Tensor, float]] = None):
    """deconv3 on a split-form input — [3,B,H/4,W/4,N], or the chunk-major [3,B,N/32,H/4,W/4,32]
    of ``deconv_igdn_x6(chunk_major=True)`` — (the halo-tiled x6 kernel); w_split:
    ``split_deconv3`` of the packed weights (Synthesis_net_17.packed_x6). The same returns as
    ``deconv3`` (bit-identical in either input form). ``bits`` = (conv3's bit partials [B, T],
    scale), chunk-major input only: the kernel also performs ``reduce_partials(partial, scale,
    per_image=False)`` (bit-identical) and a fourth value, the 0-dim total, is returned."""
    cm = isinstance(hs, Tensor) and hs.dim() == 6
    if cm:
        if hs.dtype != torch.int16 or hs.shape[0] != 3 or hs.shape[5] != 32 or not hs.is_cuda \
                or not hs.is_contiguous():
            raise Iclr17Error("iclr17: a chunk-major split activation is a contiguous device int16 "
                              "tensor [3,B,N/32,h,w,32]")
        _, B, nch, h4, w4, _ = hs.shape
        N = 32 * nch
    else:
        _check_split(hs, "activation")
        _, B, h4, w4, N = hs.shape
    if (not isinstance(w_split, Tensor) or w_split.dtype != torch.int16
            or w_split.numel() != 3 * 9 * N * 48):
        raise Iclr17Error("iclr17: deconv3_x6 takes the split weight planes (split_deconv3)")
    if bits is not None and not cm:
        raise Iclr17Error("iclr17: deconv3_x6 folds the bit reduction only on the chunk-major input")
    return _deconv3_halo("iclr17_synthesis_deconv3_x6_cm" if cm else "iclr17_synthesis_deconv3_x6",
                         hs, B, h4, w4, N, w_split, bias, x_ref, want_recon, sse_unclipped, bits)


def deconv3_h3(hs: Tensor, w_h3: Tensor, bias: Tensor, x_ref: Optional[Tensor] = None,
               want_recon: bool = False, sse_unclipped: bool = False,
               bits: Optional[Tuple[Tensor, float]] = None, bits_per_image: bool = False):
    """deconv3 on the chunk-major h3 input [2,B,N/32,H/4,W/4,32] of ``deconv_igdn_h3(chunk_major
    =True)`` (the halo-tiled kernel, three fp16 part products per MAC); w_h3: ``split_packed_h3``
    of the ICLR17_W_DECONV9 packing (Synthesis_net_17.packed_h3). Returns as ``deconv3_x6``; with
    ``bits`` and ``bits_per_image`` a fifth value, the per-image bit sums (float64 [B], those of
    ``reduce_partials``). The chain's h3 range flag (h3_range_flag) is passed: when an upstream
    h3 kernel met |x| ≥ 2^22 every output is NaN."""
    if (not isinstance(hs, Tensor) or hs.dim() != 6 or hs.dtype != torch.int16 or hs.shape[0] != 2
            or hs.shape[5] != 32 or not hs.is_cuda or not hs.is_contiguous()):
        raise Iclr17Error("iclr17: deconv3_h3 takes a contiguous chunk-major h3 activation "
                          "[2,B,N/32,h,w,32]")
    _, B, nch, h4, w4, _ = hs.shape
    N = 32 * nch
    if (not isinstance(w_h3, Tensor) or w_h3.dtype != torch.int16
            or w_h3.numel() != query("iclr17_split_packed_h3_size", 9, N, 48)):
        raise Iclr17Error("iclr17: deconv3_h3 takes split_packed_h3 of the deconv3 packing")
    _check_channels(N)
    H, W = 4 * h4, 4 * w4
    _check_image_dims(H, W)
    clipped = torch.empty(B, 3, H, W, device=hs.device, dtype=torch.float32)
    recon = torch.empty_like(clipped) if want_recon else None
    partial = None
    if x_ref is not None:
        _check(x_ref, "reference image", 4)
        if tuple(x_ref.shape) != (B, 3, H, W):
            raise Iclr17Error("iclr17: reference image shape mismatch")
        x_ref = x_ref.contiguous()
        partial = torch.empty(B, output_partials_per_image(H, W), device=hs.device, dtype=torch.float64)
    bp, scale, total, per = None, 0.0, None, None
    if bits is not None:
        bp, scale = bits
        _check_f64(bp)
        if bp.shape[0] != B:
            raise Iclr17Error("iclr17: bit partials are not [B, T]")
        bp = bp.contiguous()
        total = torch.empty((), device=hs.device, dtype=torch.float32)
        if bits_per_image:
            per = torch.empty(B, device=hs.device, dtype=torch.float64)
    call("iclr17_synthesis_deconv3_h3", _p(hs), B, H, W, N, _p(w_h3), _p(bias), _p(x_ref),
         _p(clipped), _p(recon), _p(partial), int(sse_unclipped), _p(bp),
         bp.shape[1] if bp is not None else 0, _p(per), _p(total), ctypes.c_double(scale),
         _p(h3_range_flag(hs.device)), _stream(hs))
    if bits is None:
        return clipped, recon, partial
    return (clipped, recon, partial, total, per) if bits_per_image else (clipped, recon, partial, total)


def _deconv3_halo(fn, hs, B, h4, w4, N, wp, bias, x_ref, want_recon, sse_unclipped, bits=None):
    _check_channels(N)
    H, W = 4 * h4, 4 * w4
    _check_image_dims(H, W)
    clipped = torch.empty(B, 3, H, W, device=hs.device, dtype=torch.float32)
    recon = torch.empty_like(clipped) if want_recon else None
    partial = None
    if x_ref is not None:
        _check(x_ref, "reference image", 4)
        if tuple(x_ref.shape) != (B, 3, H, W):
            raise Iclr17Error("iclr17: reference image shape mismatch")
        x_ref = x_ref.contiguous()
        partial = torch.empty(B, output_partials_per_image(H, W), device=hs.device, dtype=torch.float64)
    if bits is None:
        call(fn, _p(hs), B, H, W, N, _p(wp), _p(bias), _p(x_ref), _p(clipped), _p(recon),
             _p(partial), int(sse_unclipped), _stream(hs))
        return clipped, recon, partial
    bp, scale = bits
    _check_f64(bp)
    if bp.shape[0] != B:
        raise Iclr17Error("iclr17: bit partials are not [B, T]")
    total = torch.empty((), device=hs.device, dtype=torch.float32)
    call(fn + "_bits", _p(hs), B, H, W, N, _p(wp), _p(bias), _p(x_ref), _p(clipped), _p(recon),
         _p(partial), int(sse_unclipped), _p(bp.contiguous()), bp.shape[1], None, _p(total),
         ctypes.c_double(scale), _stream(hs))
    return clipped, recon, partial, total


# ------------------------------------------------------------ bf16 throughput precision mode
# A bf16 activation is an int16 tensor [B, h, w, N] holding the bf16 bit patterns (round to
# nearest even) of an NHWC activation; the bf16 kernels (csrc/engine_bf16.hip) read and write it.
def _check_bf16(t: Tensor, what: str):
    if not isinstance(t, Tensor) or t.dtype != torch.int16 or t.dim() != 4:
        raise Iclr17Error(f"iclr17: {what} must be a bf16-pattern int16 NHWC tensor [B,h,w,N]")
    if not t.is_cuda:
        raise Iclr17Error(f"iclr17: {what} must be a device tensor (there is no CPU path)")
    if not t.is_contiguous():
        raise Iclr17Error(f"iclr17: {what} must be contiguous")


def to_bf16(x: Tensor) -> Tensor:
    """fp32 → bf16 bit patterns (int16, same shape), round to nearest even."""
    _check(x, "tensor", x.dim())
    x = x.contiguous()
    out = torch.empty(x.shape, device=x.device, dtype=torch.int16)
    if x.numel() % 8:
        raise Iclr17Error("iclr17: to_bf16 needs a multiple of 8 elements")
    call("iclr17_to_bf16", _p(x), x.numel(), _p(out), _stream(x))
    return out


def from_bf16(t: Tensor) -> Tensor:
    """bf16 bit patterns (int16) → fp32 (exact; torch ops, a test/debug helper)."""
    return ((t.to(torch.int32) & 0xFFFF) << 16).view(torch.float32)


def pack_bf16(which: int, w: Tensor, N: int) -> Tensor:
    """k5 weights → the bf16 engine's step layout (ICLR17_BF_CONV5 / ICLR17_BF_DECONV5)."""
    _check(w, "weight", 4)
    size = query("iclr17_bf16_weight_size", which, N)
    if size == 0:
        raise Iclr17Error(f"iclr17: pack_bf16: kind {which}, N={N} unsupported")
    out = torch.empty(size, device=w.device, dtype=torch.int16)
    call("iclr17_pack_bf16", which, _p(w.detach().contiguous()), _p(out), N, _stream(w))
    return out


def round_packed(packed: Tensor, taps: int, K: int, N: int) -> Tensor:
    """Packed fp32 [taps][K/4][N][4] → bf16 fragments [taps][K/8][N][8] (round to nearest even)."""
    _check(packed, "packed operand", packed.dim())
    if packed.numel() != taps * K * N:
        raise Iclr17Error(f"iclr17: round_packed: {packed.numel()} != {taps}*{K}*{N}")
    out = torch.empty(taps * K * N, device=packed.device, dtype=torch.int16)
    call("iclr17_round_packed", _p(packed), taps, K, N, _p(out), _stream(packed))
    return out


def conv1_gdn_bf16(x: Tensor, w_bf: Tensor, bias: Tensor, beta_eff: Tensor, g_bf: Tensor,
                   N: int) -> Tensor:
    """analysis_17.py:14-17 in bf16: x NCHW fp32 → bf16 NHWC [B,H/4,W/4,N]. w_bf: round_packed
    of the ICLR17_W_CONV1_X6 packing (1, 256, N); g_bf: round_packed of γ's gp (1, N, N)."""
    _check(x, "image", 4)
    B, C, H, W = x.shape
    if C != 3:
        raise Iclr17Error(f"iclr17: the analysis transform takes 3-channel images (got {C})")
    _check_image_dims(H, W)
    _check_channels(N)
    out = torch.empty(B, H // 4, W // 4, N, device=x.device, dtype=torch.int16)
    call("iclr17_analysis_conv1_gdn_bf16", _p(x.contiguous()), B, H, W, N, _p(w_bf), _p(bias),
         _p(beta_eff), _p(g_bf), _p(out), _stream(x))
    return out


def conv2_gdn_bf16(h: Tensor, w_bf: Tensor, bias: Tensor, beta_eff: Tensor, g_bf: Tensor) -> Tensor:
    """analysis_17.py:18-21 in bf16: bf16 NHWC [B,H/4,W/4,N] → [B,H/8,W/8,N]."""
    _check_bf16(h, "activation")
    B, h4, w4, N = h.shape
    _check_channels(N)
    H, W = 4 * h4, 4 * w4
    _check_image_dims(H, W)
    out = torch.empty(B, h4 // 2, w4 // 2, N, device=h.device, dtype=torch.int16)
    call("iclr17_analysis_conv2_gdn_bf16", _p(h), B, H, W, N, _p(w_bf), _p(bias), _p(beta_eff),
         _p(g_bf), _p(out), _stream(h))
    return out


def rate_table(rate_packed: Tensor, N: int) -> Tensor:
    """element_bits(v, c) for the integer latents v ∈ [−32, 32]: float32 [N, 65]."""
    _check(rate_packed, "rate table")
    if rate_packed.numel() != 11 * N:
        raise Iclr17Error(f"iclr17: rate_table: packed rate parameters are not [11][{N}]")
    out = torch.empty(N, 65, device=rate_packed.device, dtype=torch.float32)
    call("iclr17_rate_table", _p(rate_packed), N, _p(out), _stream(rate_packed))
    return out


def conv3_quant_rate_bf16(h: Tensor, w_bf: Tensor, rate_packed: Tensor, rtab: Optional[Tensor] = None,
                          want_y: bool = False):
    """analysis_17.py:22 + model.py:56,71-73 (round mode) in bf16 → (ŷ fp32 NHWC, bits partials
    [B,T] float64, y fp32 | None, ŷ bf16 NHWC). rtab: ``rate_table`` of rate_packed (made here
    when not given)."""
    _check_bf16(h, "activation")
    B, h8, w8, N = h.shape
    _check_channels(N)
    H, W = 8 * h8, 8 * w8
    _check_image_dims(H, W)
    y_hat = torch.empty(B, h8 // 2, w8 // 2, N, device=h.device, dtype=torch.float32)
    y_hat_bf = torch.empty(B, h8 // 2, w8 // 2, N, device=h.device, dtype=torch.int16)
    y = torch.empty_like(y_hat) if want_y else None
    T = query("iclr17_bf16_rate_partials_per_image", H, W, N)
    partial = torch.empty(B, T, device=h.device, dtype=torch.float64)
    if rtab is None:
        rtab = rate_table(rate_packed, N)
    call("iclr17_analysis_conv3_quant_rate_bf16", _p(h), B, H, W, N, _p(w_bf), _p(rate_packed),
         _p(rtab), _p(y), _p(y_hat), _p(y_hat_bf), _p(partial), _stream(h))
    return y_hat, partial, y, y_hat_bf


def deconv_igdn_bf16(h: Tensor, w_bf: Tensor, bias: Tensor, beta_eff: Tensor, g_bf: Tensor) -> Tensor:
    """synthesis_17.py:15-22 in bf16: bf16 NHWC [B,h,w,N] → [B,2h,2w,N]."""
    _check_bf16(h, "activation")
    B, hh, ww, N = h.shape
    _check_channels(N)
    out = torch.empty(B, 2 * hh, 2 * ww, N, device=h.device, dtype=torch.int16)
    call("iclr17_synthesis_deconv_igdn_bf16", _p(h), B, hh, ww, N, _p(w_bf), _p(bias),
         _p(beta_eff), _p(g_bf), _p(out), _stream(h))
    return out


def deconv3_bf16(h: Tensor, wb: Tensor, bias: Tensor, x_ref: Optional[Tensor] = None,
                 want_recon: bool = False, sse_unclipped: bool = False,
                 bits: Optional[Tuple[Tensor, float]] = None):
    """synthesis_17.py:23-25 + model.py:59 in bf16: bf16 NHWC [B,H/4,W/4,N] → the ``deconv3``
    returns (wb: ``round_packed(d3, 9, N, 48)`` of the ICLR17_W_DECONV9 packing d3)."""
    _check_bf16(h, "activation")
    B, h4, w4, N = h.shape
    if wb.dtype != torch.int16 or wb.numel() != 9 * N * 48:
        raise Iclr17Error("iclr17: deconv3_bf16: weights are not round_packed(d3, 9, N, 48)")
    return _deconv3_halo("iclr17_synthesis_deconv3_bf16", h, B, h4, w4, N, wb, bias, x_ref,
                         want_recon, sse_unclipped, bits)


# ---------------------------------------------------------------- entropy coding (§8 f4)
ENTROPY_K = 32            # symbols −K..K per channel (+ escape for larger |ŷ|)
STREAMS_PER_IMAGE = 1     # rANS streams per image (contiguous channel groups; 64 states each)


def entropy_tables(rate_packed: Tensor, N: int, K: int = ENTROPY_K) -> Tensor:
    """Quantised per-channel CDFs of the factorised model: int32 [N, 2K + 3]."""
    _check(rate_packed, "rate table")
    if rate_packed.numel() != 11 * N:
        raise Iclr17Error(f"iclr17: entropy_tables: rate table is not [11][{N}]")
    cum = torch.empty(N, 2 * K + 3, device=rate_packed.device, dtype=torch.int32)
    call("iclr17_entropy_tables", _p(rate_packed), N, K, _p(cum), _stream(rate_packed))
    return cum


def _rans_status(status: Tensor, what: str) -> None:
    st = int(status.item())
    if st:
        why = []
        if st & 1:
            why.append("a latent is not integer-valued (or NaN)")
        if st & 2:
            why.append("|latent| > 32767")
        if st & 4:
            why.append("a stream ran past its words")
        if st & 8:
            why.append("a stream did not end in the initial state")
        raise Iclr17Error(f"iclr17: {what}: " + "; ".join(why))


def rans_encode(y_hat: Tensor, cum: Tensor, K: int = ENTROPY_K,
                streams_per_image: int = STREAMS_PER_IMAGE):
    """ŷ NHWC [B,h,w,N] → (words int16 [T] (uint16 bit patterns), offsets int64 [B·P + 1]);
    stream b·P + g holds channels g·N/P .. of image b."""
    _check(y_hat, "latent", 4)
    B, h, w, N = y_hat.shape
    P = streams_per_image
    cap = query("iclr17_rans_capacity", h, w, N, P)
    if cap <= 0:
        raise Iclr17Error(f"iclr17: rans_encode: N={N} not divisible into {P} streams")
    dev = y_hat.device
    scratch = torch.empty(B * P * cap, device=dev, dtype=torch.int16)
    lengths = torch.empty(B * P, device=dev, dtype=torch.int32)
    status = torch.zeros(1, device=dev, dtype=torch.int32)
    st = _stream(y_hat)
    call("iclr17_rans_encode", _p(y_hat.contiguous()), B, h, w, N, P, _p(cum), K, _p(scratch),
         scratch.numel(), _p(lengths), _p(status), st)
    offsets = torch.empty(B * P + 1, device=dev, dtype=torch.int64)
    call("iclr17_rans_offsets", _p(lengths), B * P, _p(offsets), st)
    total = int(offsets[-1].item())
    words = torch.empty(max(total, 1), device=dev, dtype=torch.int16)
    call("iclr17_rans_pack", _p(scratch), cap, _p(offsets), B * P, _p(words), st)
    _rans_status(status, "rans_encode")
    return words[:total], offsets


def rans_decode(words: Tensor, offsets: Tensor, cum: Tensor, B: int, h: int, w: int, N: int,
                K: int = ENTROPY_K, streams_per_image: int = STREAMS_PER_IMAGE) -> Tensor:
    """Inverse of rans_encode → ŷ NHWC fp32 [B,h,w,N]."""
    P = streams_per_image
    if offsets.numel() != B * P + 1 or N % P:
        raise Iclr17Error("iclr17: rans_decode: offsets do not match B x streams_per_image")
    dev = cum.device
    y = torch.empty(B, h, w, N, device=dev, dtype=torch.float32)
    status = torch.zeros(1, device=dev, dtype=torch.int32)
    words = words.contiguous() if words.numel() else torch.zeros(1, device=dev, dtype=torch.int16)
    call("iclr17_rans_decode", _p(words), _p(offsets.contiguous()), B, h, w, N, P, _p(cum), K,
         _p(y), _p(status), _stream(y))
    _rans_status(status, "rans_decode")
    return y


def reduce_partials(partial: Tensor, scale: float = 1.0, per_image: bool = True):
    """Deterministic per-image sums (float64 [B]) and scale·Σ (float32 0-dim)."""
    _check_f64(partial)
    B, T = partial.shape
    per = torch.empty(B, device=partial.device, dtype=torch.float64) if per_image else None
    total = torch.empty((), device=partial.device, dtype=torch.float32)
    call("iclr17_reduce_partials", _p(partial.contiguous()), B, T, _p(per), _p(total),
         ctypes.c_double(scale), _stream(partial))
    return per, total


def _check_f64(t: Tensor) -> None:
    if t.device.type != "cuda" or t.dtype != torch.float64 or t.dim() != 2:
        raise Iclr17Error("iclr17: partial sums must be a 2-D float64 GPU tensor")


# ------------------------------------------------------------------------------ modules
def gdn(x: Tensor, beta_eff: Tensor, gp: Tensor, inverse: bool) -> Tensor:
    """GDN.forward (models/GDN.py:64-94) on a 4-D tensor; keeps the input's memory format."""
    _check(x, "input", 4)
    B, C, H, W = x.shape
    _check_channels(C)
    if x.is_contiguous():
        layout, src = _lib.ICLR17_LAYOUT_NCHW, x
        y = torch.empty_like(x)
    elif x.is_contiguous(memory_format=torch.channels_last):
        layout, src = _lib.ICLR17_LAYOUT_NHWC, x
        y = torch.empty_like(x, memory_format=torch.channels_last)
    else:
        layout, src = _lib.ICLR17_LAYOUT_NCHW, x.contiguous()
        y = torch.empty_like(src)
    call("iclr17_gdn", _p(src), B, C, H, W, layout, int(bool(inverse)), _p(beta_eff), _p(gp),
         _p(y), _stream(x))
    return y


def _layout_inner(x: Tensor) -> Tuple[Tensor, int]:
    """(tensor, inner) such that channel of flat element i is (i // inner) % C."""
    if x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last):
        return x, 1
    x = x.contiguous()
    inner = int(np.prod(x.shape[2:])) if x.dim() > 2 else 1
    return x, inner


def bit_estimator(x: Tensor, rate_packed: Tensor, C: int) -> Tensor:
    """BitEstimator.forward (bitEstimator.py:38-42): elementwise CDF, channel dim 1."""
    _check(x, "input")
    if x.dim() < 2 or x.shape[1] != C:
        raise Iclr17Error(f"iclr17: BitEstimator input needs {C} channels in dim 1")
    src, inner = _layout_inner(x)
    out = torch.empty_like(src)
    call("iclr17_bit_estimator", _p(src), src.numel(), C, inner, _p(rate_packed), _p(out),
         _stream(x))
    return out


def bitparm(x: Tensor, h: Tensor, b: Tensor, a: Optional[Tensor]) -> Tensor:
    """One Bitparm layer (bitEstimator.py:20-25)."""
    _check(x, "input")
    C = h.numel()
    if x.dim() < 2 or x.shape[1] != C:
        raise Iclr17Error(f"iclr17: Bitparm input needs {C} channels in dim 1")
    src, inner = _layout_inner(x)
    out = torch.empty_like(src)
    work = torch.empty(2 * C, device=x.device, dtype=torch.float32)
    hc, bc = h.detach().reshape(-1).contiguous(), b.detach().reshape(-1).contiguous()
    ac = a.detach().reshape(-1).contiguous() if a is not None else None
    call("iclr17_bitparm", _p(src), src.numel(), C, inner, _p(hc), _p(bc), _p(ac), _p(work),
         _p(out), _stream(x))
    return out


def gdn_backward(x: Tensor, g: Tensor, beta_eff: Tensor, gp: Tensor, gpt: Tensor, inverse: bool):
    """Autograd of ``gdn`` (GDN.py:64-94) → (∂x in x's layout, dn NHWC [P, C], u NHWC [P, C])."""
    _check(x, "input", 4)
    B, C, H, W = x.shape
    _check_channels(C)
    if x.is_contiguous():
        layout, src = _lib.ICLR17_LAYOUT_NCHW, x
    elif x.is_contiguous(memory_format=torch.channels_last):
        layout, src = _lib.ICLR17_LAYOUT_NHWC, x
    else:
        layout, src = _lib.ICLR17_LAYOUT_NCHW, x.contiguous()
    mf = torch.channels_last if layout == _lib.ICLR17_LAYOUT_NHWC else torch.contiguous_format
    gs = g.contiguous(memory_format=mf)
    dx = torch.empty_like(src, memory_format=mf)
    P = B * H * W
    dn = torch.empty(P, C, device=x.device, dtype=torch.float32)
    u = torch.empty(P, C, device=x.device, dtype=torch.float32) if layout == _lib.ICLR17_LAYOUT_NCHW else None
    call("iclr17_gdn_bwd", _p(src), _p(gs), B, C, H, W, layout, int(bool(inverse)), _p(beta_eff),
         _p(gp), _p(gpt), _p(dx), _p(dn), _p(u), _stream(x))
    if u is None:   # NHWC input: x itself is the [P, C] operand
        u = src.permute(0, 2, 3, 1).reshape(P, C)
    return dx, dn, u


def _like_layout(g: Tensor, src: Tensor) -> Tensor:
    """g in src's memory layout (contiguous, or channels-last for a channels-last 4-D src)."""
    if src.dim() == 4 and not src.is_contiguous():
        return g.contiguous(memory_format=torch.channels_last)
    return g.contiguous()


def _bitest_partials(x: Tensor, C: int) -> Tensor:
    T = query("iclr17_bitest_bwd_chunks", x.numel(), C)
    return torch.empty(T, 11, C, device=x.device, dtype=torch.float32)


def bit_estimator_backward(x: Tensor, g: Tensor, rate_packed: Tensor, C: int):
    """Autograd of ``bit_estimator`` → (∂x, parameter partials [T, 11, C] for rate_param_grads)."""
    src, inner = _layout_inner(x)
    gs = _like_layout(g, src)
    dx = torch.empty_like(src)
    part = _bitest_partials(src, C)
    call("iclr17_bit_estimator_bwd", _p(src), _p(gs), src.numel(), C, inner, _p(rate_packed),
         _p(dx), _p(part), _stream(x))
    return dx, part


def bitparm_backward(x: Tensor, g: Tensor, h: Tensor, b: Tensor, a: Optional[Tensor]):
    """Autograd of ``bitparm`` → (∂x, parameter partials [T, 11, C]: slots 0-2, or 9-10 final)."""
    C = h.numel()
    src, inner = _layout_inner(x)
    gs = _like_layout(g, src)
    dx = torch.empty_like(src)
    part = _bitest_partials(src, C)
    work = torch.empty(11 * C, device=x.device, dtype=torch.float32)
    hc, bc = h.detach().reshape(-1).contiguous(), b.detach().reshape(-1).contiguous()
    ac = a.detach().reshape(-1).contiguous() if a is not None else None
    call("iclr17_bitparm_bwd", _p(src), _p(gs), src.numel(), C, inner, _p(hc), _p(bc), _p(ac),
         _p(work), _p(dx), _p(part), _stream(x))
    return dx, part


def rate_bits(z: Tensor, rate_packed: Tensor) -> Tensor:
    """model.py:71-73 on a 4-D latent: per-image Σ bits partials [B, T] (float64)."""
    _check(z, "latent", 4)
    B, C, h, w = z.shape
    if z.is_contiguous():
        layout, src = _lib.ICLR17_LAYOUT_NCHW, z
    elif z.is_contiguous(memory_format=torch.channels_last):
        layout, src = _lib.ICLR17_LAYOUT_NHWC, z
    else:
        layout, src = _lib.ICLR17_LAYOUT_NCHW, z.contiguous()
    T = query("iclr17_rate_bits_partials", C, h, w)
    partial = torch.empty(B, T, device=z.device, dtype=torch.float64)
    call("iclr17_rate_bits", _p(src), B, C, h, w, layout, _p(rate_packed), _p(partial), _stream(z))
    return partial


# ------------------------------------------------------------------------------ backward
def grad_recon(recon: Tensor, x: Tensor, g_mse: Optional[Tensor], g_clip: Optional[Tensor]) -> Tensor:
    """∂L/∂recon for L using mean((recon−x)²) (g_mse, 0-dim) and/or clamp(recon,0,1) (g_clip)."""
    _check(recon, "recon")
    out = torch.empty_like(recon)
    gm = g_mse.detach().reshape(()).contiguous() if g_mse is not None else None
    gc = g_clip.detach().contiguous() if g_clip is not None else None
    call("iclr17_grad_recon", _p(recon), _p(x.contiguous()), _p(gm), _p(gc), recon.numel(),
         _p(out), _stream(recon))
    return out


def _colsum_buffers(t: Tensor, kind: int, h: int, w: int):
    B, N = t.shape[0], t.shape[-1]
    T = B * query("iclr17_bwd_tiles", kind, h, w)
    return (torch.empty(T, N, device=t.device, dtype=torch.float32),
            torch.empty(T, N, device=t.device, dtype=torch.float32))


def sum_rows(part: Tensor) -> Tensor:
    """Fixed-order column sums of a [T, C] float32 partial buffer."""
    T, C = part.shape
    out = torch.empty(C, device=part.device, dtype=torch.float32)
    ws = torch.empty(query("iclr17_sum_rows_workspace_size", C), device=part.device,
                     dtype=torch.float32)
    call("iclr17_sum_rows", _p(part), T, C, _p(ws), _p(out), _stream(part))
    return out


def sum_rows2(a: Tensor, b: Tensor):
    """``sum_rows`` of two [T, C] partial buffers of one shape in one launch pair."""
    T, C = a.shape
    if tuple(b.shape) != (T, C):
        raise Iclr17Error("iclr17: sum_rows2 needs two partial buffers of one shape")
    oa = torch.empty(C, device=a.device, dtype=torch.float32)
    ob = torch.empty(C, device=a.device, dtype=torch.float32)
    ws = torch.empty(2 * query("iclr17_sum_rows_workspace_size", C), device=a.device,
                     dtype=torch.float32)
    call("iclr17_sum_rows2", _p(a), _p(b), T, C, _p(ws), _p(oa), _p(ob), _stream(a))
    return oa, ob


def _split_like(t: Tensor) -> Tensor:
    return torch.empty((3,) + tuple(t.shape), device=t.device, dtype=torch.int16)


def bwd_deconv3_igdn(g_recon: Tensor, wp_conv1form: Optional[Tensor], v_saved: Tensor,
                     beta_eff: Tensor, gp: Tensor, gpt: Tensor, w_split: Optional[Tensor] = None,
                     want_split: bool = False, g6: Optional[Tensor] = None,
                     g6t: Optional[Tensor] = None, want_f32: bool = True):
    """deconv3 input-gradient fused with IGDN2 backward →
    (g_v2 NHWC, dn NHWC, Σ g_v2 = ∂bias of deconv2, Σ dn = ∂β_eff of IGDN2[, g_v2 split]).
    w_split (``pack_conv1_x6`` of the deconv3 weight) runs the contraction in x6. want_f32=False
    (with want_split): g_v2 is not written (None), only its split form."""
    B, _, H, W = g_recon.shape
    N = v_saved.shape[3]
    g_v = torch.empty_like(v_saved) if want_f32 or not want_split else None
    dn = torch.empty_like(v_saved)
    sp = _split_like(v_saved) if want_split else None
    cs_g, cs_d = _colsum_buffers(v_saved, 0, H // 4, W // 4)
    call("iclr17_bwd_deconv3_igdn", _p(g_recon.contiguous()), B, H, W, N, _p(wp_conv1form),
         _p(w_split), _p(v_saved), _p(beta_eff), _p(gp), _p(gpt), _p(g6), _p(g6t), _p(g_v),
         _p(sp), _p(dn),
         _p(cs_g), _p(cs_d), _stream(g_recon))
    out = (g_v, dn, *sum_rows2(cs_g, cs_d))
    return out + (sp,) if want_split else out


def bwd_deconv_igdn(g_v: Optional[Tensor], wp_conv5form: Tensor, v_prev: Tensor, beta_eff: Tensor,
                    gp: Tensor, gpt: Tensor, g_split: Optional[Tensor] = None,
                    want_split: bool = False, g6: Optional[Tensor] = None,
                    g6t: Optional[Tensor] = None, want_f32: bool = True):
    """deconv2 input-gradient fused with IGDN1 backward →
    (g_v1 NHWC, dn NHWC, Σ g_v1 = ∂bias of deconv1, Σ dn = ∂β_eff of IGDN1[, g_v1 split]).
    g_split (g_v in split form) runs the contraction in x6. want_f32=False (with want_split):
    g_v1 is not written (None)."""
    B, h, w, N = v_prev.shape
    g_prev = torch.empty_like(v_prev) if want_f32 or not want_split else None
    dn = torch.empty_like(v_prev)
    sp = _split_like(v_prev) if want_split else None
    cs_g, cs_d = _colsum_buffers(v_prev, 0, h, w)
    gin = g_v.contiguous() if g_split is None else None
    call("iclr17_bwd_deconv_igdn", _p(gin), _p(g_split), B, h, w, N, _p(wp_conv5form), _p(v_prev),
         _p(beta_eff), _p(gp), _p(gpt), _p(g6), _p(g6t), _p(g_prev), _p(sp), _p(dn), _p(cs_g), _p(cs_d),
         _stream(v_prev))
    out = (g_prev, dn, *sum_rows2(cs_g, cs_d))
    return out + (sp,) if want_split else out


def bwd_deconv_rate(g_v1: Optional[Tensor], wp_conv5form: Tensor, y_tilde: Optional[Tensor],
                    rate_packed: Optional[Tensor], g_bpp: Optional[Tensor], count: float,
                    h: int, w: int, g_split: Optional[Tensor] = None, want_split: bool = False):
    """deconv1 input-gradient (+ rate backward when g_bpp is given) →
    (g_y NHWC, rate partials[, g_y split]). g_split (g_v1 in split form) runs x6."""
    ref = g_v1 if g_split is None else g_split[0]
    B, _, _, N = ref.shape
    g_y = torch.empty(B, h, w, N, device=ref.device, dtype=torch.float32)
    sp = _split_like(g_y) if want_split else None
    part = None
    gb = None
    if g_bpp is not None:
        T = query("iclr17_rate_bwd_partials", h, w)
        part = torch.empty(B * T, 11, N, device=ref.device, dtype=torch.float32)
        gb = g_bpp.detach().reshape(()).contiguous()
    gin = g_v1.contiguous() if g_split is None else None
    call("iclr17_bwd_deconv_rate", _p(gin), _p(g_split), B, h, w, N, _p(wp_conv5form),
         _p(y_tilde), _p(rate_packed), _p(gb), ctypes.c_float(count), _p(g_y), _p(sp), _p(part),
         _stream(ref))
    return (g_y, part, sp) if want_split else (g_y, part)


def bwd_conv_gdn(g_u: Optional[Tensor], wp_deconv5form: Tensor, u_prev: Tensor, beta_eff: Tensor,
                 gp: Tensor, gpt: Tensor, g_split: Optional[Tensor] = None,
                 want_split: bool = False, g6: Optional[Tensor] = None,
                 g6t: Optional[Tensor] = None, want_f32: bool = True):
    """conv3/conv2 input-gradient fused with GDN2/GDN1 backward →
    (g_u_prev NHWC, dn NHWC, Σ g_u_prev = ∂bias of the previous conv, Σ dn = ∂β_eff
    [, g_u_prev split]). g_split (g_u in split form) runs the contraction in x6. want_f32=False
    (with want_split): g_u_prev is not written (None)."""
    ref = g_u if g_split is None else g_split[0]
    B, h, w, N = ref.shape
    g_prev = torch.empty_like(u_prev) if want_f32 or not want_split else None
    dn = torch.empty_like(u_prev)
    sp = _split_like(u_prev) if want_split else None
    cs_g, cs_d = _colsum_buffers(u_prev, 1, h, w)
    gin = g_u.contiguous() if g_split is None else None
    call("iclr17_bwd_conv_gdn", _p(gin), _p(g_split), B, h, w, N, _p(wp_deconv5form), _p(u_prev),
         _p(beta_eff), _p(gp), _p(gpt), _p(g6), _p(g6t), _p(g_prev), _p(sp), _p(dn), _p(cs_g), _p(cs_d),
         _stream(u_prev))
    out = (g_prev, dn, *sum_rows2(cs_g, cs_d))
    return out + (sp,) if want_split else out


def wgrad_k5(G: Tensor, X: Tensor) -> Tensor:
    """dW [M][C][5][5] = Σ G[b,o,m] · X[b,2o−2+k,c] (NHWC G [B,Ho,Wo,M], X [B,2Ho,2Wo,C])."""
    B, Ho, Wo, M = G.shape
    C = X.shape[3]
    ws = torch.empty(query("iclr17_wgrad_workspace_size", 5, B, Ho, Wo, M, C), device=G.device,
                     dtype=torch.float32)
    dW = torch.empty(M, C, 5, 5, device=G.device, dtype=torch.float32)
    call("iclr17_wgrad_k5", _p(G.contiguous()), _p(X.contiguous()), B, Ho, Wo, M, C, _p(ws), _p(dW),
         _stream(G))
    return dW


def wgrad_k5_x6(G_split: Tensor, X_split: Tensor) -> Tensor:
    """wgrad_k5 in x6 from split-form operands (G_split [3,B,Ho,Wo,M], X_split [3,B,2Ho,2Wo,C])."""
    _check_split(G_split, "wgrad G")
    _check_split(X_split, "wgrad X")
    _, B, Ho, Wo, M = G_split.shape
    C = X_split.shape[4]
    if tuple(X_split.shape[1:4]) != (B, 2 * Ho, 2 * Wo):
        raise Iclr17Error(f"iclr17: wgrad_k5_x6: X {tuple(X_split.shape)} vs G {tuple(G_split.shape)}")
    ws = torch.empty(query("iclr17_wgrad_workspace_size", 6, B, Ho, Wo, M, C), device=G_split.device,
                     dtype=torch.float32)
    dW = torch.empty(M, C, 5, 5, device=G_split.device, dtype=torch.float32)
    call("iclr17_wgrad_k5_x6", _p(G_split), _p(X_split), B, Ho, Wo, M, C, _p(ws), _p(dW),
         _stream(G_split))
    return dW


def wgrad_k9_x6(G_split: Tensor, X: Tensor) -> Tensor:
    """wgrad_k9 in x6: G_split [3,B,Ho,Wo,M] split form, X NCHW fp32 [B,3,4Ho,4Wo]."""
    _check_split(G_split, "wgrad G")
    _check(X, "wgrad X", 4)
    _, B, Ho, Wo, M = G_split.shape
    if tuple(X.shape) != (B, 3, 4 * Ho, 4 * Wo):
        raise Iclr17Error(f"iclr17: wgrad_k9_x6: X {tuple(X.shape)} vs G {tuple(G_split.shape)}")
    ws = torch.empty(query("iclr17_wgrad_workspace_size", 7, B, Ho, Wo, M, 3), device=X.device,
                     dtype=torch.float32)
    dW = torch.empty(M, 3, 9, 9, device=X.device, dtype=torch.float32)
    call("iclr17_wgrad_k9_x6", _p(G_split), _p(X.contiguous()), B, Ho, Wo, M, _p(ws), _p(dW),
         _stream(X))
    return dW


def wgrad_k9(G: Tensor, X: Tensor) -> Tensor:
    """dW [M][3][9][9] = Σ G[b,o,m] · X[b,c,4o−4+k] (G NHWC [B,Ho,Wo,M], X NCHW [B,3,4Ho,4Wo])."""
    B, Ho, Wo, M = G.shape
    ws = torch.empty(query("iclr17_wgrad_workspace_size", 9, B, Ho, Wo, M, 3), device=G.device,
                     dtype=torch.float32)
    dW = torch.empty(M, 3, 9, 9, device=G.device, dtype=torch.float32)
    call("iclr17_wgrad_k9", _p(G.contiguous()), _p(X.contiguous()), B, Ho, Wo, M, _p(ws), _p(dW),
         _stream(G))
    return dW


def gdn_wgrad(dn: Tensor, u: Tensor, x6: Optional[bool] = None) -> Tensor:
    """dγ_eff [C, C] = Σ_p dn[p] ⊗ u[p]² (GDN.py:83); x6 (default: the build's precision) or
    exact f32."""
    C = dn.shape[-1]
    P = dn.numel() // C
    if x6 is None:
        x6 = precision() != "fp32"
    name = "iclr17_gdn_wgrad_x6" if x6 else "iclr17_gdn_wgrad"
    ws = torch.empty(query(name + "_workspace_size", P, C), device=dn.device, dtype=torch.float32)
    dge = torch.empty(C, C, device=dn.device, dtype=torch.float32)
    call(name, _p(dn.contiguous()), _p(u.contiguous()), P, C, _p(ws), _p(dge), _stream(dn))
    return dge


def gdn_param_grads(dn: Tensor, u: Tensor, dbe: Tensor, beta: Tensor, gamma: Tensor,
                    beta_bound: float = DEFAULT_BETA_BOUND, gamma_bound: float = DEFAULT_GAMMA_BOUND):
    """GDN parameter gradients (dβ, dγ) in the raw-parameter space (through GDN.py:73-79);
    dbe = ∂β_eff (Σ dn, from the backward kernel's column sums)."""
    C = dn.shape[-1]
    dge = gdn_wgrad(dn, u)
    db = torch.empty_like(dbe)
    dg = torch.empty_like(dge)
    call("iclr17_gdn_param_chain", _p(beta.detach().contiguous()), _p(gamma.detach().contiguous()),
         _p(dbe), _p(dge), C, ctypes.c_float(beta_bound), ctypes.c_float(gamma_bound), _p(db), _p(dg),
         _stream(dn))
    return db, dg


def bias_grad_nhwc(G: Tensor) -> Tensor:
    C = G.shape[-1]
    P = G.numel() // C
    ws = torch.empty((1024 + 64) * C, device=G.device, dtype=torch.float32)
    db = torch.empty(C, device=G.device, dtype=torch.float32)
    call("iclr17_bias_grad_nhwc", _p(G.contiguous()), P, C, _p(ws), _p(db), _stream(G))
    return db


def bias_grad_nchw(G: Tensor) -> Tensor:
    B, C, H, W = G.shape
    ws = torch.empty((B * ((H * W + 4095) // 4096) + 64) * C, device=G.device, dtype=torch.float32)
    db = torch.empty(C, device=G.device, dtype=torch.float32)
    call("iclr17_bias_grad_nchw", _p(G.contiguous()), B, C, H * W, _p(ws), _p(db), _stream(G))
    return db


def rate_param_grads(partial: Tensor, params: Sequence[Tensor]):
    """BitEstimator grads (h1 b1 a1 h2 b2 a2 h3 b3 a3 h4 b4) from rate partials [T,11,C]."""
    T, _, C = partial.shape
    h1, b1, a1, h2, b2, a2, h3, b3, a3, h4, b4 = [p.detach().reshape(-1).contiguous() for p in params]
    outs = [torch.empty(C, device=partial.device, dtype=torch.float32) for _ in range(11)]
    call("iclr17_rate_param_grad", _p(partial), T, C, _p(h1), _p(a1), _p(h2), _p(a2), _p(h3), _p(a3),
         _p(h4), *[_p(o) for o in outs], _stream(partial))
    return [o.view(1, C, 1, 1) for o in outs]
