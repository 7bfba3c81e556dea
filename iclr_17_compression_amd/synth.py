"""Deterministic synthetic inputs and "trained-like" codec weights.

Everything here is exact integer / dyadic arithmetic on a counter-based splitmix64
stream, so this container, the GPU box and any later round regenerate bit-identical
tensors from a seed (no transcendental functions whose last bit could depend on the
host's SIMD library). Used by tests, the golden generator, smoke() and bench.py.

Shapes and parameter names follow the reference state_dict:
``Encoder.conv1.weight [N,3,9,9]`` … ``bitEstimator.f4.b [1,N,1,1]``.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, stream: int = 0) -> np.ndarray:
    """n raw 64-bit draws of stream ``(seed, stream)``; element i depends only on i."""
    base = np.uint64(((seed & 0xFFFFFF) << 40) ^ ((stream & 0xFFFF) << 24))
    with np.errstate(over="ignore"):
        z = np.arange(n, dtype=np.uint64) + base
        z = z + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, shape, lo: float = 0.0, hi: float = 1.0, stream: int = 0) -> np.ndarray:
    """float32 uniform in [lo, hi): 24-bit dyadic draws, one multiply-add in float64."""
    n = int(np.prod(shape))
    u = (splitmix64(seed, n, stream) >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def normal_like(seed: int, shape, std: float = 1.0, stream: int = 0) -> np.ndarray:
    """Zero-mean, unit-variance Irwin-Hall(4) draws scaled by ``std`` (exact arithmetic)."""
    n = int(np.prod(shape))
    z = splitmix64(seed, 4 * n, stream)
    u = (z >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))
    s = u.reshape(n, 4).sum(axis=1) - 2.0           # var = 4/12
    return (s * (math.sqrt(3.0) * std)).astype(np.float32).reshape(shape)


def image_u8(seed: int, batch: int, height: int, width: int) -> np.ndarray:
    """Uniform uint8 pixels, NCHW (the C1/C3/C5 bench inputs: splitmix64 → u8)."""
    z = splitmix64(seed, batch * 3 * height * width, stream=7)
    return (z >> np.uint64(56)).astype(np.uint8).reshape(batch, 3, height, width)


def smooth_image_u8(seed: int, height: int, width: int, cell: int = 32) -> np.ndarray:
    """Natural-ish 3xHxW uint8 image: bilinear field over a coarse random grid plus
    fine noise, integer fixed-point arithmetic only (used for the synthetic Kodak-24)."""
    gh, gw = height // cell + 2, width // cell + 2
    grid = (splitmix64(seed, 3 * gh * gw, stream=11) >> np.uint64(56)).astype(np.int64)
    grid = grid.reshape(3, gh, gw)
    ys = np.arange(height, dtype=np.int64)
    xs = np.arange(width, dtype=np.int64)
    y0, fy = ys // cell, ys % cell
    x0, fx = xs // cell, xs % cell
    g00 = grid[:, y0][:, :, x0]
    g01 = grid[:, y0][:, :, x0 + 1]
    g10 = grid[:, y0 + 1][:, :, x0]
    g11 = grid[:, y0 + 1][:, :, x0 + 1]
    fy = fy[None, :, None]
    fx = fx[None, None, :]
    c = cell
    v = (g00 * (c - fy) * (c - fx) + g01 * (c - fy) * fx + g10 * fy * (c - fx) + g11 * fy * fx)
    v = v // (c * c)
    noise = (splitmix64(seed, 3 * height * width, stream=12) >> np.uint64(59)).astype(np.int64)
    v = v + noise.reshape(3, height, width) - 16
    return np.clip(v, 0, 255).astype(np.uint8)


def to_unit_float(u8: np.ndarray) -> np.ndarray:
    """torchvision ToTensor semantics: float32(u8) / 255 in float32."""
    return u8.astype(np.float32) / np.float32(255.0)


def _xavier_std(shape, gain: float) -> float:
    # torch.nn.init._calculate_fan_in_and_fan_out on a 4-D weight
    rf = int(np.prod(shape[2:]))
    fan_in, fan_out = shape[1] * rf, shape[0] * rf
    return gain * math.sqrt(2.0 / float(fan_in + fan_out))


def trained_like_state_dict(N: int = 192, seed: int = 1) -> Dict[str, np.ndarray]:
    """A dense, "trained-like" parameter set in the reference's state_dict layout.

    Convs at the reference init scale (analysis_17.py:15-23, synthesis_17.py:16-25);
    GDN gamma dense (γ = sqrt(0.1·I + U(0, 0.01))) so the cross-channel sum is exercised
    (reference init makes the effective gamma exactly diagonal), with a few
    entries pushed below the LowerBound bounds (models/GDN.py:10-24); BitEstimator
    h/b/a ~ U(-1, 1).
    """
    sd: Dict[str, np.ndarray] = {}
    k = [0]

    def nxt() -> int:
        k[0] += 1
        return seed * 64 + k[0]

    def conv(name, shape, gain, bias, transposed=False):
        sd[name + ".weight"] = normal_like(nxt(), shape, _xavier_std(shape, gain))
        if bias:
            cout = shape[1] if transposed else shape[0]
            sd[name + ".bias"] = uniform(nxt(), (cout,), -0.01, 0.03)

    def gdn(name, ch):
        beta = np.sqrt(uniform(nxt(), (ch,), 0.5, 1.5).astype(np.float64)).astype(np.float32)
        beta[0] = np.float32(1e-4)              # below beta_bound → LowerBound active
        beta[ch // 2] = np.float32(-0.2)        # negative reparam value
        g = 0.1 * np.eye(ch, dtype=np.float64) + uniform(nxt(), (ch, ch), 0.0, 0.01).astype(np.float64)
        gamma = np.sqrt(g).astype(np.float32)
        sel = (splitmix64(nxt(), ch * ch) >> np.uint64(58)).reshape(ch, ch) == 0   # ~1/64
        gamma[sel] = np.float32(-0.003)         # below gamma_bound (2^-18)
        sd[name + ".beta"] = beta
        sd[name + ".gamma"] = gamma

    conv("Encoder.conv1", (N, 3, 9, 9), math.sqrt(2 * (3 + N) / 6), True)
    gdn("Encoder.gdn1", N)
    conv("Encoder.conv2", (N, N, 5, 5), math.sqrt(2), True)
    gdn("Encoder.gdn2", N)
    conv("Encoder.conv3", (N, N, 5, 5), math.sqrt(2), False)
    conv("Decoder.deconv1", (N, N, 5, 5), math.sqrt(2), True, True)
    gdn("Decoder.igdn1", N)
    conv("Decoder.deconv2", (N, N, 5, 5), math.sqrt(2), True, True)
    gdn("Decoder.igdn2", N)
    conv("Decoder.deconv3", (N, 3, 9, 9), math.sqrt(2), True, True)
    for f in ("f1", "f2", "f3", "f4"):
        sd[f"bitEstimator.{f}.h"] = uniform(nxt(), (1, N, 1, 1), -1.0, 1.0)
        sd[f"bitEstimator.{f}.b"] = uniform(nxt(), (1, N, 1, 1), -1.0, 1.0)
        if f != "f4":
            sd[f"bitEstimator.{f}.a"] = uniform(nxt(), (1, N, 1, 1), -1.0, 1.0)
    return sd


STATE_DICT_KEYS = (
    "Encoder.conv1.weight", "Encoder.conv1.bias", "Encoder.gdn1.beta", "Encoder.gdn1.gamma",
    "Encoder.conv2.weight", "Encoder.conv2.bias", "Encoder.gdn2.beta", "Encoder.gdn2.gamma",
    "Encoder.conv3.weight",
    "Decoder.deconv1.weight", "Decoder.deconv1.bias", "Decoder.igdn1.beta", "Decoder.igdn1.gamma",
    "Decoder.deconv2.weight", "Decoder.deconv2.bias", "Decoder.igdn2.beta", "Decoder.igdn2.gamma",
    "Decoder.deconv3.weight", "Decoder.deconv3.bias",
    "bitEstimator.f1.h", "bitEstimator.f1.b", "bitEstimator.f1.a",
    "bitEstimator.f2.h", "bitEstimator.f2.b", "bitEstimator.f2.a",
    "bitEstimator.f3.h", "bitEstimator.f3.b", "bitEstimator.f3.a",
    "bitEstimator.f4.h", "bitEstimator.f4.b",
)


def noisy_pair_u8(B: int, H: int, W: int, seed_img: int, seed_noise: int, div: int):
    """(x, y) uint8 image pair [B,3,H,W]: x a smooth synthetic image, y = clip(x + noise // div)
    with centred uint8 noise — integer arithmetic only (the MS-SSIM fixture G6)."""
    x8 = np.stack([smooth_image_u8(seed_img + b, H, W) for b in range(B)])
    n8 = image_u8(seed_noise, B, H, W).astype(np.int32) - 128
    y8 = np.clip(x8.astype(np.int32) + n8 // div, 0, 255).astype(np.uint8)
    return x8, y8
