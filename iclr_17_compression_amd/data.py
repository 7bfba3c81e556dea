"""Training data path — datasets.py:14-37 (``Datasets``: RandomResizedCrop(256),
RandomHorizontalFlip, RandomVerticalFlip, ToTensor) with the pixel work on the GPU.

The host decodes images to uint8 RGB (PIL, as the reference does) and makes the random
choices; ``iclr17_resized_crop_batch`` (csrc/datapath.hip) resamples, flips and converts on the
device, from uint8 uploads. The random choices follow torchvision's algorithms on numpy's RNG
(the reference's torch RNG stream itself is not reproduced, only its distribution); the pixel
arithmetic is PIL's 8-bit bilinear resampling and equals the reference's PIL path bit for bit.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import kernels
from ._lib import Iclr17Error, call

PIL_PREC = 22   # Resample.c PRECISION_BITS for 8-bit images


def random_resized_crop_params(rng: np.random.Generator, height: int, width: int,
                               scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0)):
    """torchvision RandomResizedCrop.get_params: (top, left, h, w)."""
    area = height * width
    log_ratio = (math.log(ratio[0]), math.log(ratio[1]))
    for _ in range(10):
        target_area = area * rng.uniform(scale[0], scale[1])
        aspect = math.exp(rng.uniform(log_ratio[0], log_ratio[1]))
        w = int(round(math.sqrt(target_area * aspect)))
        h = int(round(math.sqrt(target_area / aspect)))
        if 0 < w <= width and 0 < h <= height:
            return int(rng.integers(0, height - h + 1)), int(rng.integers(0, width - w + 1)), h, w
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


def pil_bilinear_taps(in_size: int, out_size: int) -> Tuple[np.ndarray, int]:
    """PIL's precompute_coeffs + normalize_coeffs_8bpc for BILINEAR (support 1) resizing a whole
    axis of in_size samples to out_size: int32 rows [out][2 + ksize] = (first, count, taps…)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    center = (np.arange(out_size, dtype=np.float64) + 0.5) * scale
    xmin = np.maximum((center - support + 0.5).astype(np.int64), 0)
    xmax = np.minimum((center + support + 0.5).astype(np.int64), in_size) - xmin
    k = np.arange(ksize, dtype=np.float64)[None, :]
    arg = (k + xmin[:, None] - center[:, None] + 0.5) * (1.0 / filterscale)
    w = np.where(np.abs(arg) < 1.0, 1.0 - np.abs(arg), 0.0)
    w = np.where(k < xmax[:, None], w, 0.0)
    ww = w.sum(axis=1, keepdims=True)
    w = np.where(ww != 0.0, w / np.where(ww != 0.0, ww, 1.0), w)
    kk = np.where(w < 0, -0.5 + w * (1 << PIL_PREC), 0.5 + w * (1 << PIL_PREC)).astype(np.int64)
    rows = np.concatenate([xmin[:, None], xmax[:, None], kk], axis=1).astype(np.int32)
    return rows, ksize


def resized_crop_batch(images: Sequence[np.ndarray], boxes, flips, size: int,
                       device: torch.device) -> torch.Tensor:
    """images: uint8 HWC RGB arrays; boxes: (top, left, h, w) each; flips: (horizontal,
    vertical) each. Returns the NCHW fp32 batch [B, 3, size, size] on ``device``."""
    B = len(images)
    if B == 0 or len(boxes) != B or len(flips) != B:
        raise Iclr17Error("iclr17: resized_crop_batch needs one box and one flip pair per image")
    desc = np.zeros((B, 16), dtype=np.int64)
    tap_rows: List[np.ndarray] = []
    src_off = tmp_off = tap_off = 0
    for b, (img, (ci, cj, ch, cw), (fh, fv)) in enumerate(zip(images, boxes, flips)):
        if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
            raise Iclr17Error("iclr17: images must be uint8 HxWx3")
        H, W, _ = img.shape
        if not (0 <= ci and 0 <= cj and ch > 0 and cw > 0 and ci + ch <= H and cj + cw <= W):
            raise Iclr17Error(f"iclr17: crop box {(ci, cj, ch, cw)} outside a {H}x{W} image")
        tx, kx = pil_bilinear_taps(cw, size)
        ty, ky = pil_bilinear_taps(ch, size)
        desc[b] = (src_off, H, W, ci, cj, ch, cw, int(bool(fh)), int(bool(fv)), tmp_off,
                   tap_off, kx, tap_off + tx.size, ky, 0, 0)
        tap_rows += [tx.ravel(), ty.ravel()]
        tap_off += tx.size + ty.size
        src_off += H * W * 3
        tmp_off += ch * size * 3
    src = torch.from_numpy(np.concatenate([np.ascontiguousarray(i).ravel() for i in images]))
    src = src.pin_memory().to(device, non_blocking=True)
    taps = torch.from_numpy(np.concatenate(tap_rows)).to(device, non_blocking=True)
    d = torch.from_numpy(desc).to(device, non_blocking=True)
    tmp = torch.empty(tmp_off, dtype=torch.uint8, device=device)
    out = torch.empty(B, 3, size, size, dtype=torch.float32, device=device)
    max_ch = int(desc[:, 5].max())
    call("iclr17_resized_crop_batch", kernels._p(src), kernels._p(d), B, size, max_ch,
         kernels._p(taps), kernels._p(tmp), kernels._p(out), kernels._stream(out))
    return out
