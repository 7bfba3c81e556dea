"""ORACLE — the reference's training transform on given random choices. TEST INFRASTRUCTURE ONLY
(imported by tests/ only).

datasets.py:27-33 runs, per image, torchvision's RandomResizedCrop(256) → RandomHorizontalFlip →
RandomVerticalFlip → ToTensor on a PIL RGB image. For PIL inputs torchvision's resized_crop is
``img.crop((left, top, left + w, top + h)).resize((size, size), BILINEAR)``; the flips mirror
the pixel array; ToTensor is uint8 / 255 in fp32, CHW. ``pil_transform`` is exactly that, with
the crop box and flips passed in (torchvision draws them from torch's RNG).

``resample_with_taps`` restates PIL's 8-bit two-pass resampling (Resample.c: horizontal pass,
then vertical, 22-bit fixed-point taps, +2^21, >> 22, clip) on tap tables in the format
``iclr_17_compression_amd.data.pil_bilinear_taps`` produces — it pins that host-side table
against PIL on the CPU.
"""
from __future__ import annotations

import numpy as np

PREC = 22


def pil_transform(img_u8: np.ndarray, box, flips, size: int) -> np.ndarray:
    from PIL import Image
    top, left, h, w = box
    im = Image.fromarray(img_u8).crop((left, top, left + w, top + h))
    a = np.asarray(im.resize((size, size), Image.BILINEAR))
    if flips[0]:
        a = a[:, ::-1]
    if flips[1]:
        a = a[::-1]
    return (a.astype(np.float32) / np.float32(255)).transpose(2, 0, 1).copy()


def _pass(x: np.ndarray, taps: np.ndarray) -> np.ndarray:
    """Resample axis 0 of x ([n_in, ...] uint8) with tap rows [n_out][2 + k]."""
    out = np.empty((taps.shape[0],) + x.shape[1:], np.uint8)
    for o, row in enumerate(taps):
        first, count = int(row[0]), int(row[1])
        acc = np.full(x.shape[1:], 1 << (PREC - 1), np.int64)
        for k in range(count):
            acc += x[first + k].astype(np.int64) * int(row[2 + k])
        out[o] = np.clip(acc >> PREC, 0, 255)
    return out


def resample_with_taps(img_u8: np.ndarray, taps_x: np.ndarray, taps_y: np.ndarray) -> np.ndarray:
    h = _pass(img_u8.transpose(1, 0, 2), taps_x).transpose(1, 0, 2)   # along W first
    return _pass(h, taps_y)
