"""Training data path — datasets.py:14-37 (``Datasets``: RandomResizedCrop(256),
RandomHorizontalFlip, RandomVerticalFlip, ToTensor) with the pixel work on the GPU.

The host decodes images to uint8 RGB (PIL, as the reference does) and makes the random
choices; ``iclr17_resized_crop_batch`` (csrc/datapath.hip) resamples, flips and converts on the
device, from uint8 uploads. The random choices follow torchvision's algorithms on numpy's RNG
(the reference's torch RNG stream itself is not reproduced, only its distribution); the pixel
arithmetic is PIL's 8-bit bilinear resampling and equals the reference's PIL path bit for bit.
"""
from __future__ import annotations

import functools
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


@functools.lru_cache(maxsize=8192)
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
    offsets, shapes, off = [], [], 0
    for img in images:
        if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
            raise Iclr17Error("iclr17: images must be uint8 HxWx3")
        offsets.append(off)
        shapes.append(img.shape[:2])
        off += img.size
    src = torch.from_numpy(np.concatenate([np.ascontiguousarray(i).ravel() for i in images]))
    src = src.pin_memory().to(device, non_blocking=True)
    return resized_crop_device(src, offsets, shapes, boxes, flips, size, device)


def resized_crop_device(src: torch.Tensor, offsets, shapes, boxes, flips, size: int,
                        device: torch.device) -> torch.Tensor:
    """The same transform on images already in device memory: ``src`` a uint8 buffer holding
    image b (HWC RGB, shapes[b] = (H, W)) at byte offset offsets[b]."""
    B = len(offsets)
    if B == 0 or not (len(shapes) == len(boxes) == len(flips) == B):
        raise Iclr17Error("iclr17: resized_crop needs one shape, box and flip pair per image")
    desc = np.zeros((B, 16), dtype=np.int64)
    tap_rows: List[np.ndarray] = []
    tmp_off = tap_off = 0
    for b, (o, (H, W), (ci, cj, ch, cw), (fh, fv)) in enumerate(zip(offsets, shapes, boxes, flips)):
        if not (0 <= ci and 0 <= cj and ch > 0 and cw > 0 and ci + ch <= H and cj + cw <= W):
            raise Iclr17Error(f"iclr17: crop box {(ci, cj, ch, cw)} outside a {H}x{W} image")
        if o < 0 or o + H * W * 3 > src.numel():
            raise Iclr17Error("iclr17: image outside the source buffer")
        tx, kx = pil_bilinear_taps(cw, size)
        ty, ky = pil_bilinear_taps(ch, size)
        desc[b] = (o, H, W, ci, cj, ch, cw, int(bool(fh)), int(bool(fv)), tmp_off,
                   tap_off, kx, tap_off + tx.size, ky, 0, 0)
        tap_rows += [tx.ravel(), ty.ravel()]
        tap_off += tx.size + ty.size
        tmp_off += ch * size * 3
    taps = torch.from_numpy(np.concatenate(tap_rows)).pin_memory().to(device, non_blocking=True)
    d = torch.from_numpy(desc).pin_memory().to(device, non_blocking=True)
    tmp = torch.empty(tmp_off, dtype=torch.uint8, device=device)
    out = torch.empty(B, 3, size, size, dtype=torch.float32, device=device)
    max_ch = int(desc[:, 5].max())
    call("iclr17_resized_crop_batch", kernels._p(src), kernels._p(d), B, size, max_ch,
         kernels._p(taps), kernels._p(tmp), kernels._p(out), kernels._stream(out))
    return out


# --------------------------------------------------------------------------- loader
def _draw(seed, H: int, W: int):
    """The random choices of one sample (RandomResizedCrop box, then the h / v flips), from a
    seed fixed by (loader seed, epoch, position) — independent of which process draws them."""
    rng = np.random.default_rng(seed)
    box = random_resized_crop_params(rng, H, W)
    return box, (bool(rng.random() < 0.5), bool(rng.random() < 0.5))


def _decode(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8)   # datasets.py:29


def _decode_crop(job):
    """Worker: decode one image, draw its choices and cut the box out (crop-then-resize is what
    torchvision's resized_crop does, so resampling the cut box is exact)."""
    path, seed = job
    img = _decode(path)
    (top, left, h, w), flips = _draw(seed, img.shape[0], img.shape[1])
    return np.ascontiguousarray(img[top:top + h, left:left + w]), flips


def _image_size(path):
    from PIL import Image
    with Image.open(path) as im:   # header only
        return im.size[1], im.size[0]


class TrainLoader:
    """Epochs of training batches from an image directory — the reference's
    DataLoader(Datasets(dir, 256), batch_size, shuffle=True, pin_memory=True, num_workers=1)
    (train.py:243-249, datasets.py:14-37), re-built for a GPU that consumes a batch in a few ms.

    Each epoch is a permutation of the images; a global batch of ``batch × world`` images is
    split contiguously over the ranks (rank r takes its slice of every global batch); the last,
    partial global batch is dropped when world > 1 so every rank runs the same step count. Each
    sample's random choices come from a seed fixed by (seed, epoch, position).

    Two sources:
    * resident (``cache``, when the decoded set fits ``cache_bytes``): the uint8 images are
      decoded once, by a pool of worker processes, into one HBM buffer (a photo set of a few GB
      is small next to 288 GB); every batch is then crop + resample + flips on the GPU from
      HBM — no host decode, no PCIe traffic after the first epoch;
    * streamed: the workers decode and cut each sample's box, the boxes go up from pinned
      memory, ``prefetch`` batches in flight.
    Either way the upload and resampling run on a side HIP stream one batch ahead of the
    training stream, which waits on an event only when it takes the batch.
    """

    def __init__(self, paths: Sequence[str], batch: int, size: int, seed: int, device,
                 rank: int = 0, world: int = 1, workers: int = 4, prefetch: int = 4,
                 cache: bool = True, cache_bytes: int = 64 << 30):
        if not paths:
            raise FileNotFoundError("TrainLoader: no images")
        if world > 1 and len(paths) < batch * world:
            # every rank runs the same step count, and a partial global batch is dropped: fewer
            # images than one global batch would give zero steps per epoch
            raise ValueError(f"TrainLoader: {len(paths)} images are fewer than one global batch "
                             f"({batch} x {world} ranks)")
        self.paths, self.batch, self.size, self.seed = list(paths), batch, size, seed
        self.device, self.rank, self.world = device, rank, world
        self.prefetch = max(1, prefetch)
        self.timeout = 120.0   # s per decode: a lost worker result raises instead of hanging
        import multiprocessing as mp
        self.pool = mp.get_context("spawn").Pool(workers) if workers > 0 else None
        self.stream = torch.cuda.Stream(device=device)
        self.store = None
        if cache:
            shapes = (self.pool.map(_image_size, self.paths, chunksize=16) if self.pool
                      else [_image_size(p) for p in self.paths])
            nbytes = [h * w * 3 for h, w in shapes]
            if sum(nbytes) <= cache_bytes:
                self.shapes = shapes
                self.offsets = np.concatenate([[0], np.cumsum(nbytes)[:-1]]).astype(np.int64).tolist()
                self.store = torch.empty(sum(nbytes), dtype=torch.uint8, device=device)
                self.cached = np.zeros(len(self.paths), dtype=bool)

    def steps_per_epoch(self) -> int:
        gb = self.batch * self.world
        n = len(self.paths)
        return n // gb if self.world > 1 else (n + gb - 1) // gb

    def _jobs(self, epoch: int):
        perm = np.random.default_rng([self.seed, epoch]).permutation(len(self.paths))
        gb = self.batch * self.world
        for s in range(self.steps_per_epoch()):
            pos = np.arange(s * gb, min((s + 1) * gb, len(perm)))
            lo = self.rank * self.batch
            mine = pos[lo:lo + self.batch] if self.world > 1 else pos
            yield [(int(perm[p]), (self.seed, epoch, int(p))) for p in mine]

    # one batch: host work submitted (returns a handle), then staged on the device
    def _submit(self, jobs):
        if self.store is not None:
            todo = [i for i, _ in jobs if not self.cached[i]]
            fut = ({i: self.pool.apply_async(_decode, (self.paths[i],)) for i in todo}
                   if self.pool else {i: _decode(self.paths[i]) for i in todo})
            return jobs, fut
        crops = [(self.paths[i], seed) for i, seed in jobs]
        if self.pool is None:
            return jobs, [_decode_crop(j) for j in crops]
        return jobs, [self.pool.apply_async(_decode_crop, (j,)) for j in crops]

    def _stage(self, handle):
        jobs, fut = handle
        with torch.cuda.stream(self.stream):
            if self.store is not None:
                for i, r in fut.items():
                    if self.cached[i]:
                        continue
                    img = r if isinstance(r, np.ndarray) else r.get(timeout=self.timeout)
                    if img.shape[:2] != tuple(self.shapes[i]):
                        raise Iclr17Error(f"TrainLoader: {self.paths[i]} changed size")
                    o = self.offsets[i]
                    self.store[o:o + img.size].copy_(torch.from_numpy(img.ravel()).pin_memory(),
                                                     non_blocking=True)
                    self.cached[i] = True
                boxes, flips = zip(*(_draw(seed, *self.shapes[i]) for i, seed in jobs))
                out = resized_crop_device(self.store, [self.offsets[i] for i, _ in jobs],
                                          [self.shapes[i] for i, _ in jobs], boxes, flips,
                                          self.size, self.device)
            else:
                items = [r if isinstance(r, tuple) else r.get(timeout=self.timeout) for r in fut]
                imgs = [a for a, _ in items]
                out = resized_crop_batch(imgs, [(0, 0, a.shape[0], a.shape[1]) for a in imgs],
                                         [f for _, f in items], self.size, self.device)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return out, ev

    def epoch(self, epoch: int):
        """Iterator over this rank's batches of one epoch: NCHW fp32 [b, 3, size, size] on the
        device, ready on the current stream."""
        from collections import deque
        jobs = self._jobs(epoch)
        host = deque()
        for j in jobs:
            host.append(self._submit(j))
            if len(host) >= self.prefetch:
                break
        staged = None
        while host or staged is not None:
            if staged is None:
                staged = self._stage(host.popleft())
                j = next(jobs, None)
                if j is not None:
                    host.append(self._submit(j))
            cur, staged = staged, None
            if host:   # stage the next batch before the caller queues its step on `cur`
                staged = self._stage(host.popleft())
                j = next(jobs, None)
                if j is not None:
                    host.append(self._submit(j))
            out, ev = cur
            main = torch.cuda.current_stream(self.device)
            main.wait_event(ev)
            out.record_stream(main)
            yield out

    def close(self):
        if self.pool is not None:
            self.pool.terminate()
            self.pool.join()
            self.pool = None
