"""GPU training transform (iclr17_resized_crop_batch) against the reference's PIL path
(oracle/datapath_ref.pil_transform: crop → resize BILINEAR → flips → ToTensor), bit for bit."""
import numpy as np
import pytest
import torch

from iclr_17_compression_amd import data
from oracle import datapath_ref

pytestmark = pytest.mark.gpu


def test_resized_crop_batch_matches_pil(device):
    rng = np.random.default_rng(5)
    imgs, boxes, flips = [], [], []
    for H, W in [(512, 768), (768, 512), (300, 200), (1000, 1500), (256, 256), (200, 900)]:
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        for _ in range(2):
            imgs.append(img)
            boxes.append(data.random_resized_crop_params(rng, H, W))
            flips.append((bool(rng.random() < 0.5), bool(rng.random() < 0.5)))
    out = data.resized_crop_batch(imgs, boxes, flips, 256, device).cpu().numpy()
    for b in range(len(imgs)):
        ref = datapath_ref.pil_transform(imgs[b], boxes[b], flips[b], 256)
        assert np.array_equal(out[b], ref), (b, boxes[b], flips[b])


def test_resized_crop_batch_rejects_bad_boxes(device):
    from iclr_17_compression_amd._lib import Iclr17Error
    img = np.zeros((100, 100, 3), np.uint8)
    with pytest.raises(Iclr17Error, match="outside"):
        data.resized_crop_batch([img], [(50, 50, 60, 10)], [(False, False)], 256, device)
