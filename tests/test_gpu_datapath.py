"""GPU training transform (iclr17_resized_crop_batch) against the reference's PIL path
(oracle/datapath_ref.pil_transform: crop → resize BILINEAR → flips → ToTensor), bit for bit."""
import os

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


def _png_dir(tmp_path, n, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    paths = []
    for i in range(n):
        H, W = int(rng.integers(180, 520)), int(rng.integers(180, 520))
        p = tmp_path / f"img{i:03d}.png"
        Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(p)
        paths.append(str(p))
    return paths


@pytest.mark.parametrize("cache", [True, False])
def test_train_loader_matches_pil(device, tmp_path, cache):
    """TrainLoader — HBM-resident decoded images (cache) or streamed worker crops, the upload
    and GPU resampling on a side stream one batch ahead — gives, batch for batch, the
    reference's PIL transform of the planned images with the planned random choices."""
    paths = _png_dir(tmp_path, 11)
    ld = data.TrainLoader(paths, 4, 256, 3, device, workers=2, prefetch=2, cache=cache)
    assert (ld.store is not None) == cache
    try:
        for epoch in (0, 1):
            plan = list(ld._jobs(epoch))
            got = list(ld.epoch(epoch))
            assert [g.shape[0] for g in got] == [len(b) for b in plan] == [4, 4, 3]
            for g, jobs in zip(got, plan):
                g = g.cpu().numpy()
                for k, (i, seed) in enumerate(jobs):
                    img = data._decode(paths[i])
                    box, flips = data._draw(seed, img.shape[0], img.shape[1])
                    ref = datapath_ref.pil_transform(img, box, flips, 256)
                    assert np.array_equal(g[k], ref), (epoch, paths[i])
    finally:
        ld.close()


def test_train_driver_epochs(device, tmp_path, caplog):
    """train.main on an image directory: the epoch loop (train.py:249-260), the "Epoch N" log
    field, per-epoch learning rate and the checkpoint saves."""
    import json
    import logging
    from iclr_17_compression_amd import train
    d = tmp_path / "imgs"
    d.mkdir()
    _png_dir(d, 6)
    cfg = tmp_path / "cfg.json"
    cfg.write_text(json.dumps({"batch_size": 2, "print_freq": 1, "cal_step": 1,
                               "out_channel_N": 128, "train_lambda": 256}))
    caplog.set_level(logging.INFO, logger="ImageCompression")
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        assert train.main(["--config", str(cfg), "--train-dir", str(d), "--max-steps", "5",
                           "--workers", "2", "-n", "t"]) == 0
    finally:
        os.chdir(cwd)
    text = caplog.text
    assert "Epoch 0 begin" in text and "Epoch 1 begin" in text
    assert "| Epoch 0 |" in text and "| Epoch 1 |" in text and "Step [5/5" in text
    assert sorted(os.listdir(tmp_path / "checkpoints" / "t"))
