"""Training data path, host side: the PIL tap tables and the crop-box sampler (CPU)."""
import numpy as np

from iclr_17_compression_amd import data
from oracle import datapath_ref


def test_pil_taps_reproduce_pil_resize():
    """data.pil_bilinear_taps + the integer two-pass restatement == PIL's resize, bit for bit,
    for down- and up-scaling and near-identity sizes."""
    rng = np.random.default_rng(0)
    for (h, w) in [(300, 400), (100, 80), (700, 500), (257, 256), (256, 256), (31, 900)]:
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        tx, _ = data.pil_bilinear_taps(w, 256)
        ty, _ = data.pil_bilinear_taps(h, 256)
        mine = datapath_ref.resample_with_taps(img, tx, ty)
        ref = (datapath_ref.pil_transform(img, (0, 0, h, w), (False, False), 256) * 255).round()
        assert np.array_equal(mine.transpose(2, 0, 1).astype(np.float32), ref), (h, w)


def test_random_resized_crop_params():
    """torchvision get_params semantics: boxes inside the image, area 8–100 %, aspect 3/4–4/3
    (up to rounding), and the centred fallback for extreme aspect ratios."""
    rng = np.random.default_rng(1)
    for _ in range(2000):
        H, W = int(rng.integers(64, 1200)), int(rng.integers(64, 1200))
        top, left, h, w = data.random_resized_crop_params(rng, H, W)
        assert 0 <= top and 0 <= left and top + h <= H and left + w <= W and h > 0 and w > 0
    # 10 000 × 10: no 3/4–4/3 box fits 8 %…100 % of the area → centred 4/3 crop of full height
    assert data.random_resized_crop_params(np.random.default_rng(2), 10, 10000) == (0, 4993, 10, 13)
