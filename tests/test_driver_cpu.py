"""Host-side pieces of the training driver (train.py surface): config keys, LR schedule,
gradient clamp, meters, synthetic data stream."""
import json

import numpy as np
import torch

from iclr_17_compression_amd import data, train


def test_parse_config_keys(tmp_path):
    p = tmp_path / "c.json"
    p.write_text(json.dumps({"train_lambda": 512, "batch_size": 8, "lr": {"base": 2e-4, "decay_interval": 10}}))
    cfg = train.parse_config(str(p))
    assert cfg["train_lambda"] == 512 and cfg["batch_size"] == 8
    assert cfg["lr"] == {"base": 2e-4, "decay": 0.1, "decay_interval": 10}
    assert cfg["tot_step"] == 2500000 and cfg["cal_step"] == 40   # train.py:15-29 defaults


def test_learning_rate_schedule():
    cfg = train.parse_config("")
    cfg["lr"] = {"base": 1e-4, "decay": 0.1, "decay_interval": 100}
    assert train.learning_rate(cfg, 0) == 1e-4
    assert train.learning_rate(cfg, 99) == 1e-4
    assert abs(train.learning_rate(cfg, 100) - 1e-5) < 1e-12


def test_clip_gradient():
    p = torch.nn.Parameter(torch.zeros(4))
    p.grad = torch.tensor([-9.0, -1.0, 2.0, 7.0])
    train.clip_gradient([p], 5)
    assert torch.equal(p.grad, torch.tensor([-5.0, -1.0, 2.0, 5.0]))


def test_meter_window():
    m = train.AverageMeter(2)
    for v in (1.0, 2.0, 4.0):
        m.update(v)
    assert m.val == 4.0 and m.avg == 3.0


def test_synthetic_loader_epochs():
    ld = train.SyntheticLoader(2, 64, 0, "cpu", images=8)
    assert ld.steps_per_epoch() == 4
    e0, e1 = list(ld.epoch(0)), list(ld.epoch(1))
    assert len(e0) == 4 and e0[0].shape == (2, 3, 64, 64) and e0[0].dtype == torch.float32
    assert 0.0 <= e0[0].min() and e0[0].max() <= 1.0
    assert not torch.equal(e0[0], e0[1]) and not torch.equal(e0[0], e1[0])
    assert torch.equal(e0[2], list(ld.epoch(0))[2])   # an epoch is reproducible


def _pngs(tmp_path, n, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    paths = []
    for i in range(n):
        H, W = int(rng.integers(200, 400)), int(rng.integers(200, 400))
        p = tmp_path / f"img{i:03d}.png"
        Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(p)
        paths.append(str(p))
    return paths


def test_train_loader_epoch_plan(tmp_path):
    """Shuffled epochs, contiguous per-rank slices of each global batch, seeds fixed by
    (seed, epoch, position), drop_last only with several ranks (DataLoader(shuffle=True))."""
    paths = [f"p{i}" for i in range(10)]
    one = data.TrainLoader.__new__(data.TrainLoader)
    one.paths, one.batch, one.seed, one.rank, one.world = paths, 4, 7, 0, 1
    plan = list(one._jobs(0))
    assert [len(b) for b in plan] == [4, 4, 2] and one.steps_per_epoch() == 3
    assert sorted(i for b in plan for i, _ in b) == list(range(10))     # each image once
    assert [j for b in plan for j in b] == [j for b in one._jobs(0) for j in b]
    assert [i for b in one._jobs(1) for i, _ in b] != [i for b in plan for i, _ in b]
    ranks = []
    for r in range(2):
        ld = data.TrainLoader.__new__(data.TrainLoader)
        ld.paths, ld.batch, ld.seed, ld.rank, ld.world = paths, 2, 7, r, 2
        ranks.append(list(ld._jobs(0)))
        assert ld.steps_per_epoch() == 2
    both = [ranks[0][s] + ranks[1][s] for s in range(2)]
    assert [j for b in both for j in b] == [j for b in plan[:2] for j in b]   # same order


def test_decode_crop_worker(tmp_path):
    from PIL import Image
    p = _pngs(tmp_path, 1)[0]
    img = np.asarray(Image.open(p).convert("RGB"))
    box_img, flips = data._decode_crop((p, (3, 0, 5)))
    rng = np.random.default_rng((3, 0, 5))
    t, l, h, w = data.random_resized_crop_params(rng, img.shape[0], img.shape[1])
    assert np.array_equal(box_img, img[t:t + h, l:l + w])
    assert flips == (bool(rng.random() < 0.5), bool(rng.random() < 0.5))
