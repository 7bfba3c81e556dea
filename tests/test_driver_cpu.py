"""Host-side pieces of the training driver (train.py surface): config keys, LR schedule,
gradient clamp, meters, synthetic data stream."""
import json

import torch

from iclr_17_compression_amd import train


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


def test_synthetic_stream():
    s = train.ImageDirStream("", 256, 2, 0, synthetic=True)
    a, b = next(s), next(s)
    assert a.shape == (2, 3, 256, 256) and a.dtype == torch.float32
    assert 0.0 <= a.min() and a.max() <= 1.0 and not torch.equal(a, b)
