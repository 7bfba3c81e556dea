"""The drop-in surface: class names, constructor signatures, parameter names,
shapes and init distributions, checkpoint I/O — all host-side, no GPU needed."""
import math
import os

import numpy as np
import pytest
import torch

from iclr_17_compression_amd import synth
from iclr_17_compression_amd.model import ImageCompressor, load_model, save_model
from iclr_17_compression_amd.models import (GDN, Analysis_net_17, BitEstimator, Bitparm,
                                            LowerBound, Synthesis_net_17)


@pytest.mark.parametrize("N", [128, 192])
def test_state_dict_keys_and_shapes(N):
    net = ImageCompressor(out_channel_N=N)
    sd = net.state_dict()
    assert list(sd.keys()) == list(synth.STATE_DICT_KEYS)
    ref = synth.trained_like_state_dict(N, 1)
    for k, v in sd.items():
        assert tuple(v.shape) == ref[k].shape, k
        assert v.dtype == torch.float32


def test_defaults_match_reference():
    assert ImageCompressor().out_channel_N == 128          # model.py:39
    assert Analysis_net_17().conv1.out_channels == 192     # analysis_17.py:12
    assert Synthesis_net_17().deconv3.out_channels == 3
    assert Analysis_net_17().conv3.bias is None
    assert Bitparm(8, final=True).a is None


def test_init_distributions():
    torch.manual_seed(0)
    a = Analysis_net_17(192)
    N = 192
    fan = 3 * 81 + N * 81
    std = math.sqrt(2 * (3 + N) / 6) * math.sqrt(2.0 / fan)
    assert a.conv1.weight.std().item() == pytest.approx(std, rel=0.05)
    assert torch.all(a.conv1.bias == 0.01)
    g = GDN(16)
    beta_eff = LowerBound.apply(g.beta, g.beta_bound) ** 2 - g.pedestal
    assert torch.allclose(beta_eff, torch.ones(16))
    gamma_eff = LowerBound.apply(g.gamma, g.gamma_bound) ** 2 - g.pedestal
    assert torch.equal(gamma_eff - torch.diag(torch.diagonal(gamma_eff)), torch.zeros(16, 16))


def test_lower_bound_gradient_rule():
    x = torch.tensor([-1.0, 0.5, 2.0], requires_grad=True)
    y = LowerBound.apply(x, 1.0)
    y.backward(torch.tensor([1.0, -1.0, 1.0]))
    assert torch.equal(x.grad, torch.tensor([0.0, -1.0, 1.0]))


def test_checkpoint_roundtrip(tmp_path):
    net = ImageCompressor(128)
    sd = {k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(128, 3).items()}
    net.load_state_dict(sd)
    save_model(net, 7, str(tmp_path))
    assert os.path.exists(tmp_path / "iter_7.pth.tar")
    other = ImageCompressor(128)
    assert load_model(other, str(tmp_path / "iter_7.pth.tar")) == 0
    for k, v in other.state_dict().items():
        assert torch.equal(v, sd[k])


def test_star_imports_give_train_py_names():
    """train.py:3 does `from model import *` and then uses ImageCompressor, save_model,
    load_model, np, torch, logging and ms_ssim (train.py:26,117,178) without importing them;
    `from models import *` yields the reference's models/__init__.py:1-9 names."""
    ns = {}
    exec("from iclr_17_compression_amd.model import *", ns)
    for name in ("ImageCompressor", "save_model", "load_model", "np", "torch", "logging",
                 "ms_ssim", "ssim", "GDN", "BitEstimator", "Analysis_net_17", "Synthesis_net_17"):
        assert name in ns, name
    ns = {}
    exec("from iclr_17_compression_amd.models import *", ns)
    for name in ("GDN", "BitEstimator", "Analysis_net_17", "Synthesis_net_17", "ms_ssim", "ssim"):
        assert name in ns, name


def test_ms_ssim_argument_checks_and_no_cpu_fallback():
    """The reference's ValueError checks (ms_ssim_torch.py:140-150) come first; CPU tensors go to
    the GPU kernels, so on a host without a GPU the call fails loudly instead of computing on CPU."""
    from iclr_17_compression_amd._lib import Iclr17Error
    from iclr_17_compression_amd.models import ms_ssim, ssim
    x = torch.rand(1, 3, 176, 176)
    with pytest.raises(ValueError, match="4-d"):
        ms_ssim(x[0], x[0], data_range=1.0)
    with pytest.raises(ValueError, match="same dimensions"):
        ms_ssim(x, x[:, :, :170], data_range=1.0)
    with pytest.raises(ValueError, match="odd"):
        ssim(x, x, win_size=10)
    with pytest.raises(Iclr17Error, match="default window"):
        ms_ssim(x, x, win_sigma=2.0)
    with pytest.raises(Iclr17Error, match="weights"):
        ms_ssim(x, x, weights=[0.5, 0.5])
    if not torch.cuda.is_available():
        with pytest.raises(Iclr17Error, match="no CPU implementation"):
            ms_ssim(x, x, data_range=1.0, size_average=True)


def test_ms_ssim_refuses_a_backward_it_cannot_give():
    """The GPU MS-SSIM has no backward: an input that requires grad raises (a loss such as
    λ·(1 − ms_ssim) + bpp would otherwise silently drop that term's gradient); under no_grad or
    on detached tensors the call proceeds (here to the no-GPU error on a CPU host)."""
    from iclr_17_compression_amd._lib import Iclr17Error
    from iclr_17_compression_amd.models import ms_ssim, ssim
    from iclr_17_compression_amd.models.ms_ssim_torch import MS_SSIM
    x = torch.rand(1, 3, 176, 176, requires_grad=True)
    y = torch.rand(1, 3, 176, 176)
    for fn in (lambda: ms_ssim(x, y, data_range=1.0), lambda: ssim(y, x, data_range=1.0),
               lambda: MS_SSIM(data_range=1.0)(x, y)):
        with pytest.raises(Iclr17Error, match="no backward"):
            fn()
    if not torch.cuda.is_available():
        with torch.no_grad(), pytest.raises(Iclr17Error, match="no CPU implementation"):
            ms_ssim(x, y, data_range=1.0)


def test_train_loader_refuses_fewer_images_than_a_global_batch(tmp_path):
    from iclr_17_compression_amd import data
    with pytest.raises(ValueError, match="global batch"):
        data.TrainLoader([str(tmp_path / "a.png")] * 3, 2, 64, 0, "cpu", rank=0, world=2, workers=0)


def test_grad_reducer_refuses_a_held_gradient():
    """GradAllReducer.launch: a parameter whose .grad already holds another value (no
    set_to_none zero_grad, gradient accumulation) would lose it in finish(): it raises."""
    from iclr_17_compression_amd import dist as idist
    p = torch.nn.Parameter(torch.zeros(4))
    p.grad = torch.ones(4)
    red = idist.GradAllReducer([p])
    with pytest.raises(RuntimeError, match="already holds"):
        red.launch([p], [torch.full((4,), 2.0)])
