"""The h3 form's range limit is loud in the product path (SURVEY §8(b) "errors are loud").

An activation of magnitude ≥ 2^22 does not fit the h3 form (two fp16 planes of x·2^-6). Every h3
kernel then sets the current stream's range flag, and the chain's last kernel (deconv3_h3) reads
it and writes every result as NaN — the reconstruction, the SSE partials, the folded bit totals —
so an out-of-range input can never pass for a result, with no host synchronisation on the way.
``evaluate(h3_overflow="raise")`` reads the flag and raises; ``h3_overflow="x6"`` reruns the batch
in the x6 mode (full fp32 operands, no range limit) and returns exactly the x6 results. The flag
is cleared at the start of every chain, so the next ordinary input is unaffected.

The out-of-range activations are made by scaling one channel's parameters: conv1's bias of
channel 0 to 1e4 with that channel's GDN row γ and β at their lower bounds (y = x/√β ≈ 1e7 at
GDN1's output), or deconv1's bias of channel 0 to 1e4 (IGDN1: y ≈ √γ·x² ≈ 3e7).
"""
import pytest
import torch

from iclr_17_compression_amd import _lib, kernels, synth
from iclr_17_compression_amd.model import ImageCompressor

pytestmark = pytest.mark.gpu


def _net(device):
    net = ImageCompressor(out_channel_N=192)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(192, 1).items()})
    return net.to(device).eval()


def _image(device):
    return torch.from_numpy(synth.to_unit_float(synth.image_u8(5, 2, 64, 96))).to(device)


@pytest.fixture
def h3():
    old = kernels.precision()
    kernels.set_precision("h3")
    yield
    kernels.set_precision(old)


def _encoder_overflow(net):
    with torch.no_grad():
        net.Encoder.conv1.bias[0] = 1e4
        net.Encoder.gdn1.gamma[0].zero_()   # γ_eff row 0 = 0 (LowerBound at 2^-18, minus the pedestal)
        net.Encoder.gdn1.beta[0] = 0.0      # β_eff = the bound, ≈ 1e-6


def _decoder_overflow(net):
    with torch.no_grad():
        net.Decoder.deconv1.bias[0] = 1e4


def _bits_equal(a, b):
    return a.dtype == b.dtype and a.shape == b.shape and torch.equal(
        a.contiguous().view(torch.uint8), b.contiguous().view(torch.uint8))


def _eval_finite(ev):
    return all(bool(torch.isfinite(ev[k]).all()) for k in ("bpp", "mse", "psnr", "clipped"))


def test_ordinary_input_no_sync_and_finite(device, h3):
    """An ordinary input runs the h3 chain with no host synchronisation (torch's sync debug mode
    raises on any synchronising op) and leaves the flag clear."""
    net = _net(device)
    x = _image(device)
    with torch.no_grad():
        net.evaluate(x)          # warm the packed layouts (their first build may read sizes)
        net(x)
        torch.cuda.synchronize()
        torch.cuda.set_sync_debug_mode("error")
        try:
            ev = net.evaluate(x)
            clipped, y_hat, bpp = net(x)
        finally:
            torch.cuda.set_sync_debug_mode("default")
    assert _eval_finite(ev) and bool(torch.isfinite(bpp)) and bool(torch.isfinite(clipped).all())
    assert not kernels.h3_range_overflowed(device)


@pytest.mark.parametrize("where", ["encoder", "decoder"])
def test_overflow_is_nan_raise_or_x6(device, h3, where):
    net = _net(device)
    x = _image(device)
    (_encoder_overflow if where == "encoder" else _decoder_overflow)(net)
    with torch.no_grad():
        ev = net.evaluate(x)                                  # default: NaN results, no sync
        assert kernels.h3_range_overflowed(device)
        for k in ("bpp", "mse", "psnr"):
            assert bool(torch.isnan(ev[k]).all()), k
        assert bool(torch.isnan(ev["clipped"]).all())
        clipped, _, bpp = net(x)                              # the module forward: NaN bpp / recon
        assert bool(torch.isnan(bpp)) and bool(torch.isnan(clipped).all())
        y = net.Encoder(x)                                    # separate encode / decode
        if where == "encoder":                                # conv3 poisons the encoder's y
            assert bool(torch.isnan(y).all())
        recon = net.Decoder(torch.round(y))
        assert bool(torch.isnan(recon).all())
        if where == "encoder":                                # compress: rANS from x6's ŷ
            comp = net.compress(x)
            kernels.set_precision("x6")
            comp_ref = net.compress(x)
            kernels.set_precision("h3")
            assert comp["strings"] == comp_ref["strings"]
        with pytest.raises(_lib.Iclr17Error, match="2\\^22"):
            net.evaluate(x, h3_overflow="raise")
        fb = net.evaluate(x, want_y=True, h3_overflow="x6")   # the x6 rerun
        kernels.set_precision("x6")
        ref = net.evaluate(x, want_y=True)
        kernels.set_precision("h3")
    assert bool(torch.isfinite(ref["bpp"]).all())
    for k in ("bpp", "mse", "psnr", "clipped", "y_hat", "y"):   # bit patterns (NaN included)
        assert _bits_equal(fb[k], ref[k]), k
    with pytest.raises(_lib.Iclr17Error, match="2\\^22"):
        kernels.check_finite("bpp", ev["bpp"])
    # the training step's loss is NaN too (the driver raises where it reads it)
    net.train()
    _, mse, bpp = net.forward_train(x)
    assert bool(torch.isnan(mse))
    # the next chain of an ordinary model starts with a clear flag
    net2 = _net(device)
    with torch.no_grad():
        ev2 = net2.evaluate(x)
    assert _eval_finite(ev2) and not kernels.h3_range_overflowed(device)


def test_near_zero_pixels_stay_finite(device, h3):
    """A pixel whose channels are all (near) zero before GDN / IGDN (zero biases on a zero image
    region) keeps a finite per-pixel scale in the h3 epilogue: no NaN, the GDN of 0 is 0."""
    net = _net(device)
    with torch.no_grad():
        net.Encoder.conv1.bias.zero_()
        net.Encoder.conv1.bias[5] = 1e-20   # the pixels' largest x² is a subnormal (1e-40)
        net.Encoder.conv2.bias.zero_()
        net.Decoder.deconv1.bias.zero_()
        net.Decoder.deconv2.bias.zero_()
        x = torch.zeros(1, 3, 64, 64, device=device)
        ev = net.evaluate(x, want_y=True)
        kernels.set_precision("x6")
        ref = net.evaluate(x, want_y=True)
        kernels.set_precision("h3")
    assert _eval_finite(ev) and not kernels.h3_range_overflowed(device)
    assert torch.equal(ev["y_hat"], ref["y_hat"])
    assert ev["bpp"].item() == pytest.approx(ref["bpp"].item(), rel=1e-5)
