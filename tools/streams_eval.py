"""Eval chain on one HIP stream vs the batch split over two streams, launched (a) one half's
whole chain then the other's, (b) layer-interleaved (A1 B1 A2 B2 ...), in the bf16 and x6
modes (diagnostic, GPU). One box, interleaved rounds.

    python tools/streams_eval.py [--batch 64] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=3)
args = ap.parse_args()
dev = torch.device("cuda:0")
N = 192
net = ImageCompressor(N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
B = args.batch
x = torch.from_numpy(synth.to_unit_float(synth.image_u8(1000, B, 256, 256))).to(dev)
enc, dec = net.Encoder, net.Decoder
gd = (enc.gdn1, enc.gdn2, dec.igdn1, dec.igdn2)
rate, rtab = net.bitEstimator.packed(), net.bitEstimator.rate_table()


def layers_bf16(xb):
    """generator: one layer launched per next()"""
    (w1b, w2b, w3b), (d1b, d2b, d3b) = enc.packed_bf16(), dec.packed_bf16()
    e1, e2, e3, e4 = (m.effective_params_bf16() for m in gd)
    h = kernels.conv1_gdn_bf16(xb, w1b, enc.conv1.bias, *e1, N); yield
    h = kernels.conv2_gdn_bf16(h, w2b, enc.conv2.bias, *e2); yield
    _, partial, _, ybf = kernels.conv3_quant_rate_bf16(h, w3b, rate, rtab); yield
    h = kernels.deconv_igdn_bf16(ybf, d1b, dec.deconv1.bias, *e3); yield
    h = kernels.deconv_igdn_bf16(h, d2b, dec.deconv2.bias, *e4); yield
    kernels.deconv3_bf16(h, d3b, dec.deconv3.bias); yield
    kernels.reduce_partials(partial, 1.0, per_image=False); yield


def layers_x6(xb):
    w1, w2, w3, _, _ = enc.packed()
    d1, d2, _, _, _ = dec.packed()
    e1, e2, e3, e4 = (m.effective_params_x6() for m in gd)
    hs, _, _ = kernels.conv1x6_gdn(xb, enc.packed_conv1_x6(), enc.conv1.bias, e1[0], e1[2], N); yield
    hs, _, _ = kernels.conv2_gdn_x6(hs, w2, enc.conv2.bias, *e2); yield
    _, partial, _, ys = kernels.conv3_quant_rate_x6(hs, w3, rate, rtab=rtab); yield
    hs, _, _ = kernels.deconv_igdn_x6(ys, d1, dec.deconv1.bias, *e3); yield
    hs, _, _ = kernels.deconv_igdn_x6(hs, d2, dec.deconv2.bias, *e4, chunk_major=True); yield
    kernels.deconv3_x6(hs, dec.packed_x6(), dec.deconv3.bias); yield
    kernels.reduce_partials(partial, 1.0, per_image=False); yield


side = torch.cuda.Stream(device=dev)
halves = [x[: B // 2].contiguous(), x[B // 2:].contiguous()]


def one(layers):
    for _ in layers(x):
        pass


def two_seq(layers):
    main = torch.cuda.current_stream(dev)
    side.wait_stream(main)
    for _ in layers(halves[0]):
        pass
    with torch.cuda.stream(side):
        for _ in layers(halves[1]):
            pass
    main.wait_stream(side)


def two_inter(layers):
    main = torch.cuda.current_stream(dev)
    side.wait_stream(main)
    ga, gb = layers(halves[0]), layers(halves[1])
    for _ in range(7):
        next(ga)
        with torch.cuda.stream(side):
            next(gb)
    main.wait_stream(side)


def timeit(fn, layers):
    with torch.no_grad():
        for _ in range(5):
            fn(layers)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn(layers)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3


for prec, layers in (("bf16", layers_bf16), ("x6", layers_x6)):
    for r in range(args.rounds):
        res = {n: timeit(f, layers) for n, f in (("one", one), ("two_seq", two_seq), ("two_inter", two_inter))}
        print(prec, f"B={B}", " ".join(f"{n} {t:.4f} ms ({B * 65536 / t / 1e3:.0f} Mpix/s)" for n, t in res.items()), flush=True)
