"""Diagnostic (GPU): how far each summation order's latents y lie from the exact value, on the
G8 / G9 operating points (24 Kodak-synth images, trained weights).

Per image: y64 = the analysis transform (analysis_17.py:31-36) in float64 on the GPU (ATen's
native conv, MIOpen off), y_ref = the oracle in fp32 on the CPU (the reference's default oneDNN
order, = the G8 / G9 fixtures), and the GPU kernels' y in the x6 and exact-f32 modes. Reports
max / rms |y − y64| of each and flip counts: round(y) vs round(y64) and vs round(y_ref). Then, per
layer, each layer's error alone: the same fp32 input (the fp64 chain rounded) through the GPU x6
kernel, the GPU fp32 kernel and the CPU fp32 op, against fp64.

    python tools/latent_accuracy.py [--set g9] [--images 24] > out.json
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402
from oracle import codec_ref as oracle  # noqa: E402

SETS = {"g8": "g8_kodak24_synth_n128_trained.json", "g9": "g9_kodak24_synth_n192_trained.json"}


def stats(a, ref):
    d = (a.double() - ref).abs()
    return {"max": d.max().item(), "rms": d.pow(2).mean().sqrt().item()}


def flips(a, b):
    return int((torch.round(a.double()) != torch.round(b.double())).sum().item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="g9")
    ap.add_argument("--images", type=int, default=24)
    args = ap.parse_args()
    torch.backends.cudnn.enabled = False   # fp64 convs through ATen's native GPU kernels
    dev = torch.device("cuda:0")
    meta = json.load(open(os.path.join(REPO, "tests", "golden", SETS[args.set])))
    d = np.load(os.path.join(REPO, "tests", "golden", meta["weights"]))
    sd = {k: torch.from_numpy(d[k].astype(np.float32)) for k in d.files}
    sd64 = {k: v.double().to(dev) for k, v in sd.items()}
    net = ImageCompressor(out_channel_N=meta["N"])
    net.load_state_dict(sd)
    net = net.to(dev).eval()
    out = {"set": args.set, "N": meta["N"], "images": []}
    tot = {}
    for row in meta["images"][: args.images]:
        x = torch.from_numpy(synth.to_unit_float(synth.smooth_image_u8(
            meta["image_seed_base"] + row["index"], row["height"], row["width"])))[None]
        with torch.no_grad():
            y64 = oracle.analysis(x.double().to(dev), sd64).cpu()
            yref = oracle.analysis(x, sd)
            r = {"index": row["index"], "ref_cpu_fp32": {**stats(yref, y64), "flips_vs_exact": flips(yref, y64)}}
            for mode in ("x6", "fp32"):
                kernels.set_precision(mode)
                ev = net.evaluate(x.to(dev), want_y=True)
                y = ev["y"].cpu().contiguous()
                r[mode] = {**stats(y, y64), "flips_vs_exact": flips(y, y64), "flips_vs_ref": flips(y, yref)}
        for k in ("ref_cpu_fp32", "x6", "fp32"):
            for f in ("flips_vs_exact", "flips_vs_ref"):
                if f in r[k]:
                    tot[f"{k}.{f}"] = tot.get(f"{k}.{f}", 0) + r[k][f]
        out["images"].append(r)
        print(json.dumps(r), file=sys.stderr, flush=True)
    out["totals"] = tot
    kernels.set_precision("x6")
    out["layers"] = per_layer(net, sd, sd64, meta, dev)
    print(json.dumps(out))


def per_layer(net, sd, sd64, meta, dev):
    """Each analysis layer alone on one 256×256 crop of image 0: the same fp32 input through the
    x6 kernel, the fp32 kernel and the CPU oneDNN op, each against fp64 of that input."""
    row = meta["images"][0]
    x = torch.from_numpy(synth.to_unit_float(synth.smooth_image_u8(
        meta["image_seed_base"] + row["index"], row["height"], row["width"])))[None][:, :, :256, :256]
    xd = x.to(dev)
    N = meta["N"]
    enc = net.Encoder
    w1, w2, w3, g1, g2 = enc.packed()
    e1, e2 = enc.gdn1.effective_params_x6(), enc.gdn2.effective_params_x6()
    w1x6 = enc.packed_conv1_x6()
    rate = net.bitEstimator.packed()
    P = "Encoder."

    def gdn64(h, i):
        return oracle.gdn(h, sd64[f"{P}gdn{i}.beta"], sd64[f"{P}gdn{i}.gamma"], False)

    def gdn32(h, i):
        return oracle.gdn(h, sd[f"{P}gdn{i}.beta"], sd[f"{P}gdn{i}.gamma"], False)

    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous()   # noqa: E731
    nchw = lambda t: t.permute(0, 3, 1, 2).contiguous()   # noqa: E731
    res = {}
    with torch.no_grad():
        # conv1 + GDN1
        c64 = F.conv2d(x.double().to(dev), sd64[P + "conv1.weight"], sd64[P + "conv1.bias"], 4, 4)
        h64 = gdn64(c64, 1)
        _, x6o, x6p = kernels.conv1x6_gdn(xd, w1x6, enc.conv1.bias, e1[0], e1[2], N, want_f32=True, want_pre=True)
        f32o, f32p = kernels.conv1_gdn(xd, w1, enc.conv1.bias, g1[0], g1[1], N, want_pre=True)
        c32 = F.conv2d(x, sd[P + "conv1.weight"], sd[P + "conv1.bias"], 4, 4)
        res["conv1"] = {"x6": stats(nchw(x6p).cpu(), c64.cpu()), "fp32": stats(nchw(f32p).cpu(), c64.cpu()),
                        "cpu": stats(c32, c64.cpu())}
        res["conv1+gdn1"] = {"x6": stats(nchw(x6o).cpu(), h64.cpu()), "fp32": stats(nchw(f32o).cpu(), h64.cpu()),
                             "cpu": stats(gdn32(c32, 1), h64.cpu())}
        # conv2 + GDN2 on the fp64 chain rounded to fp32
        h1 = h64.float()
        c64 = F.conv2d(h1.double(), sd64[P + "conv2.weight"], sd64[P + "conv2.bias"], 2, 2)
        h64 = gdn64(c64, 2)
        _, x6o, x6p = kernels.conv2_gdn_x6(kernels.split_planes(nhwc(h1)), w2, enc.conv2.bias, *e2,
                                           want_f32=True, want_pre=True)
        f32o, f32p = kernels.conv2_gdn(nhwc(h1), w2, enc.conv2.bias, g2[0], g2[1], want_pre=True)
        c32 = F.conv2d(h1.cpu(), sd[P + "conv2.weight"], sd[P + "conv2.bias"], 2, 2)
        res["conv2"] = {"x6": stats(nchw(x6p).cpu(), c64.cpu()), "fp32": stats(nchw(f32p).cpu(), c64.cpu()),
                        "cpu": stats(c32, c64.cpu())}
        res["conv2+gdn2"] = {"x6": stats(nchw(x6o).cpu(), h64.cpu()), "fp32": stats(nchw(f32o).cpu(), h64.cpu()),
                             "cpu": stats(gdn32(c32, 2), h64.cpu())}
        # conv3 (y)
        h2 = h64.float()
        y64 = F.conv2d(h2.double(), sd64[P + "conv3.weight"], None, 2, 2)
        _, _, yx6, _ = kernels.conv3_quant_rate_x6(kernels.split_planes(nhwc(h2)), w3, rate, want_y=True)
        _, _, yf32 = kernels.conv3_quant_rate(nhwc(h2), w3, rate, want_y=True)
        y32 = F.conv2d(h2.cpu(), sd[P + "conv3.weight"], None, 2, 2)
        res["conv3"] = {"x6": stats(nchw(yx6).cpu(), y64.cpu()), "fp32": stats(nchw(yf32).cpu(), y64.cpu()),
                        "cpu": stats(y32, y64.cpu())}
    return res


if __name__ == "__main__":
    main()
