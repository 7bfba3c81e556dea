"""Commit the REFERENCE's own quantised latents for the G8 / G9 operating points.

Run in the build container (the only place /root/reference exists):

    python tests/golden/gen_yhat.py [--reference /root/reference]

For every one of the 24 Kodak-synth images of G8 (N=128) and G9 (N=192) it runs the reference
(imported with gen_goldens.import_reference's shims) in its default summation order, checks that
ŷ hashes to the ``y_hat_sha256`` the G8 / G9 fixture already holds (so these are the very
latents the fixture's bpp / PSNR / MS-SSIM come from), and stores

* ``yhat_XX``: ŷ as int8, NCHW [1, N, h, w] (model.py:56 torch.round of y; |ŷ| ≤ 127 checked;
  int8 keeps the value, not the sign of a −0);
* ``near_idx_XX`` / ``near_y_XX``: the flat indices and fp32 values of the reference's y where
  it lies within 1e-4 of a half-integer k + ½ — the only latents whose rounding any fp32
  summation order can change (the reference's own cross-order max |Δy| is 5.6e-5, g9s).

into ``g8_y_hat_n128.npz`` / ``g9_y_hat_n192.npz`` (compressed). The GPU tests count latent
flips against these arrays, not against the oracle run on the GPU box's CPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import gen_goldens as gg  # noqa: E402
from gen_goldens import KODAK_PORTRAIT, synth  # noqa: E402

NEAR = 1e-4
SETS = {"g8": (128, "g8_weights_n128.npz", "g8_kodak24_synth_n128_trained.json", "g8_y_hat_n128.npz"),
        "g9": (192, "g9_weights_n192.npz", "g9_kodak24_synth_n192_trained.json", "g9_y_hat_n192.npz")}


def gen(ref_model, tag):
    N, weights, fixture, out = SETS[tag]
    meta = json.load(open(os.path.join(HERE, fixture)))
    sd = gg.trained_weights(weights)
    net = ref_model.ImageCompressor(out_channel_N=N)
    net.load_state_dict(sd)
    arrays = {}
    for i in range(24):
        h, w = (768, 512) if i in KODAK_PORTRAIT else (512, 768)
        x = torch.from_numpy(synth.to_unit_float(synth.smooth_image_u8(100 + i, h, w)))[None]
        _, y_hat, _, _, y = gg.run_reference_eval(net, x)
        if gg.sha256(y_hat) != meta["images"][i]["y_hat_sha256"]:
            raise SystemExit(f"{tag}[{i}]: the reference's y_hat no longer matches {fixture}")
        yh = y_hat.numpy()
        assert np.abs(yh).max() <= 127 and np.array_equal(yh, np.round(yh))
        arrays[f"yhat_{i:02d}"] = yh.astype(np.int8)
        yf = y.numpy().reshape(-1)
        d = np.abs(np.abs(yf - np.floor(yf)) - 0.5)
        idx = np.nonzero(d < NEAR)[0]
        arrays[f"near_idx_{i:02d}"] = idx.astype(np.int32)
        arrays[f"near_y_{i:02d}"] = yf[idx].astype(np.float32)
        print(tag, i, yh.shape, "near ties:", idx.size, flush=True)
    np.savez_compressed(os.path.join(HERE, out), **arrays)
    print("wrote", out, os.path.getsize(os.path.join(HERE, out)), "bytes")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", default="g8,g9")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 1)
    ref_model, _ = gg.import_reference(args.reference)
    for tag in args.only.split(","):
        gen(ref_model, tag)


if __name__ == "__main__":
    main()
