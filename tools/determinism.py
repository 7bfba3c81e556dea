"""Run-to-run determinism of the eval chain (diagnostic, GPU): the same images through
``ImageCompressor.run`` R times per precision, every output compared bitwise with the first run.
Odd rounds first fill the caching allocator's free blocks with a poison pattern (NaN, ±huge,
denormals), so an output that reads memory no kernel wrote shows up as a mismatch.

    python tools/determinism.py [--rounds 20] [--precisions fp32,x6,bf16]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=20)
ap.add_argument("--precisions", default="fp32,x6,bf16")
args = ap.parse_args()
dev = torch.device("cuda:0")
meta = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "tests", "golden", "g5_kodak24_synth_n192.json")))
net = ImageCompressor(meta["N"])
net.load_state_dict({k: torch.from_numpy(v) for k, v in
                     synth.trained_like_state_dict(meta["N"], meta["weight_seed"]).items()})
net = net.to(dev).eval()
imgs = []
for i in (0, 3, 9, 23):
    row = meta["images"][i]
    imgs.append(torch.from_numpy(synth.to_unit_float(synth.smooth_image_u8(
        meta["image_seed_base"] + row["index"], row["height"], row["width"])))[None].to(dev))
for prec in args.precisions.split(","):
    kernels.set_precision(prec)
    bad = {}
    with torch.no_grad():
        for j, x in enumerate(imgs):
            ref = None
            for r in range(args.rounds):
                if r % 2 == 1:
                    torch.cuda.synchronize()
                    junk = torch.empty(1 << 30, device=dev, dtype=torch.float32)
                    pat = torch.tensor([float("nan"), 3e38, -3e38, 1e-40, -7.5], device=dev)
                    junk.copy_(pat.repeat((1 << 30) // 5 + 1)[: 1 << 30])
                    del junk
                    torch.cuda.synchronize()
                out = net.run(x, training=False, x_ref_sse=True, want_y=True)
                cur = {k: v.clone() for k, v in out.items() if torch.is_tensor(v)}
                if ref is None:
                    ref = cur
                    continue
                for k in ref:
                    if not torch.equal(ref[k], cur[k]):
                        d = (ref[k].double() - cur[k].double()).abs()
                        bad.setdefault(f"img{j}:{k}", []).append(
                            (r, int((d > 0).sum().item()), float(d.max().item())))
    print(json.dumps({"precision": prec, "rounds": args.rounds,
                      "mismatches": {k: v[:5] for k, v in bad.items()}}), flush=True)
