"""Trains the codec to a realistic operating point for the G8 / G9 fixtures (GPU, x6 training
path): N = 128 (train.py's default out_channel_N; G8) or 192 (BASELINE C2's N; G9), λ = 0.01·255²
(train_lambda 650.25), Adam, ±5 clamp,
B = 16 random 256² crops with h/v flips of 96 smooth synthetic photos (synth.smooth_image_u8,
seeds 20000+, disjoint from the Kodak-synth seeds 100..123). Writes the state dict as
gpurun_out/op_point/weights_n{N}.npz (stored fp16 as tests/golden/g8_weights_n128.npz /
g9_weights_n192.npz) and
prints the running loss / PSNR / bpp.

    python tools/train_operating_point.py [--steps 20000] [--N 128|192]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402
from iclr_17_compression_amd.optim import FusedAdam  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20000)
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--lr", type=float, default=3e-4)
ap.add_argument("--out", default="gpurun_out/op_point")
ap.add_argument("--N", type=int, default=128)
args = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(17)
os.makedirs(args.out, exist_ok=True)

pool = []
for i in range(96):
    H, W = (768, 512) if i % 4 == 0 else (512, 768)
    pool.append(torch.from_numpy(synth.to_unit_float(synth.smooth_image_u8(20000 + i, H, W))).to(dev))
print(f"pool of {len(pool)} images ready", flush=True)

net = ImageCompressor(out_channel_N=args.N).to(dev).train()
opt = FusedAdam(list(net.parameters()), lr=args.lr, grad_clip=5)
lam = 0.01 * 255.0 ** 2
g = torch.Generator().manual_seed(5)
S = 256
t0 = time.time()
hist = []
for step in range(1, args.steps + 1):
    if step == int(args.steps * 0.75):
        for grp in opt.param_groups:
            grp["lr"] = args.lr * 0.1
    idx = torch.randint(len(pool), (args.batch,), generator=g).tolist()
    crops = []
    for i in idx:
        img = pool[i]
        y = int(torch.randint(img.shape[1] - S + 1, (1,), generator=g))
        x = int(torch.randint(img.shape[2] - S + 1, (1,), generator=g))
        c = img[:, y:y + S, x:x + S]
        if torch.rand(1, generator=g).item() < 0.5:
            c = c.flip(2)
        if torch.rand(1, generator=g).item() < 0.5:
            c = c.flip(1)
        crops.append(c)
    xb = torch.stack(crops).contiguous()
    opt.zero_grad(set_to_none=True)
    _, mse, bpp = net.forward_train(xb)
    loss = lam * mse + bpp
    loss.backward()
    opt.step()
    if step % 50 == 0:
        hist.append((loss.item(), mse.item(), bpp.item()))
    if step % 1000 == 0:
        l, m, b = (float(np.mean([h[k] for h in hist[-20:]])) for k in range(3))
        print(f"step {step}: loss {l:.4f} psnr {10 * np.log10(1 / m):.3f} bpp {b:.4f} "
              f"({time.time() - t0:.0f} s)", flush=True)

net.eval()
with torch.no_grad():
    ev = []
    for i in range(24):
        H, W = (768, 512) if i in (3, 8, 9, 16, 17, 18) else (512, 768)
        x = torch.from_numpy(synth.to_unit_float(synth.smooth_image_u8(100 + i, H, W)))[None].to(dev)
        r = net.evaluate(x, want_msssim=True)
        ev.append((r["bpp"].item(), r["psnr"].item(), r["ms_ssim"].item()))
print("kodak-synth eval (bpp, psnr, ms_ssim) mean:", np.mean(ev, axis=0).round(5).tolist(), flush=True)
np.savez(os.path.join(args.out, f"weights_n{args.N}.npz"),
         **{k: v.detach().cpu().numpy() for k, v in net.state_dict().items()})
print("saved", flush=True)
