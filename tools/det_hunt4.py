"""ImageCompressor.run (fp32) repeated with poisoned free memory; the wrapped kernels record every
intermediate, so the first kernel whose output differs from the first run's is named
(diagnostic, GPU)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = torch.device("cuda:0")
meta = json.load(open("tests/golden/g5_kodak24_synth_n192.json"))
rec = []
for name in ("conv1_gdn", "conv2_gdn", "conv3_quant_rate", "deconv_igdn", "deconv3"):
    f = getattr(kernels, name)

    def wrap(*a, _f=f, _n=name, **k):
        out = _f(*a, **k)
        o = out[0] if isinstance(out, tuple) else out
        rec.append((_n, o.clone()))
        return out
    setattr(kernels, name, wrap)


def poison(k):
    torch.cuda.synchronize()
    n = 1 << 28
    junk = torch.empty(n, device=dev, dtype=torch.float32)
    pats = [[float("nan"), 3e38, -3e38, 1e-40, -7.5, float("inf")], [1.0, -2.0, 1e30, 0.5, 7.0, -1e-30]]
    junk.copy_(torch.tensor(pats[k % 2], device=dev).repeat(n // 6 + 1)[:n])
    del junk
    torch.cuda.synchronize()


net = ImageCompressor(meta["N"])
net.load_state_dict({k: torch.from_numpy(v) for k, v in
                     synth.trained_like_state_dict(meta["N"], meta["weight_seed"]).items()})
net = net.to(dev)
kernels.set_precision(prec)
net.train()
xt = torch.rand(4, 3, 128, 128, device=dev)
_, mse, bpp = net.forward_train(xt)
(mse * 650 + bpp).backward()
net.zero_grad(set_to_none=True)
net.eval()
nbad = 0
for i in (0, 3):
    row = meta["images"][i]
    x = torch.from_numpy(synth.to_unit_float(synth.smooth_image_u8(
        meta["image_seed_base"] + row["index"], row["height"], row["width"])))[None].to(dev)
    x2 = torch.cat([x, x.flip(3)])
    ref = None
    with torch.no_grad():
        for r in range(reps):
            if r % 2 == 1:
                poison(r // 2)
            rec.clear()
            out = net.run(x2, training=False, x_ref_sse=True, want_y=True)
            cur = list(rec)
            if ref is None:
                ref = cur
                continue
            for (n0, t0), (n1, t1) in zip(ref, cur):
                if not torch.equal(t0, t1):
                    nz = torch.nonzero(t0 != t1)
                    nbad += 1
                    print(f"image {i} rep {r}: first differing kernel {n1}: {nz.shape[0]} of {t1.numel()} "
                          f"shape {tuple(t1.shape)} first {nz[:3].tolist()} last {nz[-1:].tolist()} "
                          f"nan {torch.isnan(t1).sum().item()}", flush=True)
                    break
print(f"{prec}: {nbad} bad reps", flush=True)
