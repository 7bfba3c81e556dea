"""Times the GDN γ-gradient kernels (x6 and f32) at the train step's GDN sizes (B=32 256²)."""
import sys
import torch
sys.path.insert(0, ".")
from iclr_17_compression_amd import kernels, synth

dev = "cuda"
for P in (131072, 32768):
    dn = torch.from_numpy(synth.normal_like(1, (P, 192), 1.0)).to(dev)
    u = torch.from_numpy(synth.normal_like(2, (P, 192), 1.0)).to(dev)
    out = {}
    for x6 in (True, False):
        for _ in range(3):
            kernels.gdn_wgrad(dn, u, x6=x6)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            kernels.gdn_wgrad(dn, u, x6=x6)
        b.record()
        torch.cuda.synchronize()
        out["x6" if x6 else "f32"] = round(a.elapsed_time(b) / 50 * 1e3, 1)
    print("P", P, "us/call", out, flush=True)
