"""Per-phase cycle stamps of the persistent bf16 conv1 kernel (diagnostic build with
-DICLR17_C1P_STAMPS=1): ICLR17_LIB=build/ab_stamps/libiclr17.so python tools/c1p_stamps.py. GPU.
Phases per block: 0 patch loads issued, 1 main loop done, 2 GDN epilogue done, 3 next plane
written, 4 output stored + barrier."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iclr_17_compression_amd import _lib, kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

dev = torch.device("cuda:0")
N, B = 192, 64
net = ImageCompressor(N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
w1, _, _ = net.Encoder.packed_bf16()
e1 = net.Encoder.gdn1.effective_params_bf16()
x = torch.rand(B, 3, 256, 256, device=dev)
for _ in range(20):
    kernels.conv1_gdn_bf16(x, w1, net.Encoder.conv1.bias, *e1, N)
torch.cuda.synchronize()
WAVES, STK, STP = 8, 20, 5
buf = np.zeros(1024 * WAVES * STK * STP, dtype=np.uint64)
lib = ctypes.CDLL(os.environ["ICLR17_LIB"])
lib.iclr17_debug_c1p_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert lib.iclr17_debug_c1p_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(1024, WAVES, STK, STP).astype(np.int64)
nwg = 256
ntile = 4096 // nwg   # blocks per workgroup at B=64 (64 images x 64 blocks)
st = st[:nwg, :, :ntile, :]
d = np.diff(st, axis=3)                                   # phase durations
gap = st[:, :, 1:, 0] - st[:, :, :-1, 4]                  # loop overhead between blocks
tot = st[:, :, -1, 4] - st[:, :, 0, 0]
names = ["main loop", "GDN epilogue", "next plane", "stores+barrier"]
for i, n in enumerate(names):
    v = d[..., i]
    print(f"{n:16s} median {np.median(v):8.0f}  mean {v.mean():8.0f}  p90 {np.percentile(v, 90):8.0f} cycles")
print(f"{'between blocks':16s} median {np.median(gap):8.0f}")
print(f"per block (total/{ntile}) median {np.median(tot) / ntile:8.0f}; whole loop median {np.median(tot):.0f}")
for w in range(WAVES):
    print("wave", w, "main", np.median(d[:, w, :, 0]), "epi", np.median(d[:, w, :, 1]), "plane", np.median(d[:, w, :, 2]), "out", np.median(d[:, w, :, 3]))
