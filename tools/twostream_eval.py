"""Does splitting the eval batch over two HIP streams (half the images each, launched
interleaved) beat one stream? Times bench.Step on B images vs two Steps on B/2 (diagnostic, GPU).

    python tools/twostream_eval.py [--precision x6] [--batch 64]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from iclr_17_compression_amd import kernels, synth  # noqa: E402
from iclr_17_compression_amd.model import ImageCompressor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="x6")
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
kernels.set_precision(args.precision)
dev = torch.device("cuda:0")
net = ImageCompressor(192)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(192, 1).items()})
net = net.to(dev).eval()
B = args.batch
x = torch.from_numpy(synth.to_unit_float(synth.image_u8(1000, B, 256, 256))).to(dev)
one = bench.Step(net, x)
halves = [bench.Step(net, x[: B // 2].contiguous()), bench.Step(net, x[B // 2:].contiguous())]
side = torch.cuda.Stream(device=dev)


def run_one():
    one()


def run_two():
    main = torch.cuda.current_stream(dev)
    side.wait_stream(main)
    halves[0]()
    with torch.cuda.stream(side):
        halves[1]()
    main.wait_stream(side)


def timeit(fn):
    with torch.no_grad():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3


for r in range(3):
    t1, t2 = timeit(run_one), timeit(run_two)
    print(f"{args.precision} B={B}: one stream {t1:.3f} ms ({B * 65536 / t1 / 1e3:.0f} Mpix/s), "
          f"two streams {t2:.3f} ms ({B * 65536 / t2 / 1e3:.0f} Mpix/s)", flush=True)
