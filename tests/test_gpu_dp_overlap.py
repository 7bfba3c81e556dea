"""Data parallelism with the all-reduce overlapped with the backward (dist.GradAllReducer hooked
into autograd.CodecTrainFn), two ranks on the one GPU over gloo: after ``finish`` every rank
holds the gradient of the whole batch — the mean of the two shard gradients, which
tests/test_gpu_fullsize.py shows equals the full-batch gradient — and both ranks' gradients are
bitwise equal."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, B, S = 192, 4, 64
LAM = 0.01 * 255.0 ** 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _net(dev):
    from iclr_17_compression_amd import synth
    from iclr_17_compression_amd.model import ImageCompressor
    net = ImageCompressor(out_channel_N=N)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 3).items()})
    return net.to(dev).train()


def _batch(dev):
    from iclr_17_compression_amd import synth
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(5, B, S, S))).to(dev)
    noise = torch.from_numpy(synth.uniform(6, (B, N, S // 16, S // 16), -0.5, 0.5)).to(dev)
    return x, noise


def _worker(r, w, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(w))
    try:
        from iclr_17_compression_amd import dist as idist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=r, world_size=w)
        net = _net(dev)
        x, noise = _batch(dev)
        lo, hi = idist.shard_range(B, r, w)
        red = idist.GradAllReducer(list(net.parameters()), bucket_mb=2.0).attach(net)
        net.zero_grad(set_to_none=True)
        _, mse, bpp = net.forward_train(x[lo:hi], noise=noise[lo:hi])
        (LAM * mse + bpp).backward()
        assert red.pending, "no all-reduce was launched inside the backward"
        red.finish()
        torch.cuda.synchronize()
        q.put((r, {k: p.grad.cpu().numpy() for k, p in net.named_parameters()}))   # plain bytes
        dist.barrier()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((r, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_overlapped_allreduce_two_ranks(device):
    w = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, w, port, q)) for r in range(w)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(w))
    for p in ps:
        p.join(timeout=60)
    for r in range(w):
        assert isinstance(res[r], dict), res[r]
    # the single-process shard mean
    net = _net(device)
    x, noise = _batch(device)
    mean = None
    for lo, hi in ((0, B // 2), (B // 2, B)):
        net.zero_grad(set_to_none=True)
        _, mse, bpp = net.forward_train(x[lo:hi], noise=noise[lo:hi])
        (LAM * mse + bpp).backward()
        g = {k: p.grad.detach().cpu().clone() for k, p in net.named_parameters()}
        mean = g if mean is None else {k: (mean[k] + g[k]) for k in g}
    mean = {k: v / 2 for k, v in mean.items()}
    for k in mean:
        g0, g1 = torch.from_numpy(res[0][k]), torch.from_numpy(res[1][k])
        assert torch.equal(g0, g1), k
        err = ((g0 - mean[k]).abs().max() / mean[k].abs().max().clamp_min(1e-30)).item()
        assert err < 1e-6, (k, err)
