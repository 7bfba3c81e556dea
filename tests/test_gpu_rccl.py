"""RCCL on the GPU box before the driver's 8-GPU run (train.py:228's DataParallel gradient
reduction, re-done as one process per GPU): a world-size-1 **nccl** process group on cuda:0
(TCPStore on 127.0.0.1, ``device_id=``), the overlapped ``GradAllReducer`` launched from inside
the real fused backward (its world-size-1 short-circuit bypassed with ``always=True``), then
``finish`` and the fused clamp + Adam. A one-rank sum scaled by 1/1 is the identity, so the
gradients and the parameters after two Adam steps must equal a run without the reducer bit for
bit (Adam reads the averaged gradients that ``finish`` wrote after waiting on the RCCL work).
What a one-rank group cannot show is cross-rank traffic over xGMI: that is the driver's
8-GPU run."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, B, S = 192, 2, 64
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
    x = torch.from_numpy(synth.to_unit_float(synth.image_u8(7, B, S, S))).to(dev)
    noise = torch.from_numpy(synth.uniform(8, (B, N, S // 16, S // 16), -0.5, 0.5)).to(dev)
    return x, noise


def _step(net, opt, x, noise, red=None):
    opt.zero_grad(set_to_none=True)
    _, mse, bpp = net.forward_train(x, noise=noise)
    (LAM * mse + bpp).backward()
    launched = len(red.pending) if red is not None else 0
    if red is not None:
        red.finish()
    grads = {k: p.grad.detach().clone() for k, p in net.named_parameters()}
    opt.step()
    return grads, launched


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    try:
        from iclr_17_compression_amd import dist as idist
        from iclr_17_compression_amd.optim import FusedAdam
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        backend = dist.get_backend()
        x, noise = _batch(dev)
        # reference: the same two steps with no reducer attached
        net0 = _net(dev)
        opt0 = FusedAdam(list(net0.parameters()), lr=1e-4, grad_clip=5)
        ref = [_step(net0, opt0, x, noise)[0] for _ in range(2)]
        net = _net(dev)
        opt = FusedAdam(list(net.parameters()), lr=1e-4, grad_clip=5)
        red = idist.GradAllReducer(list(net.parameters()), bucket_mb=2.0, always=True).attach(net)
        out = []
        for _ in range(2):
            g, launched = _step(net, opt, x, noise, red)
            out.append((g, launched))
        torch.cuda.synchronize()
        res = {"backend": backend, "launched": [l for _, l in out],
               "grad_equal": [all(torch.equal(g[k], r[k]) for k in r) for (g, _), r in zip(out, ref)],
               "param_equal": all(torch.equal(p, p0) for p, p0 in zip(net.parameters(), net0.parameters())),
               "pending_after": len(red.pending)}
        # the bucketed all-reduce itself over RCCL: a one-rank SUM leaves the values unchanged
        t = torch.arange(1 << 20, device=dev, dtype=torch.float32)
        w = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
        w.wait()
        torch.cuda.synchronize()
        res["allreduce_identity"] = bool(torch.equal(t, torch.arange(1 << 20, device=dev, dtype=torch.float32)))
        q.put(res)
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(repr(e))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_rccl_world1_overlapped_allreduce(device):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert isinstance(res, dict), res
    assert res["backend"] == "nccl"
    assert all(n > 0 for n in res["launched"]), res   # launched from inside the backward
    assert res["pending_after"] == 0
    assert all(res["grad_equal"]), res
    assert res["param_equal"], res
    assert res["allreduce_identity"]
