"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL ("nccl") on MI355X.

* Inference / evaluation shards images by rank — images are independent, so there is no
  collective in the data path; per-image metrics come back with one all-gather at the end.
* Training is data parallel (the reference's DataParallel, train.py:228, re-done as one process
  per GPU): each rank holds a replica, runs the fused forward/backward on its shard, and the
  gradients are averaged with bucketed all-reduces (flat fp32 buckets sized for the xGMI ring)
  before the ±5 clamp (train.py:106-111) and the Adam step.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

Tensor = torch.Tensor


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def init_from_env(backend: str = "nccl") -> torch.device:
    """Initialise from torchrun's RANK / WORLD_SIZE / LOCAL_RANK (MASTER_ADDR 127.0.0.1)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if ws > 1 and not dist.is_initialized():
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return dev


def shard_range(n: int, r: int, w: int):
    """Contiguous, balanced split of n items over w ranks: rank r gets [lo, hi)."""
    base, extra = divmod(n, w)
    lo = r * base + min(r, extra)
    return lo, lo + base + (1 if r < extra else 0)


def shard_batch(x: Tensor, r: int = None, w: int = None) -> Tensor:
    r = rank() if r is None else r
    w = world() if w is None else w
    lo, hi = shard_range(x.shape[0], r, w)
    return x[lo:hi]


def gather_rows(t: Tensor, n_total: int) -> Tensor:
    """All-gather per-image rows (1-D or 2-D) whose shards follow shard_range; returns the
    full [n_total, ...] tensor on every rank in image order."""
    w = world()
    if w == 1:
        return t
    sizes = [shard_range(n_total, r, w)[1] - shard_range(n_total, r, w)[0] for r in range(w)]
    m = max(sizes)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    out = [torch.empty_like(pad) for _ in range(w)]
    dist.all_gather(out, pad)
    return torch.cat([o[:s] for o, s in zip(out, sizes)], dim=0)


def bucketize(params: Sequence[Tensor], bucket_bytes: int) -> List[List[Tensor]]:
    """Group parameters (in order) into buckets of at most ~bucket_bytes of fp32 gradient."""
    buckets, cur, size = [], [], 0
    for p in params:
        nb = p.numel() * 4
        if cur and size + nb > bucket_bytes:
            buckets.append(cur)
            cur, size = [], 0
        cur.append(p)
        size += nb
    if cur:
        buckets.append(cur)
    return buckets


def allreduce_grads(params: Sequence[Tensor], bucket_mb: float = 4.0) -> None:
    """Average .grad over ranks: flatten each bucket, all-reduce (sum) once, scale by 1/world.
    Ranks must call with the same parameter order (they hold identical replicas)."""
    w = world()
    if w == 1:
        return
    ps = [p for p in params if p.grad is not None]
    for bucket in bucketize(ps, int(bucket_mb * 2 ** 20)):
        flat = torch.cat([p.grad.reshape(-1) for p in bucket])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.mul_(1.0 / w)
        off = 0
        for p in bucket:
            n = p.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n


class GradAllReducer:
    """Gradient averaging overlapped with the backward (the reference's DataParallel gradient
    reduction, train.py:228, as one process per GPU).

    The fused training backward (autograd.CodecTrainFn) produces the synthesis gradients first
    and the analysis ones last. Attached to a model, it hands each group of parameter gradients
    to ``launch`` as soon as that group is computed: the gradients are packed into one flat
    buffer (≤ bucket_mb per bucket) on the compute stream and all-reduced asynchronously — RCCL
    runs on its own stream — while the compute stream goes on with the rest of the backward.
    ``finish`` makes the compute stream wait for every reduction and writes the averages into
    ``p.grad``, before the clamp + Adam launch.

    Usage per step (grads must start as None: set_to_none zero_grad)::

        opt.zero_grad(set_to_none=True); loss.backward(); reducer.finish(); opt.step()
    """

    def __init__(self, params: Sequence[Tensor], bucket_mb: float = 4.0, always: bool = False):
        self.params = list(params)
        self.bucket_bytes = int(bucket_mb * 2 ** 20)
        self.pending = []        # (work, flat, params)
        self.launched = set()
        # always: run the collective path even in a one-rank group (a world-size-1 RCCL
        # communicator on one GPU exercises launch / RCCL stream / finish ordering; tests)
        self.always = always

    def attach(self, net) -> "GradAllReducer":
        net._grad_reducer = self
        return self

    @property
    def active(self) -> bool:
        return world() > 1 or (self.always and dist.is_available() and dist.is_initialized())

    def launch(self, params: Sequence[Tensor], grads: Sequence[Optional[Tensor]]) -> None:
        """All-reduce (sum, async) these parameters' freshly computed gradients."""
        pairs = [(p, g) for p, g in zip(params, grads) if g is not None and id(p) not in self.launched]
        for p, g in pairs:
            if p.grad is not None and p.grad is not g:
                # finish() replaces p.grad with the average of g: a value p.grad already holds
                # (zero_grad without set_to_none, gradient accumulation) would be lost
                raise RuntimeError("GradAllReducer.launch: p.grad already holds a gradient; call "
                                   "zero_grad(set_to_none=True) before the backward")
        for bucket in bucketize([g for _, g in pairs], self.bucket_bytes):
            ids = {id(g) for g in bucket}
            ps = [p for p, g in pairs if id(g) in ids]
            flat = torch.cat([g.reshape(-1) for g in bucket])
            work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True)
            self.pending.append((work, flat, ps))
            self.launched.update(id(p) for p in ps)

    def wait(self) -> None:
        """Make the compute stream wait for every launched reduction and drop the results (the
        bench's all-reduce-alone timing)."""
        for work, _, _ in self.pending:
            work.wait()
        self.pending.clear()
        self.launched.clear()

    def finish(self) -> None:
        """Wait for the reductions (stream-ordered) and set p.grad = the rank average. Gradients
        no backward launched (parameters outside the fused backward) are reduced here."""
        if not self.active:
            return
        w = world()
        rest = [p for p in self.params if p.grad is not None and id(p) not in self.launched]
        if rest:
            self.launch(rest, [p.grad for p in rest])
        for work, flat, ps in self.pending:
            work.wait()
            if any(p.grad is None for p in ps):
                raise RuntimeError("GradAllReducer.finish: a launched parameter has no .grad")
            flat.mul_(1.0 / w)
            off = 0
            for p in ps:
                n = p.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n
        self.pending.clear()
        self.launched.clear()


def max_over_ranks(value: float, device) -> float:
    if world() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()
