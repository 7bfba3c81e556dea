"""Fused clamp + Adam — train.py:106-112 (clip_gradient then optimizer.step() of
torch.optim.Adam(lr), the reference's optimizer, train.py:233) as one HIP launch over every
parameter tensor (``iclr17_adam_step``).

``FusedAdam`` has torch.optim.Adam's constructor and state layout (``exp_avg``,
``exp_avg_sq``, ``step``) and the same update order, so checkpoints of its state dict look
like Adam's. ``grad_clip`` folds train.py's element-wise ±5 clamp into the same pass (the
clamped gradient is written back, as ``p.grad.data.clamp_`` does).
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch

from . import kernels
from ._lib import Iclr17Error, call


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False,
                 grad_clip: Optional[float] = None):
        if weight_decay != 0.0 or amsgrad:
            raise Iclr17Error("iclr17: FusedAdam implements the reference's Adam (no weight decay, "
                              "no amsgrad)")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        self.grad_clip = grad_clip
        self._desc = None
        self._desc_key = None

    def _descriptors(self, group):
        ps = [p for p in group["params"] if p.grad is not None]
        for p in ps:
            if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous():
                raise Iclr17Error("iclr17: FusedAdam needs contiguous fp32 device parameters")
            st = self.state[p]
            if not st:
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        rows = [(p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                 self.state[p]["exp_avg_sq"].data_ptr(), p.numel()) for p in ps]
        key = tuple(rows)
        if key != self._desc_key:   # pointer table on the device, rewritten when a buffer moves
            # (with zero_grad(set_to_none=True) the gradients are new tensors every step). The
            # table goes up by a non-blocking copy from one of two pinned host buffers, so the
            # host never waits for the device here; a buffer is refilled only after the copy
            # that last read it has completed (its event).
            n = len(rows)
            if self._desc is None or self._desc.shape[0] != n:
                self._desc = torch.empty((n, 5), dtype=torch.int64, device=ps[0].device)
                self._host = [torch.empty((n, 5), dtype=torch.int64, pin_memory=True)
                              for _ in range(2)]
                self._host_ev = [None, None]
                self._slot = 0
            slot, self._slot = self._slot, self._slot ^ 1
            if self._host_ev[slot] is not None:
                self._host_ev[slot].synchronize()
            self._host[slot].copy_(torch.tensor(rows, dtype=torch.int64))
            self._desc.copy_(self._host[slot], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(ps[0].device))
            self._host_ev[slot] = ev
            self._desc_key = key
        return ps, max(r[4] for r in rows)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            if not any(p.grad is not None for p in group["params"]):
                continue
            ps, max_n = self._descriptors(group)
            steps = {int(self.state[p]["step"].item()) for p in ps}
            if len(steps) != 1:
                raise Iclr17Error("iclr17: FusedAdam needs one step count per parameter group")
            t = steps.pop() + 1
            for p in ps:
                self.state[p]["step"].fill_(float(t))
            b1, b2 = group["betas"]
            clip = float(self.grad_clip) if self.grad_clip else 0.0
            call("iclr17_adam_step", kernels._p(self._desc), len(ps), max_n, float(group["lr"]),
                 float(b1), float(b2), float(group["eps"]), t, clip, kernels._stream(ps[0]))
            # the kernel updated the parameters through raw pointers: move their version
            # counters as an in-place op would, so version-keyed caches (packed weights) refresh
            torch.autograd.graph.increment_version(ps)
        return loss
