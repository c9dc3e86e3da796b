"""Ray-batch data parallelism: one process per GPU, one gradient all-reduce per step.

Rays are independent through sampling, encoding, the field MLP, compositing and
resampling, so every rank renders its own ray shard and the only
exchange is the mean of the parameter gradients — one flat fp32 bucket (~2.6 MB
for NerfModel) per step over RCCL ("nccl" backend = RCCL on ROCm; xGMI on one
node).  The reference itself is single-device (run_barf.py:103-148).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradAllReduce:
    """Averages ``.grad`` of ``params`` across the process group with ONE collective.

    Gradients are packed into a persistent flat buffer (allocated once), reduced
    in place and copied back; parameters without a gradient contribute zeros so
    every rank issues the same collective."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.numel = sum(p.numel() for p in self.params)
        self.flat = None

    def __call__(self) -> None:
        if not dist.is_available() or not dist.is_initialized():
            return
        world = dist.get_world_size(self.group)
        if world == 1:
            return
        dev = self.params[0].device
        if self.flat is None or self.flat.device != dev:
            self.flat = torch.empty(self.numel, device=dev, dtype=torch.float32)
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                self.flat[off:off + n].zero_()
            else:
                self.flat[off:off + n].copy_(p.grad.reshape(-1))
            off += n
        dist.all_reduce(self.flat, group=self.group)
        self.flat.div_(world)
        off = 0
        for p in self.params:
            n = p.numel()
            g = self.flat[off:off + n].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            off += n


def shard_rays(n_global: int, rank: int, world: int) -> slice:
    """Contiguous shard of a global ray batch (sizes differ by at most one ray)."""
    base, rem = divmod(n_global, world)
    start = rank * base + min(rank, rem)
    return slice(start, start + base + (1 if rank < rem else 0))
