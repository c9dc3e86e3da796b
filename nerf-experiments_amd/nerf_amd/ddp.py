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

    The gradients are concatenated into one flat fp32 bucket (a single copy kernel) followed by
    one "has a gradient" flag per parameter, reduced in place, scaled by 1/world, and every
    parameter's ``.grad`` becomes a view of its slice of the bucket — no copy back.  A parameter
    without a gradient contributes zeros so every rank issues the same collective; a parameter
    that NO rank produced a gradient for ends with ``.grad = None``, as with one process and as
    torch DDP leaves it, so the optimizer skips it on every rank (no momentum or weight-decay
    drift).  Deciding that needs the reduced flags on the host: the read happens only on a rank
    that itself lacks some gradient (if every local gradient exists, every reduced flag is >= 1)."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.sizes = [p.numel() for p in self.params]
        self.numel = sum(self.sizes)

    def __call__(self) -> None:
        if not dist.is_available() or not dist.is_initialized():
            return
        world = dist.get_world_size(self.group)
        if world == 1:
            return
        missing = [p.grad is None for p in self.params]
        ref = self.params[0]
        grads = [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in self.params]
        flags = torch.tensor([0.0 if m else 1.0 for m in missing], dtype=ref.dtype).to(ref.device, non_blocking=True)
        flat = torch.cat(grads + [flags])
        dist.all_reduce(flat, group=self.group)
        flat.div_(world)
        parts = flat.split(self.sizes + [len(self.params)])
        used = None
        if any(missing):
            used = (parts[-1] > 0).tolist()       # host read of the reduced flags (only here)
        for i, (p, g) in enumerate(zip(self.params, parts[:-1])):
            p.grad = g.view_as(p) if used is None or used[i] else None


def shard_rays(n_global: int, rank: int, world: int) -> slice:
    """Contiguous shard of a global ray batch (sizes differ by at most one ray)."""
    base, rem = divmod(n_global, world)
    start = rank * base + min(rank, rem)
    return slice(start, start + base + (1 if rank < rem else 0))
