"""Adam with one fused HIP launch per step.

The reference trains every model with ``torch.optim.Adam(eps=1e-5)`` (configure_optimizers,
barf/model_interpolation.py:543-584).  ``FusedAdam`` IS a ``torch.optim.Adam`` (same
constructor, ``param_groups``, ``state`` layout — ``step`` / ``exp_avg`` / ``exp_avg_sq`` — and
state_dict, so LR schedulers and checkpoints work unchanged); only ``step()`` differs: every
parameter with a gradient is updated by ``nerf_adam_step`` (csrc/adam.hip), one launch per 48
tensors, instead of torch's ~7 multi-tensor kernels.  The bias corrections are formed on the
host exactly as torch forms them (Python floats).  amsgrad / maximize / capturable are not
supported and raise.
"""
from __future__ import annotations

import torch

from . import kernels as K


class FusedAdam(torch.optim.Adam):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        batches: dict[tuple, list] = {}
        for group in self.param_groups:
            if group.get("amsgrad") or group.get("maximize") or group.get("capturable"):
                raise NotImplementedError("FusedAdam supports plain Adam (no amsgrad / maximize / capturable)")
            beta1, beta2 = group["betas"]
            lr = float(group["lr"])
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                if not g.is_contiguous():
                    g = g.contiguous()
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                state["step"] += 1
                t = float(state["step"])
                bc1 = 1 - beta1 ** t
                bc2 = 1 - beta2 ** t
                key = (float(beta1), float(beta2), float(group["eps"]), p.device)
                batches.setdefault(key, []).append((p, g, state["exp_avg"], state["exp_avg_sq"], -lr / bc1, bc2 ** 0.5,
                                                    float(group["weight_decay"])))
        for (beta1, beta2, eps, dev), entries in batches.items():
            K.adam_step(entries, beta1, beta2, eps, dev)
            # the kernel writes through raw pointers: bump the version counters as an in-place
            # torch op would, so version-keyed caches (the MLP's packed weights) see the update
            for e in entries:
                torch.autograd.graph.increment_version(e[0])
        return loss


__all__ = ["FusedAdam"]
