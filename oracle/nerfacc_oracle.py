"""CPU oracle of the nerfacc proposal sampler and interlevel loss — TEST INFRASTRUCTURE ONLY.

nerfacc (used by garf/model_garf.py:81,210-230,257) is an external CUDA package, version unpinned
(environment.yml:26), not vendored in the reference and not installed here: this restates its
published algorithm (PropNetEstimator.sampling / compute_loss, the mip-NeRF 360 interlevel loss)
in PyTorch CPU fp32/fp64 and is **parity unpinned** — no nerfacc output pins it.  It checks
nerf_amd.prop_sampler and its kernels (csrc/propnet.hip) against the same restatement.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
from __future__ import annotations

import torch


def prop_cdf(w: torch.Tensor) -> torch.Tensor:
    """[R, K] weights -> [R, K+1]: 0, exclusive sums (fp64), 1 (= 1 - [trans, 0])."""
    ex = torch.cumsum(w.double(), dim=-1)[:, :-1]
    z = torch.zeros(w.shape[0], 1, dtype=torch.float64)
    return torch.cat([z, ex, torch.ones_like(z)], dim=-1).float()


def quantiles(R: int, n: int) -> torch.Tensor:
    return (torch.arange(n + 1, dtype=torch.float32) / n).expand(R, n + 1)


def invert_cdf(vals: torch.Tensor, cdf: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """s at quantiles u of the piecewise-linear cdf over the edges vals (both [R, K+1])."""
    K = vals.shape[1] - 1
    b = (torch.searchsorted(cdf.contiguous(), u.contiguous(), right=True) - 1).clamp(0, K - 1)
    c0, c1 = cdf.gather(1, b), cdf.gather(1, b + 1)
    v0, v1 = vals.gather(1, b), vals.gather(1, b + 1)
    den = c1 - c0
    f = torch.where(den > 0, (u - c0) / torch.where(den > 0, den, torch.ones_like(den)), torch.zeros_like(den))
    return v0 + f.clamp(0, 1) * (v1 - v0)


def stot(s: torch.Tensor, transform: str, near: float, far: float) -> torch.Tensor:
    if transform == "uniform":
        return s * far + (1 - s) * near
    return 1.0 / (s * (1.0 / far) + (1 - s) * (1.0 / near))


def render_weights(sigmas: torch.Tensor, delta: torch.Tensor) -> torch.Tensor:
    """w = trans * alpha, alpha = 1 - exp(-sigma delta), trans exclusive (fp64 prefix)."""
    sd = (sigmas * delta).double()
    excl = torch.cumsum(sd, dim=-1) - sd
    return (torch.exp(-excl) * (1 - torch.exp(-sd))).float()


def pdf_loss(q_vals, q_cdf, k_vals, k_cdf, eps: float = 1e-7) -> torch.Tensor:
    """Per query interval max(w - w_outer, 0)^2 / (w + eps) (mip-NeRF 360 lossfun_outer as nerfacc's
    _pdf_loss): w_outer = k_cdf[right(q[j+1])] - k_cdf[left(q[j])]."""
    K = k_vals.shape[1] - 1
    right = torch.searchsorted(k_vals.contiguous(), q_vals.contiguous(), right=True)
    left = (right - 1).clamp(0, K)
    right = right.clamp(0, K)
    w = q_cdf[:, 1:] - q_cdf[:, :-1]
    w_outer = k_cdf.gather(1, right[:, 1:]) - k_cdf.gather(1, left[:, :-1])
    return torch.clamp(w - w_outer, min=0) ** 2 / (w + eps)


def interlevel_loss(q_vals, q_cdf, k_vals, key_w, eps: float = 1e-7) -> torch.Tensor:
    """mean loss, differentiable in the key weights through k_cdf = [0, exclusive sums, 1]."""
    z = torch.zeros(key_w.shape[0], 1)
    k_cdf = torch.cat([z, torch.cumsum(key_w, dim=-1)[:, :-1], torch.ones_like(z)], dim=-1)
    return pdf_loss(q_vals, q_cdf, k_vals, k_cdf, eps).mean()
