"""nerfacc's proposal estimator and renderer as GARF uses them, on the device.

The reference's GARF renderer (garf/model_garf.py:81, 194-236, 257) calls
  * ``nerfacc.PropNetEstimator().sampling(prop_sigma_fns, prop_samples, num_samples, n_rays,
    near_plane, far_plane, sampling_type="lindisp", stratified, requires_grad)``,
  * ``nerfacc.rendering(t_starts, t_ends, ray_indices=None, n_rays=None, rgb_sigma_fn, render_bkgd)``,
  * ``estimator.compute_loss(extras["trans"])``.
nerfacc is an external CUDA package (environment.yml:26, version unpinned), not vendored in the
reference and not installed here; this module restates its published algorithm with the same call
signatures, and its numerics are **parity unpinned** (checked against oracle/nerfacc_oracle.py, a
restatement of the same algorithm):
  * intervals live in s-space [0, 1]; ``lindisp`` maps s -> t with 1/t = s/far + (1-s)/near;
  * each level inverts the previous level's piecewise-linear cdf (initially uniform) at n + 1
    quantiles u_0 = 0, u_n = 1, u_i = i/n (stratified: (i - 1/2 + U)/n), evaluates the proposal
    density on the resulting intervals and forms cdf = 1 - [trans, 0] (trans = exclusive
    transmittance, alpha = 1 - exp(-sigma delta));
  * compute_loss: the mip-NeRF 360 interlevel loss, max(w - w_outer, 0)^2 / (w + 1e-7) per final
    interval (w from the radiance pass's trans, detached; w_outer the proposal's cdf mass over
    the key intervals overlapping it), averaged, summed over proposal levels.
Kernels: nerf_prop_sample / nerf_prop_cdf / nerf_prop_loss (csrc/propnet.hip); compositing is
nerf_composite_fwd/bwd with density factor 1.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch as th

from . import kernels as K
from .model_interpolation import _RenderRaysFn, _rng_seed

_EPS = 1e-7
_TRANSFORMS = {"uniform": 0, "lindisp": 1}


class _PropLossFn(th.autograd.Function):
    """mean interlevel loss of the query intervals against one proposal level; differentiable in
    the proposal's weights only."""

    @staticmethod
    def forward(ctx, key_w, key_vals, key_cdf, q_vals, q_cdf):
        lr, _ = K.prop_loss(q_vals, q_cdf, key_vals, key_cdf, _EPS)
        ctx.save_for_backward(key_vals, key_cdf, q_vals, q_cdf)
        ctx.count = q_vals.shape[0] * (q_vals.shape[1] - 1)
        return lr.sum() / ctx.count

    @staticmethod
    def backward(ctx, g):
        key_vals, key_cdf, q_vals, q_cdf = ctx.saved_tensors
        _, gw = K.prop_loss(q_vals, q_cdf, key_vals, key_cdf, _EPS, 1.0 / ctx.count, want_loss=False,
                            want_grad=True)
        return gw * g, None, None, None, None


class PropNetEstimator:
    """nerfacc.PropNetEstimator (sampling / compute_loss) restated; ``prop_cache`` holds, per level
    of the last ``requires_grad`` sampling, (s edges, weights, cdf)."""

    def __init__(self, optimizer=None, scheduler=None):
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.prop_cache: list = []

    @th.no_grad()
    def _sample(self, vals, cdf, n, stratified, sampling_type, near_plane, far_plane):
        return K.prop_sample(vals, cdf, n, stratified, _rng_seed() if stratified else 0, _TRANSFORMS[sampling_type],
                             near_plane, far_plane)

    def sampling(self, prop_sigma_fns: Sequence[Callable], prop_samples: Sequence[int], num_samples: int, n_rays: int,
                 near_plane: float, far_plane: float, sampling_type: str = "lindisp", stratified: bool = False,
                 requires_grad: bool = False):
        if sampling_type not in _TRANSFORMS:
            raise ValueError(f"sampling_type must be one of {tuple(_TRANSFORMS)}, was '{sampling_type}'")
        if len(prop_sigma_fns) != len(prop_samples):
            raise ValueError("prop_sigma_fns and prop_samples must have the same length")
        dev = th.device("cuda", th.cuda.current_device())
        vals = th.tensor([[0.0, 1.0]], device=dev).expand(n_rays, 2).contiguous()
        cdf = vals.clone()
        self.prop_cache = []
        for level_fn, level_samples in zip(prop_sigma_fns, prop_samples):
            s, t = self._sample(vals, cdf, level_samples, stratified, sampling_type, near_plane, far_plane)
            t_starts, t_ends = t[:, :-1].contiguous(), t[:, 1:].contiguous()
            with th.set_grad_enabled(requires_grad):
                sigmas = level_fn(t_starts, t_ends)
                _, w = _RenderRaysFn.apply(sigmas.reshape(n_rays, level_samples),
                                           th.zeros(n_rays, level_samples, 3, device=dev), t_ends - t_starts, 1.0, 1.0)
            cdf = K.prop_cdf(w.detach())
            if requires_grad:
                self.prop_cache.append((s, w, cdf))
            vals = s
        s, t = self._sample(vals, cdf, num_samples, stratified, sampling_type, near_plane, far_plane)
        if requires_grad:
            self.prop_cache.append((s, None, None))
        return t[:, :-1].contiguous(), t[:, 1:].contiguous()

    def compute_loss(self, trans: th.Tensor, loss_scaler: float = 1.0) -> th.Tensor:
        if len(self.prop_cache) == 0:
            return th.zeros((), device=trans.device)
        q_vals, _, _ = self.prop_cache[-1]
        if trans.dim() != 2 or tuple(trans.shape) != (q_vals.shape[0], q_vals.shape[1] - 1):
            raise ValueError(f"trans must be [{q_vals.shape[0]}, {q_vals.shape[1] - 1}] (the last sampling's "
                             f"intervals), got {tuple(trans.shape)}")
        self.prop_cache.pop()
        q_cdf = (1.0 - th.cat([trans, th.zeros_like(trans[:, :1])], dim=-1)).detach().contiguous()
        loss = th.zeros((), device=trans.device)
        while self.prop_cache:
            k_vals, k_w, k_cdf = self.prop_cache.pop()
            loss = loss + _PropLossFn.apply(k_w, k_vals, k_cdf, q_vals, q_cdf)
        return loss * loss_scaler


def rendering(t_starts: th.Tensor, t_ends: th.Tensor, ray_indices: Optional[th.Tensor] = None,
              n_rays: Optional[int] = None, rgb_sigma_fn: Optional[Callable] = None,
              render_bkgd: Optional[th.Tensor] = None):
    """nerfacc.rendering for batched [n_rays, n_samples] intervals (ray_indices must be None):
    (colors [R, 3], opacities [R, 1], depths [R, 1], extras) with extras weights / trans / sigmas /
    rgbs / alphas; trans (exclusive transmittance, 1 - the exclusive weight sum) is detached."""
    if ray_indices is not None:
        raise NotImplementedError("nerf_amd.prop_sampler.rendering supports batched (ray_indices=None) samples")
    if rgb_sigma_fn is None:
        raise ValueError("rgb_sigma_fn is required")
    rgbs, sigmas = rgb_sigma_fn(t_starts, t_ends, None)
    R, S = t_starts.shape
    delta = (t_ends - t_starts).contiguous()
    colors, weights = _RenderRaysFn.apply(sigmas.reshape(R, S), rgbs.reshape(R, S, 3), delta, 1.0, 1.0)
    trans = 1.0 - K.prop_cdf(weights.detach())[:, :S]
    with th.no_grad():
        alphas = 1.0 - th.exp(-sigmas.reshape(R, S) * delta)
    opacities = weights.sum(dim=-1, keepdim=True)
    depths = (weights * (t_starts + t_ends) / 2).sum(dim=-1, keepdim=True)
    if render_bkgd is not None:
        colors = colors + render_bkgd * (1.0 - opacities)
    return colors, opacities, depths, {"weights": weights, "trans": trans, "sigmas": sigmas, "rgbs": rgbs,
                                       "alphas": alphas}


__all__ = ["PropNetEstimator", "rendering"]
