"""Positional encodings on gfx950 kernels, with the reference module API.

Mirrors barf/positional_encodings.py (class names, constructor arguments,
``output_dim`` / ``space_dimensions`` / ``levels`` / ``alpha`` attributes,
``forward(x, dir, pixel_width, t_start, t_end)``, ``update_alpha`` and
``compute_mask``).  The encoding itself runs in ``nerf_encode_fwd`` /
``nerf_encode_bwd`` (csrc/encode.hip); the BARF coarse-to-fine mask is computed
on the host from a host-side copy of alpha, so the reference's per-call
``int(alpha)`` device sync (positional_encodings.py:110) is gone.

Besides the reference API, every encoder exposes
  * ``padded_dim``      — output width rounded up to 32 (the MLP kernels' K tile);
  * ``encode_padded``   — [N, padded_dim] encoding (pad columns are zero);
  * ``encode_rays``     — the same, with sample positions generated in-kernel
                          from rays and t intervals (fuses _compute_positions).
"""
from __future__ import annotations

from typing import Optional

import torch as th
import torch.nn as nn

from . import kernels as K


class _EncodeFn(th.autograd.Function):
    """x [N,3] (+ IPE side inputs) -> padded encoding.

    Backward: d/dx for every encoding (nerf_encode_bwd, kind 0; nerf_encode_bwd_integrated,
    kind 1) and d/d(dir) for the integrated encodings, whose output depends on the direction
    through the mean shift and the diagonal variance (positional_encodings.py:190-226) — the
    gradient BARF-style pose refinement needs.  Fourier/BARF encodings ignore dir."""

    @staticmethod
    def forward(ctx, x, xdir, pixel_width, t_start, t_end, enc: "PositionalEncoding", defer: bool = False):
        params = enc._pe_params(query=1, pw_mode=2)
        n = x.shape[0]
        out = K.encode_fwd(params, enc.output_dim, x=x, xdir=xdir, t_start=t_start, t_end=t_end,
                           pixel_width=pixel_width, n_samples=n, samples_per_ray=1, n_rays=n,
                           out_ld=enc.padded_dim, device=x.device, defer=defer)
        ctx.params = params
        ctx.kind = params.kind
        if params.kind == 1:
            ctx.save_for_backward(x, xdir, pixel_width, t_start, t_end)
        else:
            ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, g):
        if any(ctx.needs_input_grad[2:5]):
            raise NotImplementedError("nerf_amd encodings do not propagate gradients to pixel_width / t")
        dx = ddir = None
        if ctx.kind == 1:
            x, xdir, pw, t0, t1 = ctx.saved_tensors
            if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
                dx, ddir = K.encode_bwd_integrated(ctx.params, x, xdir, t0, t1, pw, g, ctx.needs_input_grad[0],
                                                   ctx.needs_input_grad[1])
        elif ctx.needs_input_grad[0]:
            (x,) = ctx.saved_tensors
            dx = K.encode_bwd(ctx.params, x, g)
        return dx, ddir, None, None, None, None, None


class _EncodeRaysFn(th.autograd.Function):
    """Encoding of o + t_query * d for every (ray, sample), positions generated in-kernel
    (fuses _compute_positions, model_interpolation.py:288-312).  Backward: dL/d origins and
    dL/d directions per ray (nerf_encode_bwd_rays) — BARF pose refinement's gradient path."""

    @staticmethod
    def forward(ctx, ray_o, ray_d, t_start, t_end, pixel_width, enc: "PositionalEncoding", samples_per_ray: int,
                query: int, pw_mode: int, defer: bool = False):
        params = enc._pe_params(query=query, pw_mode=pw_mode)
        n_rays = ray_o.shape[0]
        out = K.encode_fwd(params, enc.output_dim, ray_o=ray_o, ray_d=ray_d, t_start=t_start, t_end=t_end,
                           pixel_width=pixel_width, n_samples=n_rays * samples_per_ray,
                           samples_per_ray=samples_per_ray, n_rays=n_rays, out_ld=enc.padded_dim,
                           device=ray_o.device, defer=defer)
        ctx.params = params
        ctx.S = samples_per_ray
        ctx.has_pw = pixel_width is not None
        ctx.save_for_backward(ray_o, ray_d, t_start, t_end, pixel_width if pixel_width is not None else ray_o)
        return out

    @staticmethod
    def backward(ctx, g):
        if any(ctx.needs_input_grad[2:5]):
            raise NotImplementedError("nerf_amd encodings do not propagate gradients to t / pixel_width")
        ray_o, ray_d, t0, t1, pw = ctx.saved_tensors
        d_o = d_d = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            d_o, d_d = K.encode_bwd_rays(ctx.params, ray_o, ray_d, t0, t1, pw if ctx.has_pw else None, g, ctx.S,
                                         ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return d_o, d_d, None, None, None, None, None, None, None, None


def _as_rows(t, n: int, device=None) -> th.Tensor | None:
    if t is None:
        return None
    if isinstance(t, (int, float)):
        return th.full((n,), float(t), device=device, dtype=th.float32)
    t = t.reshape(-1)
    if t.numel() == 1 and n != 1:
        t = t.expand(n)
    return t.contiguous().float()


class PositionalEncoding(nn.Module):
    def __init__(self):
        super().__init__()
        self.output_dim = None
        self.space_dimensions = None

    @property
    def padded_dim(self) -> int:
        return K.pad32(self.output_dim)

    def _pe_params(self, query: int = 1, pw_mode: int = 2):
        raise NotImplementedError()

    # -- reference API ---------------------------------------------------------------
    def forward(self, x: th.Tensor, dir: th.Tensor | None = None, pixel_width: th.Tensor | None = None,
                t_start: th.Tensor | None = None, t_end: th.Tensor | None = None) -> th.Tensor:
        return self.encode_padded(x, dir, pixel_width, t_start, t_end)[:, : self.output_dim]

    # -- kernel-facing API -------------------------------------------------------------
    def _check_x(self, x: th.Tensor) -> None:
        if x.dim() != 2 or x.shape[1] != self.space_dimensions:
            raise ValueError(f"Input shape {tuple(x.shape)} does not match space dimensionality "
                             f"{self.space_dimensions}")

    def encode_padded(self, x, dir=None, pixel_width=None, t_start=None, t_end=None, defer: bool = False) -> th.Tensor:
        """defer: the rows may be left to the consuming fused field-MLP kernel (kernels.encode_fwd);
        only for a tensor handed straight to the field MLP."""
        self._check_x(x)
        n = x.shape[0]
        x = x.contiguous()
        return _EncodeFn.apply(x, dir.contiguous() if dir is not None else None,
                               _as_rows(pixel_width, n, x.device), _as_rows(t_start, n, x.device),
                               _as_rows(t_end, n, x.device), self, defer)

    def encode_rays(self, ray_origs: th.Tensor, ray_dirs: th.Tensor, t_start: th.Tensor, t_end: th.Tensor,
                    pixel_width: th.Tensor | None, samples_per_ray: int, query: int, pw_mode: int,
                    defer: bool = False) -> th.Tensor:
        """Encoding of o + t_query*d for every (ray, sample); differentiable w.r.t. the rays.  defer: as
        encode_padded."""
        pw = None
        if isinstance(self, (IntegratedFourierFeatures, IntegratedBarfFourierFeatures)):
            pw = pixel_width.reshape(-1).contiguous().float()
        return _EncodeRaysFn.apply(ray_origs.contiguous(), ray_dirs.contiguous(), t_start.contiguous(),
                                   t_end.contiguous(), pw, self, samples_per_ray, query, pw_mode, defer)


class IdentityPositionalEncoding(PositionalEncoding):
    def __init__(self, space_dimensions: int = 3):
        super().__init__()
        self.output_dim = space_dimensions
        self.space_dimensions = space_dimensions
        if space_dimensions != 3:
            raise ValueError("nerf_amd encodings support 3-D inputs only")

    def _pe_params(self, query: int = 1, pw_mode: int = 2):
        return K.make_pe_params(0, 0, True, 1.0, query=query)


class FourierFeatures(PositionalEncoding):
    """[cos(x*s*2^k) (d-major) | sin(...)]; barf/positional_encodings.py:28-57."""

    def __init__(self, levels: int, scale: float = 2 * th.pi, space_dimensions: int = 3):
        super().__init__()
        if space_dimensions != 3:
            raise ValueError("nerf_amd encodings support 3-D inputs only")
        self.levels = levels
        self.scale = scale
        self.space_dimensions = space_dimensions
        self.output_dim = levels * 2 * space_dimensions

    def _pe_params(self, query: int = 1, pw_mode: int = 2):
        return K.make_pe_params(0, self.levels, False, float(self.scale), query=query)


def barf_mask_values(alpha: float, levels: int) -> list[float]:
    """BarfPositionalEncoding.compute_mask (positional_encodings.py:105-122) in the
    reference's fp32 arithmetic, on host scalars."""
    a = th.tensor(float(alpha), dtype=th.float32)
    mask = th.zeros(levels, dtype=th.float32)
    idx_ramp = int(a)
    mask[:idx_ramp] = 1.0
    if idx_ramp < levels:
        mask[idx_ramp] = (1 - th.cos((a - idx_ramp) * th.pi)) / 2
    return mask.tolist()


class BarfPositionalEncoding(PositionalEncoding):
    """[x | m_k*cos | m_k*sin]; barf/positional_encodings.py:61-148."""

    def __init__(self, levels: int, alpha_start: float, alpha_increase_start_epoch: float,
                 alpha_increase_end_epoch: float, include_identity: bool = True, scale: float = 2 * th.pi,
                 space_dimensions: int = 3):
        super().__init__()
        if space_dimensions != 3:
            raise ValueError("nerf_amd encodings support 3-D inputs only")
        self.levels = levels
        self.alpha_start = alpha_start
        self.output_dim = (levels * 2 + include_identity) * space_dimensions
        self.alpha_increase_start_epoch = alpha_increase_start_epoch
        self.alpha_increase_end_epoch = alpha_increase_end_epoch
        self.include_identity = include_identity
        self.scale = scale
        self.space_dimensions = space_dimensions
        self.register_buffer("alpha", th.tensor(float(alpha_start)))
        self._alpha_host = float(th.tensor(float(alpha_start), dtype=th.float32))
        self._alpha_seen = (self.alpha, self.alpha._version)

    def update_alpha(self, epoch: float) -> None:
        if epoch < self.alpha_increase_start_epoch:
            alpha = self.alpha_start
        elif self.alpha_increase_start_epoch <= epoch < self.alpha_increase_end_epoch:
            alpha = (self.alpha_start + (epoch - self.alpha_increase_start_epoch) * (self.levels - self.alpha_start)
                     / (self.alpha_increase_end_epoch - self.alpha_increase_start_epoch))
        else:
            alpha = float(self.levels)
        # device-side buffer kept for state_dict compatibility; fill_ enqueues, never syncs
        self.alpha.fill_(float(alpha))
        self._alpha_host = float(th.tensor(float(alpha), dtype=th.float32))
        self._alpha_seen = (self.alpha, self.alpha._version)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)
        key = prefix + "alpha"
        if key in state_dict:
            self._alpha_host = float(state_dict[key].float().cpu())
            self._alpha_seen = (self.alpha, self.alpha._version)

    def _sync_alpha_host(self) -> None:
        """Refresh the host mirror of alpha after a write that bypassed update_alpha: assigning a new
        tensor (``enc.alpha = th.tensor(a)``, what the reference's own update_alpha does) or an
        in-place write (``enc.alpha.fill_(a)``, ``.to()``/``_apply`` moves).  Detected by the buffer's
        identity and version counter (a host-side check; the device read happens only then).  The
        last-seen tensor is held by reference and compared with ``is``: a freed tensor's id() can be
        reused by the next one, a live one's cannot."""
        seen, version = self._alpha_seen
        if self.alpha is not seen or self.alpha._version != version:
            self._alpha_host = float(self.alpha.detach().float().cpu())
            self._alpha_seen = (self.alpha, self.alpha._version)

    def compute_mask(self, alpha: th.Tensor) -> th.Tensor:
        vals = barf_mask_values(float(alpha), self.levels)
        return th.tensor(vals * self.space_dimensions, device=alpha.device).view(1, -1)

    def mask_values(self) -> list[float]:
        self._sync_alpha_host()
        return barf_mask_values(self._alpha_host, self.levels)

    def _pe_params(self, query: int = 1, pw_mode: int = 2):
        return K.make_pe_params(0, self.levels, self.include_identity, float(self.scale), query=query,
                                mask=self.mask_values())


class IntegratedFourierFeatures(PositionalEncoding):
    """mip-NeRF integrated encoding; barf/positional_encodings.py:151-240."""

    def __init__(self, levels: int, scale: float = 2 * th.pi, include_identity=True,
                 distribute_variance: Optional[bool] = False):
        super().__init__()
        self.levels = levels
        self.space_dimensions = 3
        self.scale = scale
        self.include_identity = include_identity
        self.output_dim = (levels * 2 + include_identity) * self.space_dimensions
        self.distribute_variance = distribute_variance
        self.pixel_width_sigma = None

    def _pws(self) -> float:
        if self.pixel_width_sigma is None:
            # the reference compares None > 0.25 here and raises TypeError (positional_encodings.py:204)
            raise TypeError("IntegratedFourierFeatures.pixel_width_sigma must be set before use")
        return float(self.pixel_width_sigma)

    def _mask(self):
        return None

    def _pe_params(self, query: int = 1, pw_mode: int = 2):
        return K.make_pe_params(1, self.levels, self.include_identity, float(self.scale), query=query,
                                pixel_width_sigma=self._pws(), distribute_variance=bool(self.distribute_variance),
                                pw_mode=pw_mode, mask=self._mask())

    def encode_padded(self, x, dir=None, pixel_width=None, t_start=None, t_end=None, defer: bool = False) -> th.Tensor:
        if dir is None or pixel_width is None or t_start is None or t_end is None:
            raise ValueError("integrated encodings need dir, pixel_width, t_start and t_end")
        if x.dim() != 2 or x.shape[1] != 3:
            raise ValueError(f"Only 3D supported - was {x.shape[1] if x.dim() == 2 else x.dim()}D")
        return PositionalEncoding.encode_padded(self, x, dir, pixel_width, t_start, t_end, defer)


class IntegratedBarfFourierFeatures(BarfPositionalEncoding):
    """BARF-masked integrated encoding; barf/positional_encodings.py:242-282."""

    def __init__(self, levels: int, alpha_start: float, alpha_increase_start_epoch: float,
                 alpha_increase_end_epoch: float, include_identity: bool = True, scale: float = 2 * th.pi,
                 distribute_variance=True):
        BarfPositionalEncoding.__init__(self, levels=levels, alpha_start=alpha_start,
                                        alpha_increase_start_epoch=alpha_increase_start_epoch,
                                        alpha_increase_end_epoch=alpha_increase_end_epoch,
                                        include_identity=include_identity, scale=scale, space_dimensions=3)
        self.distribute_variance = distribute_variance
        self.pixel_width_sigma = None

    def _pe_params(self, query: int = 1, pw_mode: int = 2):
        return K.make_pe_params(1, self.levels, self.include_identity, float(self.scale), query=query,
                                pixel_width_sigma=IntegratedFourierFeatures._pws(self),
                                distribute_variance=bool(self.distribute_variance), pw_mode=pw_mode,
                                mask=self.mask_values())

    encode_padded = IntegratedFourierFeatures.encode_padded


__all__ = ["PositionalEncoding", "IdentityPositionalEncoding", "FourierFeatures", "BarfPositionalEncoding",
           "IntegratedFourierFeatures", "IntegratedBarfFourierFeatures", "barf_mask_values"]
