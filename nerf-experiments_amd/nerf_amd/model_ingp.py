"""Hash-grid NeRF (config C5) on gfx950 kernels, with the reference's 3d-ingp module API.

Mirrors 3d-ingp/model.py as VERDICT r2 states its interface (the builder's round-1 read of that
file was refused; the file is not read again in any form) together with SURVEY.md §8(a) rows a7 /
a9 and the readable sibling statements of the same lineage (2d-ingp/model.py:13-115 for the tables,
naive-to-vanilla/relics/model_original.py:32-120 for the field MLP, nerf-siren/model.py:9-281 for
the renderer):

* ``INGPTable(resolution, table_size, n_features, pi1, pi2, pi3)`` — one level; its ``table``
  Parameter has (r+1)^3 rows when bijective ((r+1)^3 <= table_size) and table_size rows
  otherwise, initialised ``(th.rand(rows, n_features) * 2 - 1) * 10**-4`` (model.py:14-33).
  ``forward(x)`` on points already normalised to [0, 1): nerf_hashgrid_fwd with one level.
* ``INGPEncoding(resolution_max, resolution_min, table_size, n_features, n_levels, pi1=1,
  pi2=2654435761, pi3=805459861)`` — ``encodings`` ModuleList of INGPTables (state_dict keys
  ``encodings.{l}.table``), resolutions ``th.floor(resolution_min * b ** th.arange(n_levels))``;
  ``forward(x)`` = the levels' features of x / 8 + 0.5, concatenated (model.py:92-121).  The level
  Parameters are views of one packed buffer (re-established after ``.to()`` / ``load_state_dict``
  or any reassignment), so one kernel launch reads every level; the table gradient is the
  deterministic fixed-point nerf_hashgrid_bwd; positions (x, or the rays' origins / directions)
  receive theirs through the multilinear weights (nerf_hashgrid_bwd_pos, round 5).
* ``FourierFeatures(levels)`` — 3d-ingp's own encoding: [cos(x 2^k) | sin(x 2^k)], scale 1
  (model.py:124-148; nerf_encode_fwd kind 0).
* ``NerfModelINGP(n_hidden, hidden_dim, position_encoder, direction_encoder)`` — ``model_density``
  (Linear(enc -> h), (n_hidden - 1) x [ReLU, Linear(h -> h)], ReLU, Linear(h -> h + 1); layer1 and
  layer2 created first), ``model_color`` (Linear(h + dir -> h/2), ReLU, Linear(h/2 -> 3));
  ``forward(pos, dir) -> (density, rgb)`` with density = Softplus(threshold=8)(z[:, h] - 1) and
  rgb = sigmoid(model_color([z[:, :h] | dir])) (model.py:151-193).  The whole network runs on the
  fused MLP kernel (the hash features are its HBM-fed input).
* ``NaiveINGP(near_sphere_normalized, far_sphere_normalized, samples_per_ray_fine,
  samples_per_ray_coarse, position_encoder, direction_encoder, n_hidden, hidden_dim,
  learning_rate=1e-4, learning_rate_decay=0.5, weight_decay=0.0)`` — fine BEFORE coarse, the
  reference's positional order (model.py:196-209 as VERDICT r3 quotes it); separate
  ``model_coarse`` / ``model_fine`` sharing the encoders; stratified coarse t; positions at the
  sample t; distances = t differences plus far - t_last; compositing without a density factor;
  fine pass of samples_per_ray_coarse + samples_per_ray_fine samples from the round/argmax
  allocation (or multinomial).  ``configure_optimizers`` returns only
  ``{"optimizer": Adam(betas=(0.9, 0.99), eps=1e-15)}`` — the reference's ExponentialLR is
  commented out (model.py:503-519), so ``learning_rate_decay`` is stored but unused, as there.
  The reference's class is a ``pl.LightningModule`` whose ``training_step`` calls
  ``_step_helpher`` (model.py:480-500); this one is an ``nn.Module`` with ``training_loss`` (the
  helper without logging) — INTEGRATION.md gives the Lightning mix-in.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch as th
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import kernels as K
from . import positional_encodings as _pe
from .mlp import nerf_model_plan
from .model_interpolation import _RenderRaysFn, _rng_seed, composite_raw
from .model_interpolation_architecture import NerfBaseModel, NerfModel, RawHeads
from .optim import FusedAdam


def ingp_resolutions(n_levels: int = 16, resolution_min: int = 16, resolution_max: int = 1600) -> list[int]:
    """floor(resolution_min * b^l) in the reference's fp32 tensor arithmetic (2d-ingp/model.py:101-103)."""
    b = 1 if n_levels == 1 else math.exp((math.log(resolution_max) - math.log(resolution_min)) / (n_levels - 1))
    return [int(r) for r in th.floor(resolution_min * b ** th.arange(n_levels))]


# Hash-grid features generated inside the fused field-MLP forward (NERF_FUSE_HASH=1).  Off by default:
# bitwise equal to the stand-alone launch, but on the C5 step the forward grew by 1.9 ms against the
# 0.45 ms of the level-grid launches it replaces (the tile-start gathers of all eight waves at once,
# one level per trip; profiles/r04e)
FUSE_HASH = os.environ.get("NERF_FUSE_HASH", "0") == "1"


def _hash_spec(params, packed, out, ray_o, ray_d, t_start, t_end, samples_per_ray: int, n: int):
    """nerf_fused_encoding of kind 2: the features of ray-mode positions generated inside the fused
    field-MLP forward at every tile start (include/nerf_amd.h), bitwise as nerf_hashgrid_fwd."""
    e = _lib.NerfFusedEncoding()
    e.params = K.make_pe_params(0, 0, False, 1.0, query=params.query)
    e.params.kind = 2
    e.ray_o, e.ray_d, e.t_start = ray_o.data_ptr(), ray_d.data_ptr(), t_start.data_ptr()
    e.t_end = t_end.data_ptr() if t_end is not None else None
    e.samples_per_ray, e.n_rays, e.per_ray = samples_per_ray, n // samples_per_ray, 0
    e.out, e.ld, e.out_dim = out.data_ptr(), out.stride(0), params.levels * params.features
    e.hash = ctypes.addressof(params)
    e.hash_table = packed.data_ptr()
    return e


class _HashGridFn(th.autograd.Function):
    """Features of every level in one launch; the gradient of each level's table is a view of one
    packed fixed-point gradient (nerf_hashgrid_bwd).  defer (ray-mode positions, a table the fused
    kernel can read): the rows are left to the consuming fused field-MLP forward, which generates
    them at every tile start (kernels.DeferredEncoding; any other consumer fills them first)."""

    @staticmethod
    def forward(ctx, params, packed, rows, out_cols, x, ray_o, ray_d, t_start, t_end, samples_per_ray, n, defer,
                *tables):
        out = th.empty(n, out_cols, device=packed.device, dtype=th.float32)
        used = params.levels * params.features

        def fill(out):
            if out_cols > used:
                out[:, used:].zero_()
            K.hashgrid_fwd(params, packed, out, x=x, ray_o=ray_o, ray_d=ray_d, t_start=t_start, t_end=t_end,
                           n_samples=n, samples_per_ray=samples_per_ray)

        if (defer and FUSE_HASH and x is None and n > 0 and params.levels <= 16 and params.features in (1, 2, 4)
                and used <= 64 and out_cols <= 64 and packed.data_ptr() % 16 == 0):
            if os.environ.get("NERF_POISON_DEFERRED", "0") == "1":
                out.fill_(float("nan"))            # tests: a row read before its store fails every time
            spec = _hash_spec(params, packed, out, ray_o, ray_d, t_start, t_end, samples_per_ray, n)
            # keep: the inputs the spec points at, and the params struct its `hash` pointer names
            out._nerf_deferred = K.DeferredEncoding(spec, (ray_o, ray_d, t_start, t_end, packed, params), fill)
        else:
            fill(out)
        ctx.params = params
        ctx.rows = rows
        ctx.meta = (samples_per_ray, n, packed.shape)
        # the packed table is read back only by the position gradient: saving it otherwise would make any
        # in-place table update between forward and backward trip autograd's version check
        keep = packed if any(ctx.needs_input_grad[4:7]) else None
        ctx.save_for_backward(*(t if t is not None else th.empty(0) for t in (x, ray_o, ray_d, t_start, t_end, keep)))
        return out

    @staticmethod
    def backward(ctx, g):
        spr, n, shape = ctx.meta
        x, o, d, t0, t1, packed = (t if t.numel() else None for t in ctx.saved_tensors)
        grads = [None] * len(ctx.rows)
        gx = go = gd = None
        if g is not None and any(ctx.needs_input_grad[12:]):
            gp = th.empty(shape, device=g.device, dtype=th.float32)
            ws = th.empty((K.hashgrid_workspace_bytes(ctx.params, n) + 7) // 8, dtype=th.int64, device=g.device)
            K.hashgrid_bwd(ctx.params, g.contiguous(), gp, ws, x=x, ray_o=o, ray_d=d, t_start=t0, t_end=t1,
                           n_samples=n, samples_per_ray=spr)
            off = 0
            for l, r in enumerate(ctx.rows):
                grads[l] = gp[off:off + r]
                off += r
        # the positions' gradient through the multilinear weights (nerf_hashgrid_bwd_pos), for
        # explicit positions x or the rays' origins / directions
        if g is not None and n > 0 and any(ctx.needs_input_grad[4:7]):
            if x is not None:
                gx = K.hashgrid_bwd_pos(ctx.params, packed, g.contiguous(), x=x, n_samples=n)
            else:
                go, gd = K.hashgrid_bwd_pos(ctx.params, packed, g.contiguous(), ray_o=o, ray_d=d, t_start=t0,
                                            t_end=t1, n_samples=n, samples_per_ray=spr,
                                            want_o=ctx.needs_input_grad[5], want_d=ctx.needs_input_grad[6])
        return (None,) * 4 + (gx, go, gd) + (None,) * 5 + tuple(grads)


class INGPTable(nn.Module):
    def __init__(self, resolution, table_size, n_features, pi1, pi2, pi3):
        super().__init__()
        self.resolution = int(resolution)
        self.table_size = table_size
        self.n_features = n_features
        self.pi1 = pi1
        self.pi2 = pi2
        self.pi3 = pi3
        self.bijective = table_size >= (self.resolution + 1) ** 3
        rows = (self.resolution + 1) ** 3 if self.bijective else table_size
        self.table = nn.Parameter((th.rand((rows, n_features)) * 2 - 1) * 10 ** (-4))

    def _params(self, query: int = 1, normalize: bool = False):
        return K.make_hashgrid_params(1, self.table_size, self.n_features, [self.resolution], query,
                                      primes=(self.pi1, self.pi2, self.pi3), normalize=normalize)

    def forward(self, x: th.Tensor) -> th.Tensor:
        """Features [N, n_features] of points x [N, 3] already normalised to [0, 1)."""
        if x.dim() != 2 or x.shape[1] != 3:
            raise ValueError(f"x must be [N, 3] (got {tuple(x.shape)})")
        x = x.contiguous()
        table = self.table
        if not table.is_contiguous():
            raise ValueError("INGPTable.table must be contiguous")
        return _HashGridFn.apply(self._params(), table, [table.shape[0]], self.n_features, x, None, None, None, None,
                                 1, x.shape[0], False, table)


class INGPEncoding(nn.Module):
    def __init__(self, resolution_max, resolution_min, table_size, n_features, n_levels, pi1=1, pi2=2654435761,
                 pi3=805459861):
        super().__init__()
        self.output_dim = n_features * n_levels
        self.resolution_max = resolution_max
        self.resolution_min = resolution_min
        self.table_size = table_size
        self.n_features = n_features
        self.n_levels = n_levels
        self.pi1, self.pi2, self.pi3 = pi1, pi2, pi3
        self.space_dimensions = 3
        self.b = 1 if n_levels == 1 else math.exp((math.log(resolution_max) - math.log(resolution_min)) / (n_levels - 1))
        self.resolution = th.floor(resolution_min * self.b ** th.arange(n_levels))
        self.encodings = nn.ModuleList(
            [INGPTable(int(r), table_size, n_features, pi1, pi2, pi3) for r in self.resolution])
        self.resolutions = [e.resolution for e in self.encodings]
        self._rows = [e.table.shape[0] for e in self.encodings]
        self._packed_table = None
        self._pack()

    @property
    def padded_dim(self) -> int:
        return K.pad32(self.output_dim)

    def _params(self, query: int = 1):
        return K.make_hashgrid_params(self.n_levels, self.table_size, self.n_features, self.resolutions, query,
                                      primes=(self.pi1, self.pi2, self.pi3), normalize=True)

    # -- the level Parameters as views of one buffer -------------------------------------------
    def _aliased(self) -> bool:
        buf = self._packed_table
        if buf is None:
            return False
        F_ = self.n_features
        off = 0
        for e, rows in zip(self.encodings, self._rows):
            t = e.table
            if (t.device != buf.device or t.dtype != th.float32 or t.shape != (rows, F_) or not t.is_contiguous()
                    or t.data_ptr() != buf.data_ptr() + off * F_ * 4):
                return False
            off += rows
        return True

    def _pack(self) -> th.Tensor:
        """The packed [sum rows, F] table the kernels read; re-points the level Parameters at it
        when a conversion, load or reassignment has separated them (a device copy, no sync)."""
        if self._aliased():
            return self._packed_table
        t0 = self.encodings[0].table
        buf = th.empty(sum(self._rows), self.n_features, device=t0.device, dtype=th.float32)
        off = 0
        with th.no_grad():
            for e, rows in zip(self.encodings, self._rows):
                view = buf[off:off + rows]
                view.copy_(e.table)
                e.table.data = view
                off += rows
        self._packed_table = buf
        return buf

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        self._pack()
        return out

    def packed_table(self) -> th.Tensor:
        return self._pack()

    def _run(self, x, ray_o, ray_d, t_start, t_end, samples_per_ray, query, n, defer=False):
        packed = self._pack()
        tables = [e.table for e in self.encodings]
        return _HashGridFn.apply(self._params(query), packed, self._rows, K.pad32(self.output_dim), x, ray_o, ray_d,
                                 t_start, t_end, samples_per_ray, n, defer, *tables)

    # -- kernel-facing API (the NerfModel lowering's encoder interface) -------------------------
    def encode_padded(self, x: th.Tensor, dir=None, pixel_width=None, t_start=None, t_end=None,
                      defer: bool = False) -> th.Tensor:
        """[N, pad32(output_dim)] features of explicit positions x [N, 3] (defer: accepted, ignored —
        only ray-mode positions are generated inside the fused MLP)."""
        if x.dim() != 2 or x.shape[1] != 3:
            raise ValueError(f"x must be [N, 3] (got {tuple(x.shape)})")
        x = x.contiguous()
        return self._run(x, None, None, None, None, 1, 1, x.shape[0])

    def encode_rays(self, ray_origs, ray_dirs, t_start, t_end, pixel_width, samples_per_ray: int, query: int,
                    pw_mode: int = 0, defer: bool = False) -> th.Tensor:
        """Features of the samples o + t_q d generated in-kernel (rays that require grad get their
        gradient through the multilinear weights, nerf_hashgrid_bwd_pos); defer: the rows may be
        generated by the consuming fused field-MLP forward itself (only for a tensor handed straight
        to the field MLP, as PositionalEncoding.encode_rays)."""
        n = t_start.numel()
        return self._run(None, ray_origs.contiguous(), ray_dirs.contiguous(),
                         t_start.detach().contiguous(), t_end.detach().contiguous(), samples_per_ray, query, n,
                         defer)

    # -- reference API ----------------------------------------------------------------------------
    def forward(self, x: th.Tensor, dir=None, pixel_width=None, t_start=None, t_end=None) -> th.Tensor:
        return self.encode_padded(x)[:, :self.output_dim]


class FourierFeatures(_pe.FourierFeatures):
    """3d-ingp's FourierFeatures(levels): [cos(x 2^k) | sin(x 2^k)] (d-major), scale 1, no pi."""

    def __init__(self, levels: int):
        super().__init__(levels, 1.0)


class NerfModelINGP(NerfModel):
    DENSITY_SHIFT = 1.0

    def __init__(self, n_hidden: int, hidden_dim: int, position_encoder, direction_encoder):
        NerfBaseModel.__init__(self)
        self.n_hidden = n_hidden
        self.hidden_dim = hidden_dim
        self.position_encoder = position_encoder
        self.direction_encoder = direction_encoder
        self.model_density = self.contruct_model_density(position_encoder.output_dim, hidden_dim, hidden_dim + 1)
        self.model_color = nn.Sequential(
            nn.Linear(hidden_dim + direction_encoder.output_dim, hidden_dim // 2),
            nn.ReLU(inplace=True),
            nn.Linear(hidden_dim // 2, 3),
        )
        self.relu = nn.ReLU(inplace=True)
        self.softplus = nn.Softplus(threshold=8)
        self.sigmoid = nn.Sigmoid()
        # the NerfModel lowering: one segment, direction at the colour head, density = trunk column h
        self.delayed_direction = True
        self.delayed_density = False
        self.n_segments = 1
        self._plan = None

    def _get_plan(self):
        if self._plan is None:
            self._plan, self._z_last, self._head_out = nerf_model_plan(
                1, [self.model_density], self.model_color, self.hidden_dim, self.position_encoder.output_dim,
                self.direction_encoder.output_dim, True, False)
        return self._plan

    def list_segments(self):
        print(f"Density: {self.model_density}")
        print(f"Final layer: {self.model_color}")

    def _heads(self, z_last, head, dens) -> RawHeads:
        return RawHeads(head, dens.view(-1, 1), 0, self.DENSITY_SHIFT)

    def forward(self, pos: th.Tensor, dir: th.Tensor, pixel_width=None, t_start=None, t_end=None):
        pos_pe = self.position_encoder.encode_padded(pos)
        dir_pe = self.direction_encoder.encode_padded(dir)
        z_last, head, dens = self._run_mlp(pos_pe, dir_pe, 1)
        density = F.softplus(dens - self.DENSITY_SHIFT, beta=1, threshold=8)
        rgb = th.sigmoid(head[:, :3])
        return density, rgb


class NaiveINGP(nn.Module):
    def __init__(self, near_sphere_normalized: float, far_sphere_normalized: float, samples_per_ray_fine: int,
                 samples_per_ray_coarse: int, position_encoder, direction_encoder, n_hidden: int, hidden_dim: int,
                 learning_rate: float = 1e-4, learning_rate_decay: float = 0.5, weight_decay: float = 0.0):
        super().__init__()
        self.near_sphere_normalized = near_sphere_normalized
        self.far_sphere_normalized = far_sphere_normalized
        self.samples_per_ray_coarse = samples_per_ray_coarse
        self.samples_per_ray_fine = samples_per_ray_fine
        self.learning_rate = learning_rate
        self.learning_rate_decay = learning_rate_decay
        self.weight_decay = weight_decay
        self.model_coarse = NerfModelINGP(n_hidden, hidden_dim, position_encoder, direction_encoder)
        self.model_fine = NerfModelINGP(n_hidden, hidden_dim, position_encoder, direction_encoder)
        # bit 0: the fine allocation fell back to equidistant samples; bit 1: a multinomial row was
        # not a distribution (nerf_resample_pdf; device int32, read only if the caller wants it)
        self.last_resample_status: th.Tensor | None = None

    @property
    def device(self) -> th.device:
        return next(self.parameters()).device

    # ---------------------------------------------------------------- sampling
    def _sample_t_coarse(self, batch_size: int) -> th.Tensor:
        """linspace(near, far - D, S) + U[0, 1) * D, D = (far - near) / S (Philox draws)."""
        t, _ = K.sample_uniform(batch_size, self.samples_per_ray_coarse, self.near_sphere_normalized,
                                self.far_sphere_normalized, True, 0.0, _rng_seed(), 0, self.device)
        return t

    def _sample_t_fine(self, t_coarse: th.Tensor, weights: th.Tensor, distances_coarse: th.Tensor,
                       linspace: bool = True) -> th.Tensor:
        """[batch, coarse + fine] sample t: round(w * fine) per bin with the remainder on the first
        argmax bin, +1 (the coarse point), spread evenly over each bin (linspace=True); or fine
        multinomial draws jittered within their bins, joined with t_coarse and sorted."""
        if weights.dim() == 3:
            weights = weights.squeeze(2)
        t0, _, status = K.resample_pdf(t_coarse.detach(), weights.detach(), distances_coarse.detach(),
                                       self.samples_per_ray_coarse + self.samples_per_ray_fine, 1 if linspace else 2,
                                       self.near_sphere_normalized, self.far_sphere_normalized, _rng_seed(), 0)
        self.last_resample_status = status
        return t0

    def _intervals(self, t: th.Tensor) -> th.Tensor:
        t_end = th.empty_like(t)
        t_end[:, :-1] = t[:, 1:]
        t_end[:, -1] = self.far_sphere_normalized
        return t_end

    def _compute_positions(self, origins: th.Tensor, directions: th.Tensor, t: th.Tensor):
        """(positions o + t d [B, S, 3], directions [B, S, 3], distances [B, S]: t differences and
        far - t_last)."""
        positions = origins.unsqueeze(1) + t.unsqueeze(2) * directions.unsqueeze(1)
        distances = self._intervals(t) - t
        directions = directions.unsqueeze(1).repeat(1, positions.shape[1], 1)
        return positions, directions, distances

    # ---------------------------------------------------------------- rendering
    def _render_rays(self, densities: th.Tensor, colors: th.Tensor, distances: th.Tensor):
        """(rgb [B, 3], weights [B, S, 1]); no density factor in 3d-ingp's compositor."""
        rgb, w = _RenderRaysFn.apply(densities, colors, distances, 1.0, 1.0)
        return rgb, w.unsqueeze(-1)

    def _compute_color(self, model, t: th.Tensor, ray_origs: th.Tensor, ray_dirs: th.Tensor, batch_size: int,
                       samples_per_ray: int):
        t = t.contiguous()
        t_end = self._intervals(t)
        sample_dist = t_end - t
        if isinstance(model, NerfModel):
            # fused: positions o + t d generated in the encoding kernel, direction encoding once per
            # ray, softplus(z - 1) / sigmoid applied in the compositor — inside the field MLP's
            # launches when the rays fill its tiles (the 64-sample coarse pass) or span two of them
            # (the 256-sample fine pass: a workgroup runs a ray's two tiles back to back)
            if model.fused_composite_ok(batch_size * samples_per_ray, samples_per_ray):
                rgb, weights = model.render_composite(ray_origs, ray_dirs, None, t, t_end, samples_per_ray, 0, 1,
                                                      sample_dist, 1.0, 1.0)
                return rgb, weights.unsqueeze(-1), sample_dist
            heads = model.render_raw(ray_origs, ray_dirs, None, t, t_end, samples_per_ray, 0, 1)
            rgb, weights = composite_raw(heads, sample_dist, batch_size, samples_per_ray, 1.0, 1.0)
            return rgb, weights.unsqueeze(-1), sample_dist
        sample_pos, sample_dir, _ = self._compute_positions(ray_origs, ray_dirs, t)
        density, color = model(sample_pos.view(batch_size * samples_per_ray, 3),
                               sample_dir.reshape(batch_size * samples_per_ray, 3))
        rgb, weights = self._render_rays(density.view(batch_size, samples_per_ray),
                                         color.view(batch_size, samples_per_ray, 3), sample_dist)
        return rgb, weights, sample_dist

    def forward(self, ray_origs: th.Tensor, ray_dirs: th.Tensor):
        """(rgb_fine, rgb_coarse) [B, 3] each."""
        batch_size = ray_origs.shape[0]
        t_coarse = self._sample_t_coarse(batch_size)
        rgb_coarse, weights, sample_dist_coarse = self._compute_color(
            self.model_coarse, t_coarse, ray_origs, ray_dirs, batch_size, self.samples_per_ray_coarse)
        t_fine = self._sample_t_fine(t_coarse, weights, sample_dist_coarse)
        rgb_fine, _, _ = self._compute_color(self.model_fine, t_fine, ray_origs, ray_dirs, batch_size,
                                             self.samples_per_ray_coarse + self.samples_per_ray_fine)
        return rgb_fine, rgb_coarse

    # ---------------------------------------------------------------- training helpers
    def training_loss(self, ray_origs: th.Tensor, ray_dirs: th.Tensor, ray_colors: th.Tensor):
        """MSE(coarse) + MSE(fine) of the step helper, without Lightning logging or syncs."""
        fine, coarse = self(ray_origs, ray_dirs)
        loss_coarse = nn.functional.mse_loss(coarse, ray_colors)
        loss_fine = nn.functional.mse_loss(fine, ray_colors)
        return loss_coarse + loss_fine, {"loss_coarse": loss_coarse.detach(), "loss_fine": loss_fine.detach()}

    def configure_optimizers(self):
        params = list(self.parameters())
        opt_cls = FusedAdam if all(p.is_cuda for p in params) else th.optim.Adam
        optimizer = opt_cls(params, lr=self.learning_rate, betas=(0.9, 0.99), eps=1e-15,
                            weight_decay=self.weight_decay)
        # no scheduler: the reference's ExponentialLR(gamma=learning_rate_decay) is commented out
        # (3d-ingp/model.py:503-519), so its learning rate stays constant
        return {"optimizer": optimizer}
