"""NerfModel on gfx950 kernels, with the reference module API and parameter layout.

Mirrors barf/model_interpolation_architecture.py:11-168: same constructor,
same submodule names and construction order (``model_segments.{i}.{j}``,
``model_color.{0,2}``; layer1 and layer2 are created before the intermediate
layers, so ``th.manual_seed`` gives the reference's initial weights), same
``param_groups`` and ``forward(pos, dir, pixel_width, t_start, t_end) ->
(density[N], rgb[N, 3])``.  The forward runs the encoders' kernels and one
``MLPFunction`` node (fp32 MFMA linear kernels); activations of the heads are
applied with the reference's semantics (Softplus(threshold=8), Sigmoid).

``render_raw`` is the fused entry used by the renderer: encodings are computed
from rays in-kernel, the direction encoding once per ray, and the raw head
outputs are handed to the compositing kernel which applies the activations.
"""
from __future__ import annotations

import os
from typing import Iterator, Literal

import torch as th
import torch.nn as nn
import torch.nn.functional as F
from .mlp import CompositeSpec, MLPFunction, composite_eligible, nerf_model_plan
from .positional_encodings import PositionalEncoding

# encodings generated inside the fused field-MLP kernel (NERF_FUSE_ENC=0: stand-alone encoding
# launches, for A/B timing; results are bitwise the same)
FUSE_ENCODINGS = os.environ.get("NERF_FUSE_ENC", "1") != "0"


class NerfBaseModel(nn.Module):
    def __init__(self):
        super().__init__()
        self.param_groups: list[dict[Literal["parameters", "learning_rate_start", "learning_rate_stop",
                                             "learning_rate_decay_end", "weight_decay"], float]] = []

    def _add_param_group(self, parameters: Iterator, learning_rate_start: float, learning_rate_stop: float,
                         learning_rate_decay_end: float, weight_decay: float = 0.0):
        self.param_groups.append({
            "parameters": parameters,
            "learning_rate_start": learning_rate_start,
            "learning_rate_stop": learning_rate_stop,
            "learning_rate_decay_end": learning_rate_decay_end,
            "weight_decay": weight_decay,
        })


class RawHeads:
    """Where a field MLP's raw (pre-activation) outputs live, for the compositor:
    rgb in columns 0..2 of ``color_base``, density in column ``dens_col`` of
    ``dens_base`` (possibly the same buffer); sigma = softplus(raw - density_shift)."""

    __slots__ = ("color_base", "dens_base", "dens_col", "density_shift")

    def __init__(self, color_base, dens_base, dens_col, density_shift=0.0):
        self.color_base = color_base
        self.dens_base = dens_base
        self.dens_col = dens_col
        self.density_shift = density_shift


class NerfModel(NerfBaseModel):
    def __init__(self, n_hidden: int, hidden_dim: int, delayed_direction: bool, delayed_density: bool,
                 n_segments: int, position_encoder: PositionalEncoding, direction_encoder: PositionalEncoding,
                 learning_rate_start: float = 5e-4, learning_rate_stop: float = 5e-5,
                 learning_rate_decay_end: float = 0):
        NerfBaseModel.__init__(self)
        self.n_hidden = n_hidden
        self.hidden_dim = hidden_dim
        self.delayed_direction = delayed_direction
        self.delayed_density = delayed_density
        self.n_segments = n_segments
        self.position_encoder = position_encoder
        self.direction_encoder = direction_encoder

        positional_dim = self.position_encoder.output_dim
        directional_dim = self.direction_encoder.output_dim

        self.model_segments = nn.ModuleList()
        if n_segments == 0:
            raise NotImplementedError("n_segments must be greater than 0")
        for i in range(self.n_segments):
            input_size = positional_dim + (not self.delayed_direction) * directional_dim + (i > 0) * self.hidden_dim
            out = self.hidden_dim + (not self.delayed_density) * (i == self.n_segments - 1)
            self.model_segments.append(self.contruct_model_density(input_size, self.hidden_dim, out))

        self.model_color = nn.Sequential(
            nn.Linear(self.hidden_dim + self.delayed_direction * directional_dim, self.hidden_dim // 2),
            nn.ReLU(inplace=True),
            nn.Linear(self.hidden_dim // 2, 3 + self.delayed_density),
        )
        self.relu = nn.ReLU(inplace=True)
        self.softplus = nn.Softplus(threshold=8)
        self.sigmoid = nn.Sigmoid()

        self._add_param_group(self.parameters(), learning_rate_start, learning_rate_stop, learning_rate_decay_end)
        self._plan = None

    def contruct_model_density(self, input_dim: int, hidden_dim: int, output_dim: int) -> nn.Module:
        if self.n_hidden == 0:
            return nn.Linear(input_dim, output_dim)
        layer1 = nn.Linear(input_dim, hidden_dim)
        layer2 = nn.Linear(hidden_dim, output_dim)
        intermediate_layers = []
        for _ in range(self.n_hidden - 1):
            intermediate_layers += [nn.ReLU(True), nn.Linear(hidden_dim, hidden_dim)]
        return nn.Sequential(layer1, *intermediate_layers, nn.ReLU(True), layer2)

    def list_segments(self):
        for i, segment in enumerate(self.model_segments):
            print(f"Segment {i}: {segment}")
        print(f"Final layer: {self.model_color}")

    # ------------------------------------------------------------------------------
    def _get_plan(self):
        if self._plan is None:
            self._plan, self._z_last, self._head_out = nerf_model_plan(
                self.n_segments, self.model_segments, self.model_color, self.hidden_dim,
                self.position_encoder.output_dim, self.direction_encoder.output_dim,
                self.delayed_direction, self.delayed_density)
        return self._plan

    def _run_mlp(self, pos_pe: th.Tensor, dir_pe: th.Tensor, dir_row_div: int):
        """(z_last, head, raw density [M] or None): without delayed density the density column
        comes out of the MLP node as its own contiguous output."""
        plan = self._get_plan()
        M = pos_pe.shape[0]
        outs = MLPFunction.apply(plan, M, pos_pe, dir_pe, dir_row_div, *plan.params())
        return outs[0], outs[1], (outs[2] if len(outs) > 2 else None)

    def _heads(self, z_last: th.Tensor, head: th.Tensor, dens: th.Tensor | None) -> RawHeads:
        if self.delayed_density:
            return RawHeads(head, head, 3)
        return RawHeads(head, dens.view(-1, 1), 0)

    def forward(self, pos: th.Tensor, dir: th.Tensor, pixel_width: th.Tensor, t_start: th.Tensor,
                t_end: th.Tensor) -> tuple[th.Tensor, th.Tensor]:
        pos_pe = self.position_encoder.encode_padded(pos, dir, pixel_width, t_start, t_end)
        dir_pe = self.direction_encoder.encode_padded(dir)
        z_last, head, dens = self._run_mlp(pos_pe, dir_pe, 1)
        density = head[:, 3] if self.delayed_density else dens
        density = F.softplus(density, beta=1, threshold=8)
        rgb = th.sigmoid(head[:, :3])
        return density, rgb

    def render_raw(self, ray_origs: th.Tensor, ray_dirs: th.Tensor, pixel_width: th.Tensor | None,
                   t_start: th.Tensor, t_end: th.Tensor, samples_per_ray: int, query: int,
                   pw_mode: int) -> RawHeads:
        """Raw head outputs for every (ray, sample); positions generated in-kernel.  Differentiable
        w.r.t. ray_origs / ray_dirs (pose refinement): the position encoding's ray-mode backward plus
        the per-ray direction encoding's backward."""
        # both encodings go straight to the field MLP: their rows may be generated inside the fused
        # kernel (kernels.encode_fwd(defer=True); MLPFunction fills them itself on any other path)
        pos_pe = self.position_encoder.encode_rays(ray_origs, ray_dirs, t_start, t_end, pixel_width,
                                                   samples_per_ray, query, pw_mode, defer=FUSE_ENCODINGS)
        dir_pe = self.direction_encoder.encode_padded(ray_dirs, defer=FUSE_ENCODINGS)
        z_last, head, dens = self._run_mlp(pos_pe, dir_pe, samples_per_ray)
        return self._heads(z_last, head, dens)

    def fused_composite_ok(self, n_samples: int, samples_per_ray: int) -> bool:
        """render_composite can run these rays (nerf_mlp_fused_render: split precision, whole rays
        per 128-sample tile)."""
        return composite_eligible(self._get_plan(), n_samples, samples_per_ray)

    def render_composite(self, ray_origs: th.Tensor, ray_dirs: th.Tensor, pixel_width: th.Tensor | None,
                         t_start: th.Tensor, t_end: th.Tensor, samples_per_ray: int, query: int, pw_mode: int,
                         distances: th.Tensor, scale_a: float, scale_b: float) -> tuple[th.Tensor, th.Tensor]:
        """render_raw followed by the renderer's compositing (_render_rays on the activated heads,
        barf/model_interpolation.py:316-353), both inside the field MLP's launches: (rgb [B, 3],
        weights [B, S]); rgb and weights bitwise those of composite_raw, weights non-differentiable."""
        pos_pe = self.position_encoder.encode_rays(ray_origs, ray_dirs, t_start, t_end, pixel_width,
                                                   samples_per_ray, query, pw_mode, defer=FUSE_ENCODINGS)
        dir_pe = self.direction_encoder.encode_padded(ray_dirs, defer=FUSE_ENCODINGS)
        plan = self._get_plan()
        # (NerfModelINGP's density is softplus(z - 1): its DENSITY_SHIFT, applied by the compositor)
        comp = CompositeSpec(distances.contiguous().view(-1), samples_per_ray, scale_a, scale_b,
                             getattr(self, "DENSITY_SHIFT", 0.0))
        outs = MLPFunction.apply(plan, pos_pe.shape[0], pos_pe, dir_pe, samples_per_ray, *plan.params(),
                                 composite=comp)
        return outs[-2], outs[-1]
