"""Hash-grid NeRF (config C5) on gfx950 kernels: INGPTable, INGPEncoding, NerfModelINGP.

The reference's 3d-ingp/model.py:14-193 as SURVEY.md §8(a) describes it (rows a7, a9): the
builder's read of that file was refused in round 1, so constructor arguments,
parameter names and initialisation here are this package's own and the numerics are **parity
unpinned** (checked against oracle/hashgrid_oracle.py, a restatement of the same description).

* ``INGPEncoding``: ``levels`` resolutions r_l = floor(16 b^l), b = exp((ln 1600 - ln 16) / 15),
  one ``[levels, table_size, feature_dim]`` table (bijective rows while (r+1)^3 <= table_size, the
  product-xor hash otherwise), positions normalised as x / 8 + 0.5; output [N, levels * feature_dim]
  (level-major).  Forward and the (deterministic, fixed-point) table gradient are nerf_hashgrid_fwd /
  nerf_hashgrid_bwd; positions receive no gradient.
* ``NerfModelINGP``: the NerfModel lowering with one segment of 9 Linear layers
  (enc -> 256, 7 x 256 -> 256, 256 -> 257), the colour head [z | dir PE] -> 128 -> 3, direction
  encoding FourierFeatures(4, 1.0) (3d-ingp/model.py:137-148, scale 1), density softplus(z - 1).
  The whole field MLP runs on the fused kernel (the hash features are its HBM-fed input).
"""
from __future__ import annotations

import math

import torch as th
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from .model_interpolation_architecture import NerfModel, RawHeads
from .positional_encodings import FourierFeatures


def ingp_resolutions(levels: int = 16, resolution_min: int = 16, resolution_max: int = 1600) -> list[int]:
    if levels == 1:
        return [resolution_min]
    b = math.exp((math.log(resolution_max) - math.log(resolution_min)) / (levels - 1))
    return [int(math.floor(resolution_min * b ** l)) for l in range(levels)]


class _HashGridFn(th.autograd.Function):
    @staticmethod
    def forward(ctx, enc, x, ray_o, ray_d, t_start, t_end, samples_per_ray, query, n, table):
        params = enc._params(query)
        out = th.empty(n, K.pad32(enc.output_dim), device=table.device, dtype=th.float32)
        if out.shape[1] > enc.output_dim:
            out[:, enc.output_dim:].zero_()
        K.hashgrid_fwd(params, table, out, x=x, ray_o=ray_o, ray_d=ray_d, t_start=t_start, t_end=t_end,
                       n_samples=n, samples_per_ray=samples_per_ray)
        ctx.enc = enc
        ctx.meta = (samples_per_ray, query, n)
        ctx.save_for_backward(*(t if t is not None else th.empty(0) for t in (x, ray_o, ray_d, t_start, t_end)))
        return out

    @staticmethod
    def backward(ctx, g):
        enc = ctx.enc
        spr, query, n = ctx.meta
        x, o, d, t0, t1 = (t if t.numel() else None for t in ctx.saved_tensors)
        grad_table = None
        if ctx.needs_input_grad[9] and g is not None:
            grad_table = th.empty_like(enc.table)
            K.hashgrid_bwd(enc._params(query), g.contiguous(), grad_table, enc._workspace(g.device), x=x,
                           ray_o=o, ray_d=d, t_start=t0, t_end=t1, n_samples=n, samples_per_ray=spr)
        return None, None, None, None, None, None, None, None, None, grad_table


class INGPEncoding(nn.Module):
    """Multiresolution hash encoding with the PositionalEncoding interface of the renderer
    (``forward(x, dir, pixel_width, t_start, t_end)``, ``output_dim``)."""

    def __init__(self, levels: int = 16, resolution_min: int = 16, resolution_max: int = 1600,
                 table_size: int = 2 ** 16, feature_dim: int = 2, init_scale: float = 1e-4):
        super().__init__()
        self.levels = levels
        self.table_size = table_size
        self.feature_dim = feature_dim
        self.resolutions = ingp_resolutions(levels, resolution_min, resolution_max)
        self.output_dim = levels * feature_dim
        self.space_dimensions = 3
        self.table = nn.Parameter(th.empty(levels, table_size, feature_dim).uniform_(-init_scale, init_scale))
        self._ws = {}

    def _params(self, query: int = 1):
        return K.make_hashgrid_params(self.levels, self.table_size, self.feature_dim, self.resolutions, query)

    def _workspace(self, device) -> th.Tensor:
        # the fixed-point accumulators: zero on the first call, left zero by every call
        ws = self._ws.get(device)
        if ws is None:
            nbytes = K.hashgrid_workspace_bytes(self._params())
            ws = self._ws[device] = th.zeros((nbytes + 7) // 8, dtype=th.int64, device=device)
        return ws

    def bijective(self, level: int) -> bool:
        r = self.resolutions[level]
        return (r + 1) ** 3 <= self.table_size

    def encode_padded(self, x: th.Tensor, dir=None, pixel_width=None, t_start=None, t_end=None) -> th.Tensor:
        """[N, pad32(output_dim)] features of explicit positions x [N, 3]."""
        x = x.contiguous()
        return _HashGridFn.apply(self, x, None, None, None, None, 1, 1, x.shape[0], self.table)

    def encode_rays(self, ray_origs, ray_dirs, t_start, t_end, pixel_width, samples_per_ray: int, query: int,
                    pw_mode: int = 0) -> th.Tensor:
        """Features of the samples o + t_q d generated in-kernel (no gradient to the rays)."""
        n = t_start.numel()
        return _HashGridFn.apply(self, None, ray_origs.detach().contiguous(), ray_dirs.detach().contiguous(),
                                 t_start.contiguous(), t_end.contiguous(), samples_per_ray, query, n, self.table)

    def forward(self, x: th.Tensor, dir=None, pixel_width=None, t_start=None, t_end=None) -> th.Tensor:
        return self.encode_padded(x)[:, :self.output_dim]


class INGPTable(nn.Module):
    """One level of an INGPEncoding (its resolution, table rows and features): a view onto the
    encoding's shared table, so the kernels read every level from one contiguous tensor."""

    def __init__(self, encoding: INGPEncoding, level: int):
        super().__init__()
        self._encoding = [encoding]          # not a submodule: the parameter belongs to the encoding
        self.level = level
        self.resolution = encoding.resolutions[level]
        self.table_size = encoding.table_size
        self.feature_dim = encoding.feature_dim

    @property
    def table(self) -> th.Tensor:
        return self._encoding[0].table[self.level]

    def forward(self, x: th.Tensor) -> th.Tensor:
        enc = self._encoding[0]
        f = enc(x)
        return f[:, self.level * self.feature_dim:(self.level + 1) * self.feature_dim]


class NerfModelINGP(NerfModel):
    """Hash-grid field (config C5): NerfModel lowering with one 9-layer segment and density
    softplus(z - 1)."""

    DENSITY_SHIFT = 1.0

    def __init__(self, position_encoder: INGPEncoding | None = None, direction_encoder=None, n_hidden: int = 8,
                 hidden_dim: int = 256, learning_rate_start: float = 5e-4, learning_rate_stop: float = 5e-5,
                 learning_rate_decay_end: float = 0):
        super().__init__(n_hidden, hidden_dim, True, False, 1,
                         position_encoder if position_encoder is not None else INGPEncoding(),
                         direction_encoder if direction_encoder is not None else FourierFeatures(4, 1.0),
                         learning_rate_start, learning_rate_stop, learning_rate_decay_end)

    def _heads(self, z_last, head, dens) -> RawHeads:
        return RawHeads(head, dens.view(-1, 1), 0, self.DENSITY_SHIFT)

    def forward(self, pos: th.Tensor, dir: th.Tensor, pixel_width=None, t_start=None, t_end=None):
        pos_pe = self.position_encoder.encode_padded(pos)
        dir_pe = self.direction_encoder.encode_padded(dir)
        z_last, head, dens = self._run_mlp(pos_pe, dir_pe, 1)
        density = F.softplus(dens - self.DENSITY_SHIFT, beta=1, threshold=8)
        rgb = th.sigmoid(head[:, :3])
        return density, rgb
