"""GARF field MLPs (Gaussian-activation radiance / proposal networks) on gfx950 kernels.

Mirrors, with the same class names, constructor arguments, submodule names and construction
order (so ``th.manual_seed`` gives the reference's initial parameters and state_dicts
interchange):
  * ``GaussAct``          garf/gaussian.py:34-63 (GaussActivation autograd :8-31); copy barf/gaussian.py
  * ``RadianceNetwork``   barf/model_garf_radiance.py:10-113 (garf/model_radiance.py:9-96 is the
                          same network built under ``th.compile``, whose state_dict keys carry an
                          extra ``_orig_mod.`` — see ``strip_compile_prefix``)
  * ``ProposalNetwork``   barf/model_garf_proposal.py:10-77 (garf/model_proposal.py:9-56)
The learning-rate arguments of the barf copies are optional, so the garf two-argument
constructor works too; ``param_groups`` exist when they are given.

Each network runs as ONE ``MLPFunction`` autograd node: every Linear on the MFMA linear
kernels (fp32 or 3 x bf16 split, per ``torch.get_float32_matmul_precision``), each Gaussian
activation in ``nerf_gauss_act_fwd/bwd`` (per-channel inverse-std gradient reduced in a fixed
order), RadianceNetwork's ``z1[:, :128] + z2[:, :128]`` folded into the accumulate epilogue of
the last density layer, and the concatenations ``[z1 | pos]`` / ``[z1 + z2 | dir]`` read as
multi-segment GEMM operands (never materialised).  Only the final softplus / sigmoid heads are
applied with torch ops, as in NerfModel.forward.
"""
from __future__ import annotations

from typing import Iterator

import torch as th
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from .mlp import LayerPlan, MLPFunction, MLPPlan, Source
from .model_interpolation_architecture import NerfBaseModel


class _GaussActFn(th.autograd.Function):
    @staticmethod
    def forward(ctx, x, inv_std):
        K._require_cuda_f32("x", x)
        if x.dim() != 2 or x.shape[1] != inv_std.shape[0]:
            raise ValueError(f"GaussAct expects [batch, {inv_std.shape[0]}] input, got {tuple(x.shape)}")
        if x.stride(1) != 1:
            x = x.contiguous()
        y = th.empty(x.shape, device=x.device, dtype=th.float32)
        K.gauss_act_fwd(x, x.shape[1], inv_std, y)
        ctx.save_for_backward(x, inv_std)
        return y

    @staticmethod
    def backward(ctx, g):
        x, inv_std = ctx.saved_tensors
        g = g.contiguous()
        dx = th.empty_like(x)
        ds = th.empty_like(inv_std)
        K.gauss_act_bwd(g, x, x.shape[1], inv_std, dx, ds)
        return dx, ds


class GaussAct(nn.Module):
    def __init__(self, features_in: int, inv_standard_deviation_init_min: float = 0.,
                 inv_standard_deviation_init_max: float = 1.):
        super().__init__()
        # negative values allowed: only inv_std ** 2 is used (gaussian.py:56-59)
        self.inv_standard_deviation = nn.Parameter(
            th.rand(features_in) * (inv_standard_deviation_init_max - inv_standard_deviation_init_min)
            + inv_standard_deviation_init_min)

    def forward(self, x: th.Tensor) -> th.Tensor:
        return _GaussActFn.apply(x, self.inv_standard_deviation)


class _Pad4Fn(th.autograd.Function):
    """[M,3] -> [M,4] (zero 4th column) with nerf_encode_fwd's identity encoding: the
    MFMA linear kernels read operand rows in 16-byte quads."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        params = K.make_pe_params(0, 0, True, 1.0)
        return K.encode_fwd(params, 3, x=x, n_samples=x.shape[0], n_rays=x.shape[0], out_ld=4, device=x.device)

    @staticmethod
    def backward(ctx, g):
        return g[:, :3]


def _pad4(x: th.Tensor) -> th.Tensor:
    if x.dim() != 2 or x.shape[1] != 3:
        raise ValueError(f"expected [batch, 3] input, got {tuple(x.shape)}")
    K._require_cuda_f32("input", x)
    return _Pad4Fn.apply(x)


def strip_compile_prefix(state_dict: dict) -> dict:
    """State dict of garf's ``th.compile``-wrapped networks -> this module's key names."""
    return {k.replace("._orig_mod", ""): v for k, v in state_dict.items()}


class _GarfBase(NerfBaseModel):
    def __init__(self, gaussian_init_min: float, gaussian_init_max: float):
        super().__init__()
        self.gaussian_init_min = gaussian_init_min
        self.gaussian_init_max = gaussian_init_max
        self._parameters_linear: list[nn.Parameter] = []
        self._parameters_gaussian: list[nn.Parameter] = []
        self._plan: MLPPlan | None = None

    def _create_linear(self, features_in: int, features_out: int) -> nn.Linear:
        linear = nn.Linear(features_in, features_out)
        self._parameters_linear.append(linear.weight)
        self._parameters_linear.append(linear.bias)
        return linear

    def _create_gaussian(self, features_in) -> GaussAct:
        act = GaussAct(features_in, self.gaussian_init_min, self.gaussian_init_max)
        self._parameters_gaussian.append(act.inv_standard_deviation)
        return act

    def parameters_linear(self) -> Iterator[nn.Parameter]:
        return iter(self._parameters_linear)

    def parameters_gaussian(self) -> Iterator[nn.Parameter]:
        return iter(self._parameters_gaussian)

    def _maybe_param_groups(self, learning_rate_start, learning_rate_stop, learning_rate_decay_end,
                            gaussian_learning_rate_factor, weight_decay):
        if learning_rate_start is None:
            return
        self._add_param_group(self.parameters_linear(), learning_rate_start, learning_rate_stop,
                              learning_rate_decay_end, weight_decay)
        self._add_param_group(self.parameters_gaussian(), learning_rate_start * gaussian_learning_rate_factor,
                              learning_rate_stop * gaussian_learning_rate_factor, learning_rate_decay_end,
                              weight_decay)


def _gauss_chain(seq: nn.Sequential, first_sources: list[Source], layers: list[LayerPlan]) -> int:
    """Lower Linear/GaussAct pairs of ``seq`` (a trailing Linear without activation allowed);
    returns the index of the last layer."""
    mods = list(seq)
    i = 0
    srcs = first_sources
    while i < len(mods):
        lin = mods[i]
        if not isinstance(lin, nn.Linear):
            break
        act = mods[i + 1] if i + 1 < len(mods) and isinstance(mods[i + 1], GaussAct) else None
        if srcs is None:
            prev = layers[-1].module.out_features
            srcs = [Source("act", prev, K.pad32(prev), len(layers) - 1)]
        layers.append(LayerPlan(lin, srcs, False, gauss=act.inv_standard_deviation if act is not None else None))
        srcs = None
        i += 2 if act is not None else 1
    return len(layers) - 1


class RadianceNetwork(_GarfBase):
    def __init__(self, gaussian_init_min: float, gaussian_init_max: float, learning_rate_start: float | None = None,
                 learning_rate_stop: float | None = None, learning_rate_decay_end: float = 0,
                 gaussian_learning_rate_factor: float = 1.0, weight_decay: float = 0.0):
        super().__init__(gaussian_init_min, gaussian_init_max)
        self.model_density_1 = nn.Sequential(
            self._create_linear(3, 1024), self._create_gaussian(1024),
            self._create_linear(1024, 256), self._create_gaussian(256),
            self._create_linear(256, 128), self._create_gaussian(128),
            self._create_linear(128, 128), self._create_gaussian(128),
        )
        self.model_density_2 = nn.Sequential(
            self._create_linear(128 + 3, 512), self._create_gaussian(512),
            self._create_linear(512, 256), self._create_gaussian(256),
            self._create_linear(256, 128), self._create_gaussian(128),
            self._create_linear(128, 128 + 1),
        )
        self.softplus = nn.Softplus(threshold=8)
        self.model_color = nn.Sequential(
            self._create_linear(128 + 3, 256), self._create_gaussian(256),
            self._create_linear(256, 3), nn.Sigmoid(),
        )
        self._maybe_param_groups(learning_rate_start, learning_rate_stop, learning_rate_decay_end,
                                 gaussian_learning_rate_factor, weight_decay)

    def _get_plan(self) -> MLPPlan:
        if self._plan is None:
            layers: list[LayerPlan] = []
            pos = Source("pos", 3, K.pad32(3))
            z1 = _gauss_chain(self.model_density_1, [pos], layers)
            z2 = _gauss_chain(self.model_density_2, [Source("act", 128, 128, z1), pos], layers)
            # z2 output holds [z1[:, :128] + z2[:, :128] | z2[:, 128]] (model_radiance.py:89,92)
            layers[z2].residual, layers[z2].residual_cols = z1, 128
            head = _gauss_chain(self.model_color, [Source("act", 128, 128, z2), Source("dir", 3, K.pad32(3))],
                                layers)
            # sigma = softplus(z2[:, 128] - 1) reads one column: exposed as its own [M] output
            self._plan = MLPPlan(layers, [z2, head], [(z2, 128)])
        return self._plan

    def forward(self, pos: th.Tensor, dir: th.Tensor) -> tuple[th.Tensor, th.Tensor]:
        plan = self._get_plan()
        _, head, sigma_raw = MLPFunction.apply(plan, pos.shape[0], _pad4(pos), _pad4(dir), 1, *plan.params())
        density = F.softplus(sigma_raw - 1, beta=1, threshold=8)
        rgb = th.sigmoid(head[:, :3])
        return rgb, density


class ProposalNetwork(_GarfBase):
    def __init__(self, gaussian_init_min: float, gaussian_init_max: float, learning_rate_start: float | None = None,
                 learning_rate_stop: float | None = None, learning_rate_decay_end: float = 0,
                 gaussian_learning_rate_factor: float = 1.0, weight_decay: float = 0.0):
        super().__init__(gaussian_init_min, gaussian_init_max)
        self.model = nn.Sequential(
            self._create_linear(3, 512), self._create_gaussian(512),
            self._create_linear(512, 256), self._create_gaussian(256),
            self._create_linear(256, 128), self._create_gaussian(128),
            self._create_linear(128, 1), nn.Softplus(threshold=8),
        )
        self._maybe_param_groups(learning_rate_start, learning_rate_stop, learning_rate_decay_end,
                                 gaussian_learning_rate_factor, weight_decay)

    def _get_plan(self) -> MLPPlan:
        if self._plan is None:
            layers: list[LayerPlan] = []
            out = _gauss_chain(self.model, [Source("pos", 3, K.pad32(3))], layers)
            self._plan = MLPPlan(layers, [out])
        return self._plan

    def forward(self, pos: th.Tensor) -> th.Tensor:
        plan = self._get_plan()
        (y,) = MLPFunction.apply(plan, pos.shape[0], _pad4(pos), None, 1, *plan.params())
        return F.softplus(y[:, :1], beta=1, threshold=8)


__all__ = ["GaussAct", "RadianceNetwork", "ProposalNetwork", "strip_compile_prefix"]
