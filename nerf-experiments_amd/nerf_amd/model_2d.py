"""2d-reconstruction (config C1): a single-image coordinate MLP on gfx950 kernels.

Mirrors 2d-reconstruction/model.py with the same class names, constructor arguments, submodule
layout (so ``th.manual_seed`` gives the reference's initial parameters and state_dicts
interchange: ``model.1`` / ``model.3`` / ``model.5`` / ``model.7``) and training API:
  * ``FourierFeatures2d``  model.py:6-22 — [cos(x_d * pi 2^k) (d-major) | sin(...)] of 2-D points;
    the argument is x_d * fp32(pi * 2^k), as the reference's fp32 ``2**arange * pi`` scale.
  * ``Nerf2d``             model.py:25-102 — FourierFeatures(10) -> Linear(40, 256) -> Tanh ->
    Linear(256, 256) -> Tanh -> Linear(256, 256) -> Tanh -> Linear(256, 3) -> Sigmoid; MSE
    training step; Adam + ReduceLROnPlateau(mode="min", monitor train_loss).

On the device: the encoding is ``nerf_encode_fwd`` on the points padded to 3-D (x, y, 0), and the
whole MLP is one ``MLPFunction`` autograd node with tanh in the GEMM epilogues
(``NERF_EPI_TANH`` / ``NERF_EPI_TANH_BWD``); the first layer reads the encoding's cos(x, y) and
sin(x, y) columns straight from that buffer through its packed-weight column map (the z columns
meet zero weights).  Only the final sigmoid is a torch op, as the heads of NerfModel.
"""
from __future__ import annotations

import torch as th
import torch.nn as nn

from . import kernels as K
from .mlp import LayerPlan, MLPFunction, MLPPlan, Source


class FourierFeatures2d(nn.Module):
    """2d-reconstruction/model.py:6-22 FourierFeatures (scale pi * 2^k, no parameters)."""

    def __init__(self, levels: int):
        super().__init__()
        self.levels = levels
        self.output_dim = 2 * 2 * levels

    def encode3(self, x: th.Tensor) -> th.Tensor:
        """[M, pad32(6L)] encoding of (x, y, 0): cos blocks at 0 (x, y: 2L columns), 2L (z), sin
        blocks at 3L (x, y) and 5L (z)."""
        if x.dim() != 2 or x.shape[1] != 2:
            raise ValueError(f"expected [batch, 2] points, got {tuple(x.shape)}")
        K._require_cuda_f32("x", x)
        x3 = th.nn.functional.pad(x, (0, 1)).contiguous()
        params = K.make_pe_params(0, self.levels, False, float(th.pi))
        n = x.shape[0]
        return K.encode_fwd(params, 6 * self.levels, x=x3, n_samples=n, samples_per_ray=1, n_rays=n,
                            out_ld=K.pad32(6 * self.levels), device=x.device)

    def forward(self, x: th.Tensor) -> th.Tensor:
        L = self.levels
        e = self.encode3(x)
        return th.cat((e[:, :2 * L], e[:, 3 * L:5 * L]), dim=1)


class Nerf2d(nn.Module):
    def __init__(self, width: int, height: int, fourier_levels: int, learning_rate: float = 1e-3,
                 learning_rate_decay: float = 0.5, learning_rate_decay_patience: int = 20,
                 weight_decay: float = 0.0):
        super().__init__()
        self.width = width
        self.height = height
        self.fourier_levels = fourier_levels
        self.learning_rate = learning_rate
        self.learning_rate_decay = learning_rate_decay
        self.learning_rate_decay_patience = learning_rate_decay_patience
        self.weight_decay = weight_decay
        self.model = nn.Sequential(
            FourierFeatures2d(levels=self.fourier_levels),
            nn.Linear(2 * 2 * self.fourier_levels, 256),
            nn.Tanh(),
            nn.Linear(256, 256),
            nn.Tanh(),
            nn.Linear(256, 256),
            nn.Tanh(),
            nn.Linear(256, 3),
            nn.Sigmoid(),
        )
        self._plan: MLPPlan | None = None

    def _get_plan(self) -> MLPPlan:
        if self._plan is None:
            L = self.fourier_levels
            width = 6 * L
            # buffer column -> Linear input: cos(x, y) -> 0 .. 2L-1, sin(x, y) -> 2L .. 4L-1, z unused
            cols = [c if c < 2 * L else (-1 if c < 3 * L else (c - L if c < 5 * L else -1)) for c in range(width)]
            enc = Source("pos", width, K.pad32(width), cols=cols)
            m = self.model
            layers = [LayerPlan(m[1], [enc], False, tanh=True)]
            for i in (3, 5):
                layers.append(LayerPlan(m[i], [Source("act", 256, 256, len(layers) - 1)], False, tanh=True))
            layers.append(LayerPlan(m[7], [Source("act", 256, 256, len(layers) - 1)], False))
            self._plan = MLPPlan(layers, [len(layers) - 1])
        return self._plan

    def forward(self, x: th.Tensor) -> th.Tensor:
        plan = self._get_plan()
        enc = self.model[0].encode3(x)
        (head,) = MLPFunction.apply(plan, x.shape[0], enc, None, 1, *plan.params())
        return th.sigmoid(head[:, :3])

    def training_step(self, batch: tuple[th.Tensor, th.Tensor], batch_idx: int = 0) -> th.Tensor:
        x, y = batch
        return nn.functional.mse_loss(self(x), y)

    def validation_step(self, batch, batch_idx: int = 0) -> th.Tensor:
        x, y = batch
        with th.no_grad():
            return nn.functional.mse_loss(self(x), y)

    def configure_optimizers(self):
        # model.py:88-102; on the GPU Adam's step is nerf_amd's fused launch
        from .optim import FusedAdam
        on_gpu = next(self.parameters()).is_cuda
        optimizer = (FusedAdam if on_gpu else th.optim.Adam)(self.parameters(), lr=self.learning_rate,
                                                             weight_decay=self.weight_decay)
        scheduler = th.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=self.learning_rate_decay,
                                                            patience=self.learning_rate_decay_patience)
        return {"optimizer": optimizer, "lr_scheduler": scheduler, "monitor": "train_loss"}


__all__ = ["FourierFeatures2d", "Nerf2d"]
