"""The older mip_NeRF experiment's module API (mip_NeRF/mip_model.py, model_interpolation.py) on the
gfx950 kernels.

mip_NeRF predates barf/'s generic encoders and renderer and has its own signatures:

* ``IntegratedFourierFeatures(levels, scale=2*pi, distribute_variance=False)`` with
  ``forward(pos, dir, t_start, t_end, pixel_width, distribute_variance=None)`` — note the argument
  order (t_start, t_end before pixel_width), no identity block and no pixel-width-sigma term
  (mip_NeRF/mip_model.py:11-75);
* ``MipNerfModel(n_hidden, hidden_dim, fourier=(use, levels_pos, levels_dir), n_segments,
  distribute_variance)`` with ``forward(pos, dir, t_start, t_end, pixel_width) -> (density, rgb)``
  (mip_model.py:79-105): the NerfModel of mip_NeRF/model_interpolation_architecture.py:26-160 with
  delayed direction, non-delayed density, Fourier direction encoding (scale 1) and the integrated
  position encoding;
* ``MipNerf(near, far, samples_per_ray, n_hidden, proposal=(use, coarse), fourier, n_segments, ...)``
  (mip_model.py:107-167 on mip_NeRF/model_interpolation.py:10-400): stratified coarse t (no offset),
  the round/argmax fine allocation (``_sample_t_fine``, :122-164), density factor 3*7, a coarse
  model that is the fine model unless ``seperate_coarse_fine``.

Everything runs on the same kernels as the barf API: the integrated encoding is
``nerf_encode_fwd`` kind 1 without identity and with pixel_width_sigma = 0 (the mip_NeRF formula has
no such term, and the kernel adds it only above 0.25), the renderer is ``NerfInterpolation`` with
``resample_mode=1``.  The mip_NeRF renderer repeats pixel widths as
``pixel_width.view(B, 1).repeat(S, 1)`` (:266), i.e. row n reads pw[n mod B], for both (B,) and (B, 1)
inputs; MipNerf passes them in that layout.  Parameter names, shapes and construction order equal
the reference's, so its state_dicts load and ``th.manual_seed`` gives its initial weights.
"""
from __future__ import annotations

from typing import Optional

import torch as th
import torch.nn as nn

from .model_interpolation import NerfInterpolation
from .model_interpolation_architecture import NerfModel
from .positional_encodings import FourierFeatures, IdentityPositionalEncoding
from .positional_encodings import IntegratedFourierFeatures as _BarfIntegratedFourierFeatures

MIP_NERF_MAGIC_NUMBER = 7      # mip_NeRF/model_interpolation.py:8 (density factor 3 * 7)


class IntegratedFourierFeatures(_BarfIntegratedFourierFeatures):
    """mip_NeRF/mip_model.py:11-75: IPE without the identity block, argument order
    (pos, dir, t_start, t_end, pixel_width)."""

    def __init__(self, levels: int, scale: float = 2 * th.pi, distribute_variance: Optional[bool] = False):
        super().__init__(levels, scale, include_identity=False, distribute_variance=distribute_variance)
        self.pixel_width_sigma = 0.0

    def forward(self, pos: th.Tensor, dir: th.Tensor, t_start: th.Tensor, t_end: th.Tensor, pixel_width,
                distribute_variance: Optional[bool] = None) -> th.Tensor:
        if pos.dim() != 2 or pos.shape[1] != 3:
            raise AssertionError("Only 3D supported")
        dv = distribute_variance or self.distribute_variance
        saved = self.distribute_variance
        self.distribute_variance = dv
        try:
            return self.encode_padded(pos, dir, pixel_width, t_start, t_end)[:, :self.output_dim]
        finally:
            self.distribute_variance = saved


class MipNerfModel(NerfModel):
    """mip_NeRF/mip_model.py:79-105."""

    def __init__(self, n_hidden: int, hidden_dim: int, fourier: tuple[bool, int, int], n_segments: int,
                 distribute_variance: Optional[bool] = False):
        fourier_flag, levels_pos, levels_dir = fourier
        if fourier_flag:
            pos_enc = IntegratedFourierFeatures(levels_pos, 2 * th.pi, distribute_variance)
            dir_enc = FourierFeatures(levels_dir, 1.0)
        else:
            pos_enc, dir_enc = IdentityPositionalEncoding(), IdentityPositionalEncoding()
        super().__init__(n_hidden, hidden_dim, True, False, n_segments, pos_enc, dir_enc)
        self.fourier = fourier_flag

    def forward(self, pos: th.Tensor, dir: th.Tensor, t_start: th.Tensor, t_end: th.Tensor, pixel_width):
        return NerfModel.forward(self, pos, dir, pixel_width, t_start, t_end)


class MipNerf(NerfInterpolation):
    """mip_NeRF/mip_model.py:107-167 (+ the renderer of mip_NeRF/model_interpolation.py)."""

    def __init__(self, near_sphere_normalized: float, far_sphere_normalized: float, samples_per_ray: int,
                 n_hidden: int, proposal: tuple[bool, int], fourier: tuple[bool, int, int], n_segments: int,
                 learning_rate: float = 1e-4, learning_rate_decay: float = 0.5, weight_decay: float = 0.0,
                 distribute_variance: Optional[bool] = False, seperate_coarse_fine: Optional[bool] = False):
        use_proposal = bool(proposal[0])
        nn.Module.__init__(self)
        self.use_proposal = use_proposal
        if use_proposal:
            coarse, fine = proposal[1], samples_per_ray - proposal[1]
        else:
            coarse, fine = samples_per_ray, 0
        model_fine = MipNerfModel(n_hidden, 256, fourier, n_segments, distribute_variance)
        model_coarse = MipNerfModel(n_hidden, 256, fourier, n_segments, distribute_variance) \
            if seperate_coarse_fine else model_fine
        if use_proposal:
            super().__init__(near_sphere_normalized, far_sphere_normalized, model_fine, coarse + fine,
                             "stratified_uniform", 0.0, "middle", model_coarse, coarse,
                             density_factor=(3.0, float(MIP_NERF_MAGIC_NUMBER)), resample_mode=1)
        else:
            super().__init__(near_sphere_normalized, far_sphere_normalized, model_coarse, coarse,
                             "stratified_uniform", 0.0, "middle",
                             density_factor=(3.0, float(MIP_NERF_MAGIC_NUMBER)), resample_mode=1)
        # the reference registers exactly model_fine and model_coarse (the same object when shared):
        # drop the renderer's own names so state_dict keys equal the reference's
        self._modules.pop("model_radiance", None)
        self._modules.pop("model_proposal", None)
        self.model_fine = model_fine
        self.model_coarse = model_coarse
        self.samples_per_ray_coarse = coarse
        self.samples_per_ray_fine = fine
        self.learning_rate = learning_rate
        self.learning_rate_decay = learning_rate_decay
        self.weight_decay = weight_decay

    @property
    def model_radiance(self):
        return self.model_fine if self.use_proposal else self.model_coarse

    @property
    def model_proposal(self):
        return self.model_coarse if self.use_proposal else None

    def _sample_t_coarse(self, batch_size: int):
        """mip_NeRF/model_interpolation.py:91-120: stratified bins, no per-ray offset."""
        return self._sample_t_stratified_uniform(batch_size, self.samples_per_ray_coarse, "stratified_uniform", 0.0)

    def _sample_t_fine(self, t_coarse: th.Tensor, weights: th.Tensor, distances_coarse: th.Tensor):
        """mip_NeRF/model_interpolation.py:122-164: round/argmax allocation of the fine samples."""
        return self._sample_t_pdf_weighted(t_coarse, weights, distances_coarse,
                                           self.samples_per_ray_coarse + self.samples_per_ray_fine)

    def forward(self, ray_origs: th.Tensor, ray_dirs: th.Tensor, pixel_width: th.Tensor):
        # mip_NeRF repeats pixel widths per ray with .view(B, 1).repeat(S, 1): pw[n mod B] (layout 1)
        pw = pixel_width.reshape(-1)
        rgb_fine, rgb_coarse = super().forward(ray_origs, ray_dirs, pw)
        if not self.use_proposal:
            return rgb_fine, th.zeros_like(rgb_fine)
        return rgb_fine, rgb_coarse

    def training_loss(self, ray_origs, ray_dirs, pixel_width, ray_colors):
        """_step_helpher (mip_NeRF/model_interpolation.py:343-375): proposal + radiance MSE."""
        fine, coarse = self.forward(ray_origs, ray_dirs, pixel_width)
        radiance = nn.functional.mse_loss(fine, ray_colors)
        proposal = nn.functional.mse_loss(coarse, ray_colors)
        return proposal + radiance, {"proposal_loss": proposal.detach(), "radiance_loss": radiance.detach(),
                                     "psnr": -10 * th.log10(radiance.detach())}

    def configure_optimizers(self):
        """mip_NeRF/model_interpolation.py:384-400: Adam over all parameters + ExponentialLR."""
        from .optim import FusedAdam
        params = list(self.parameters())
        on_gpu = all(p.is_cuda for p in params)
        optimizer = (FusedAdam if on_gpu else th.optim.Adam)(params, lr=self.learning_rate,
                                                             weight_decay=self.weight_decay)
        scheduler = th.optim.lr_scheduler.ExponentialLR(optimizer, gamma=self.learning_rate_decay)
        return {"optimizer": optimizer, "lr_scheduler": scheduler}


__all__ = ["IntegratedFourierFeatures", "MipNerfModel", "MipNerf", "MIP_NERF_MAGIC_NUMBER"]
