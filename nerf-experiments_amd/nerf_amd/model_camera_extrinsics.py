"""Per-image camera pose refinement (BARF): the caller that pulls gradients through the hot path.

Mirrors barf/model_camera_extrinsics.py:7-85 (``CameraExtrinsics``: so3 rotation and translation
per training image, ``so3_to_SO3`` by the matrix exponential of the skew matrix, ``forward``
returning the refined origins / directions and the per-ray R, t).  ``forward`` is one HIP launch
(nerf_pose_rays_fwd, csrc/camera.hip) and its backward one more (nerf_pose_rays_bwd: per-image
fixed-order sums and the analytic so3 derivative); the gradient reaching it comes out of the fused
ray-mode encoding backward (nerf_encode_bwd_rays) and the direction encoding's backward.
``so3_to_SO3`` / ``get_rotations`` stay the reference's torch expressions (the noise generation
of the ray feed calls them on host tensors).
"""
from __future__ import annotations

import torch as th
import torch.nn as nn

from . import kernels as K
from .model_interpolation_architecture import NerfBaseModel

# barf/magic.py:1
MAGIC_NUMBER_THE_SECOND = 1


class CameraExtrinsics(NerfBaseModel):
    def __init__(self, n_train_images: int, learning_rate_start: float, learning_rate_stop: float,
                 learning_rate_decay_end: int = -1) -> None:
        super().__init__()
        self.size = n_train_images
        self.rotation = nn.Parameter(th.zeros((n_train_images, 3)))      # so3 Lie algebra
        self.translation = nn.Parameter(th.zeros((n_train_images, 3)))
        self._add_param_group(self.parameters(), learning_rate_start, learning_rate_stop, learning_rate_decay_end)

    @staticmethod
    def so3_to_SO3(so3: th.Tensor) -> th.Tensor:
        """[N, 3] so3 -> [N, 3, 3] rotations: matrix_exp of the skew matrix, built as the
        reference builds it (cross product of -I with the vector, model_camera_extrinsics.py:39-43)."""
        return th.matrix_exp(th.cross(-th.eye(3, device=so3.device).view(1, 3, 3), so3.view(-1, 3, 1), dim=1))

    def get_rotations(self, img_idx: th.Tensor) -> th.Tensor:
        return CameraExtrinsics.so3_to_SO3(self.rotation).index_select(0, img_idx.reshape(-1)).view(
            *img_idx.shape, 3, 3)

    def forward_origins(self, i: th.Tensor, o: th.Tensor) -> tuple[th.Tensor, th.Tensor]:
        # translation only (model_camera_extrinsics.py:61-74): rotation takes no part and gets no
        # gradient, as in the reference (the validation alignment calls this under no_grad)
        t = self.translation.index_select(0, i.reshape(-1)).view(*i.shape, 3) / MAGIC_NUMBER_THE_SECOND
        return o + t, t

    def forward(self, i: th.Tensor, o: th.Tensor, d: th.Tensor):
        """(new_o, new_d, R, t) as model_camera_extrinsics.py:77-85 returns them ([B, 3], [B, 3],
        [B, 3, 3], [B, 3]); ROCm tensors only (nerf_amd has no CPU path)."""
        return K.pose_rays(self.rotation, self.translation, i, o, d, MAGIC_NUMBER_THE_SECOND)


__all__ = ["CameraExtrinsics"]
