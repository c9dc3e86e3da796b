"""Per-image camera pose refinement (BARF): the caller that pulls gradients through the hot path.

Mirrors barf/model_camera_extrinsics.py:7-85 (``CameraExtrinsics``: so3 rotation and translation
per training image, ``so3_to_SO3`` by the matrix exponential of the skew matrix, ``forward``
returning the refined origins / directions).  Plain torch ops on tiny [n_images, 3] tensors —
the gradient reaching ``rotation`` / ``translation`` comes out of the fused ray-mode encoding
backward (nerf_encode_bwd_rays) and the direction encoding's backward.
"""
from __future__ import annotations

import torch as th
import torch.nn as nn

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
        # index_select == [img_idx] for a 1-D index; its backward is an index_add (the advanced-
        # indexing backward sorts the indices: three extra kernels per step)
        return CameraExtrinsics.so3_to_SO3(self.rotation).index_select(0, img_idx.reshape(-1)).view(
            *img_idx.shape, 3, 3)

    def forward_origins(self, i: th.Tensor, o: th.Tensor) -> tuple[th.Tensor, th.Tensor]:
        t = self.translation.index_select(0, i.reshape(-1)).view(*i.shape, 3) / MAGIC_NUMBER_THE_SECOND
        return o + t, t

    def forward(self, i: th.Tensor, o: th.Tensor, d: th.Tensor):
        new_o, t = self.forward_origins(i, o)
        R = self.get_rotations(i)
        # R @ d per ray as a 3-term elementwise sum (a batched 3x3 GEMM on hipBLASLt is ~4 kernels)
        new_d = (R * d.unsqueeze(-2)).sum(-1)
        return new_o, new_d, R, t


__all__ = ["CameraExtrinsics"]
