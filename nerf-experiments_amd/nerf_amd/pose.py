"""Camera-pose alignment of BARF's calibration model on the device.

Mirrors CameraCalibrationModel's helpers (barf/model_camera_calibration.py), same argument
order, shapes and conventions:
  * ``kabsch_algorithm(point_cloud_from, point_cloud_to, remove_outliers=True) -> (R, t, c)``
    (:69-156): R [3, 3], t [1, 3], c [] with ``R @ from * c + t`` estimating ``to``;
  * ``compute_pose_error(origs_raw, origs_pred)`` (:340-345): align the predicted camera origins to
    the raw ones (with outlier removal), mean Euclidean distance over all cameras;
  * ``validation_transform_rays(origs_val, dirs_val, post_transform_params)`` (:159-193).
The alignment and the error run in one HIP launch (nerf_kabsch, csrc/pose.hip); the reference's
trainer / datamodule plumbing that collects the origins stays with the caller.
"""
from __future__ import annotations

import torch as th

from . import kernels as K


def kabsch_algorithm(point_cloud_from: th.Tensor, point_cloud_to: th.Tensor, remove_outliers: bool = True):
    assert point_cloud_from.shape == point_cloud_to.shape, \
        "point_cloud_from and point_cloud_to must have the same shape"
    assert point_cloud_from.shape[1] == 3 and len(point_cloud_from.shape) == 2, \
        "point_cloud_from and point_cloud_to must be of shape (N, 3)"
    return K.kabsch(point_cloud_from, point_cloud_to, remove_outliers)


def compute_pose_error(origs_raw: th.Tensor, origs_pred: th.Tensor) -> th.Tensor:
    assert origs_raw.shape == origs_pred.shape and origs_raw.dim() == 2 and origs_raw.shape[1] == 3
    return K.kabsch(origs_pred, origs_raw, True, error=True)[3]


def validation_transform_rays(origs_val: th.Tensor, dirs_val: th.Tensor,
                              post_transform_params: tuple[th.Tensor, th.Tensor, th.Tensor]):
    R, t, c = post_transform_params
    origs_model = th.matmul(R, origs_val.unsqueeze(-1)).squeeze(-1) * c + t
    dirs_model = th.matmul(R, dirs_val.unsqueeze(-1)).squeeze(-1)
    return origs_model, dirs_model, post_transform_params


__all__ = ["kabsch_algorithm", "compute_pose_error", "validation_transform_rays"]
