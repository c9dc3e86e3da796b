"""On-device training-batch feed.

The reference feeds training through ``ImagePoseDataset`` (barf/dataset.py:24-641): it
precomputes every ray of every training image on the host (``_get_directions_meshgrid``
:417-451, ``_meshgrid_to_world`` :453-481, ``_apply_noise`` :512-557), and a shuffling
``DataLoader`` (barf/data_module.py:202-209) calls ``__getitem__`` (:613-637) once per ray and
collates; ``ImagePoseDataModule.get_blurred_pixel_colors`` (data_module.py:276-367) then picks or
interpolates the blur level.  ``DeviceRayFeed`` keeps the images and camera matrices in HBM and
builds each batch in one ``nerf_ray_batch`` launch from a slice of the same shuffled index order
the reference's DataLoader produces (same generator rule, so the same rays in the same batches).

Batches are the reference's tuple ``(ray_origs_raw, ray_origs_noisy, ray_dirs_raw,
ray_dirs_noisy, ray_colors, img_idx, pixel_width)`` with ray_colors ``[B, n_sigmas, 3]``, or
``[B, 2, 3]`` (blurred, original) when a blur sigma is given (the fused
get_blurred_pixel_colors)."""
from __future__ import annotations

import warnings

import torch as th

from . import kernels as K
from .model_camera_extrinsics import CameraExtrinsics


def dataloader_epoch_order(n: int, generator: th.Generator) -> th.Tensor:
    """The index order of one epoch of ``DataLoader(dataset, shuffle=True, generator=g)``
    (RandomSampler without replacement): the loader iterator draws its base seed from g, the
    sampler draws the permutation, and on exhaustion one more (empty-sliced) permutation.
    Checked against torch's DataLoader in tests/test_host_logic.py."""
    th.empty((), dtype=th.int64).random_(generator=generator)
    order = th.randperm(n, generator=generator)
    th.randperm(n, generator=generator)
    return order


def pose_noise(n_images: int, rotation_noise_sigma: float, translation_noise_sigma: float,
               noise_seed: int | None) -> tuple[th.Tensor, th.Tensor]:
    """``_apply_noise``'s per-image rotation and translation (barf/dataset.py:535-547), on the CPU
    with the same generator draws."""
    g = th.Generator()
    if noise_seed is not None:
        g.manual_seed(noise_seed)
    rot = CameraExtrinsics.so3_to_SO3(th.randn((n_images, 3, 1), generator=g) * rotation_noise_sigma)
    trans = th.randn((n_images, 3), generator=g) * translation_noise_sigma
    return rot, trans


def blur_selection(sigmas: list[float], sigma: float) -> tuple[int, int, int, float, float]:
    """get_blurred_pixel_colors' case split (data_module.py:324-365) as (mode, lo, hi, coef_lo,
    coef_hi) for nerf_ray_batch: mode 1 no blur, 2 the most blurred level, 3 interpolation."""
    if sigma <= 0.25:
        return 1, 0, 0, 0.0, 0.0
    if sigma >= max(sigmas):
        if sigma > max(sigmas):
            warnings.warn(f"Tried to get blur with sigma {sigma} but used maximal possible: {max(sigmas)}.")
        return 2, 0, 0, 0.0, 0.0
    index_low = 0
    index_high = 0
    for index_high, s in enumerate(sigmas):
        if s < sigma:
            break
        index_low = index_high
    coef = (sigma - sigmas[index_high]) / (sigmas[index_low] - sigmas[index_high] + 1e-8)
    # tensor * python float: the scalar enters the fp32 product as fp32 (1 - coef formed in double)
    return 3, index_low, index_high, float(coef), float(1 - coef)


class DeviceRayFeed:
    """Shuffled training batches of an image/pose dataset, assembled on the GPU.

    images: [n_images, H, W, n_sigmas, 3] fp32 (blur levels in ``gaussian_blur_sigmas`` order,
    the layout ``__getitem__``'s ``img.view(-1, n_sigmas, 3)`` reads); camera_to_worlds:
    [n_images, 4, 4] after the dataset's space transform; focal_length as the dataset computes it."""

    def __init__(self, images: th.Tensor, camera_to_worlds: th.Tensor, focal_length: float, batch_size: int,
                 rotation_noise_sigma: float = 0.0, translation_noise_sigma: float = 0.0,
                 noise_seed: int | None = None, gaussian_blur_sigmas: list[float] | None = None,
                 dataloader_seed: int = 0, drop_last: bool = False, device: th.device | str = "cuda"):
        self.device = th.device(device)
        if images.dim() != 5 or images.shape[-1] != 3:
            raise ValueError("images must be [n_images, H, W, n_sigmas, 3]")
        self.n_images, self.H, self.W, self.n_sigmas = (int(x) for x in images.shape[:4])
        if camera_to_worlds.shape != (self.n_images, 4, 4):
            raise ValueError("camera_to_worlds must be [n_images, 4, 4]")
        self.gaussian_blur_sigmas = list(gaussian_blur_sigmas) if gaussian_blur_sigmas is not None else [0.0]
        if len(self.gaussian_blur_sigmas) != self.n_sigmas:
            raise ValueError("one blur sigma per image level")
        self.images = images.to(self.device, th.float32).contiguous()
        self.camera_to_worlds = camera_to_worlds.to(self.device, th.float32).contiguous()
        self.focal_length = float(focal_length)
        self.pixel_width = th.tensor(1 / self.focal_length)
        self.batch_size = int(batch_size)
        # the collated per-ray pixel widths, resident (a per-batch host->device copy of a pageable
        # tensor would drain the stream)
        self._pixel_widths = self.pixel_width.to(self.device).repeat(self.batch_size)
        rot, trans = pose_noise(self.n_images, rotation_noise_sigma, translation_noise_sigma, noise_seed)
        self.noise_rotation = rot.to(self.device, th.float32).contiguous()
        self.noise_translation = trans.to(self.device, th.float32).contiguous()
        self.drop_last = drop_last
        self.generator = th.Generator().manual_seed(dataloader_seed)
        self.status = th.zeros(1, dtype=th.int32, device=self.device)

    def __len__(self) -> int:
        n = self.n_images * self.H * self.W
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def batch(self, indices: th.Tensor, sigma: float | None = None):
        """The batch of the given dataset indices (device int64)."""
        blur = blur_selection(self.gaussian_blur_sigmas, sigma) if sigma is not None else None
        o_raw, o_n, d_raw, d_n, craw, cpair, img_idx = K.ray_batch(
            indices, self.H, self.W, self.focal_length, self.camera_to_worlds, self.noise_rotation,
            self.noise_translation, self.images, blur, sigma is None, self.status)
        B = indices.shape[0]
        pw = self._pixel_widths[:B] if B <= self.batch_size else self.pixel_width.to(self.device).repeat(B)
        return o_raw, o_n, d_raw, d_n, (cpair if sigma is not None else craw), img_idx, pw

    def epoch(self, sigma: float | None = None):
        """One epoch of batches in the reference DataLoader's order."""
        n = self.n_images * self.H * self.W
        order = dataloader_epoch_order(n, self.generator).to(self.device)
        for i in range(len(self)):
            yield self.batch(order[i * self.batch_size:(i + 1) * self.batch_size], sigma)

    def check(self) -> None:
        """Raise if any launched batch held an index outside the dataset (one host sync)."""
        if int(self.status.item()) & 1:
            raise IndexError("nerf_ray_batch: dataset index out of range")
