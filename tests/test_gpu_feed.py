"""On-device training-batch feed (nerf_ray_batch / nerf_amd.ray_feed.DeviceRayFeed) against the
oracle's restatement of ImagePoseDataset + DataLoader + get_blurred_pixel_colors
(oracle/nerf_oracle.py: ray_batch, barf/dataset.py:417-637, data_module.py:276-367).

Gathers (colours, origins, image indices) and the blur selection are bit-exact; ray directions
come from the kernel's own pixel-centre arithmetic instead of the reference's precomputed batched
matmul, and agree to 2e-7 absolute (unit vectors: a few ulp)."""
import math
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-experiments_amd"))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dataset(n, H, W, S, seed=0):
    g = torch.Generator().manual_seed(seed)
    images = torch.rand(n, H, W, S, 3, generator=g)
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    R = CameraExtrinsics.so3_to_SO3(torch.randn(n, 3, generator=g))
    c2w = torch.zeros(n, 4, 4)
    c2w[:, :3, :3] = R
    c2w[:, :3, 3] = torch.randn(n, 3, generator=g) * 4
    c2w[:, 3, 3] = 1
    return images, c2w


@pytest.mark.parametrize("n,H,W,S", [(3, 7, 5, 3), (2, 64, 48, 1), (4, 1, 9, 2)])
@pytest.mark.parametrize("sigma", [None, 0.1, 2.0, 5.0, 9.0])
def test_ray_batch_matches_oracle(n, H, W, S, sigma):
    from oracle import nerf_oracle as O
    from nerf_amd.ray_feed import DeviceRayFeed
    images, c2w = _dataset(n, H, W, S)
    sigmas = [8.0, 4.0, 0.0][:S] if S > 1 else [0.0]
    if S == 2:
        sigmas = [4.0, 0.0]
    focal = W / 2 / math.tan(0.6911112 / 2)
    feed = DeviceRayFeed(images, c2w, focal, 64, rotation_noise_sigma=0.1, translation_noise_sigma=0.2,
                         noise_seed=3, gaussian_blur_sigmas=sigmas, dataloader_seed=1, device=DEV)
    total = n * H * W
    idx = torch.randperm(total, generator=torch.Generator().manual_seed(2))[:97]
    if sigma is not None and sigma > 0.25 and sigma > max(sigmas):   # the reference warns then
        with pytest.warns(UserWarning):
            got = feed.batch(idx.to(DEV), sigma)
    else:
        got = feed.batch(idx.to(DEV), sigma)
    want = O.ray_batch(images, c2w, focal, idx, feed.noise_rotation.cpu(), feed.noise_translation.cpu(), sigmas,
                       sigma)
    o, on, d, dn, col, img, pw = [t.cpu() if isinstance(t, torch.Tensor) else t for t in got]
    assert torch.equal(o, want[0]) and torch.equal(on, want[1]) and torch.equal(img, want[5])
    assert (d - want[2]).abs().max() <= 2e-7 and (dn - want[3]).abs().max() <= 3e-7
    assert torch.equal(col, want[4])
    assert pw.shape == (len(idx),) and float(pw[0]) == float(torch.tensor(1 / focal))
    feed.check()


def test_feed_epoch_batches_follow_dataloader_order():
    """The epoch iterator yields the rays the reference's DataLoader would, batch by batch."""
    from oracle import nerf_oracle as O
    from nerf_amd.ray_feed import DeviceRayFeed, dataloader_epoch_order
    images, c2w = _dataset(2, 6, 4, 1, seed=4)
    feed = DeviceRayFeed(images, c2w, 5.0, 10, noise_seed=0, dataloader_seed=9, device=DEV)
    batches = list(feed.epoch())
    assert len(batches) == len(feed) == 5
    order = dataloader_epoch_order(48, torch.Generator().manual_seed(9))
    for i, b in enumerate(batches):
        want = O.ray_batch(images, c2w, 5.0, order[i * 10:(i + 1) * 10], feed.noise_rotation.cpu(),
                           feed.noise_translation.cpu())
        assert torch.equal(b[5].cpu(), want[5]) and torch.equal(b[4].cpu(), want[4])


def test_feed_reports_out_of_range_index():
    from nerf_amd.ray_feed import DeviceRayFeed
    images, c2w = _dataset(1, 4, 4, 1)
    feed = DeviceRayFeed(images, c2w, 3.0, 4, device=DEV)
    feed.batch(torch.tensor([0, 5, 16, 3], device=DEV))
    with pytest.raises(IndexError):
        feed.check()
