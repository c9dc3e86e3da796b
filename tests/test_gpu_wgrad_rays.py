"""Weight gradient of a layer whose last input is per ray (NerfModel's colour layer: the direction
encoding read once per ray, row divisor S) through nerf_linear_wgrad_x3_rays: the streamed kernel over
the per-sample inputs also sums dY over each ray's samples, and the per-ray input's columns come from
those sums over the B rays (mlp._wgrad_rays).  Against fp64 over every sample's row with the
split-precision bound of test_gpu_parity.py (2^-15 of |dY|^T |X|), rays of S | 128 or 256 samples (3d-ingp's fine pass), one or two row blocks (the two
passes of a shared field), and the layer-level switch (NERF_WGRAD_RAYS) on a NerfModel step."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("B0,S0,B1,S1,N,kmain,kray", [(64, 64, 32, 128, 128, 256, 27), (100, 64, 0, 0, 128, 256, 27),
                                                       (48, 16, 16, 32, 200, 96, 12), (2048, 128, 4096, 64, 128, 256, 27),
                                                       (300, 256, 0, 0, 128, 256, 24), (512, 64, 37, 256, 128, 256, 24),
                                                       (20, 256, 64, 128, 200, 256, 24)])
def test_wgrad_rays_matches_fp64(B0, S0, B1, S1, N, kmain, kray):
    from nerf_amd import kernels as K, mlp
    torch.manual_seed(B0 + B1 + N)
    N4 = (N + 3) // 4 * 4
    blocks, ref_x, ref_y = [], [], []
    for B, S in ((B0, S0), (B1, S1)):
        if B == 0:
            continue
        M = B * S
        dY = torch.randn(M, N4)
        dY[:, N:] = 0
        xm = torch.randn(M, kmain)
        xr = torch.randn(B, (kray + 3) // 4 * 4)
        blocks.append((dY.to(DEV), [(xm.to(DEV), kmain, 1), (xr.to(DEV), (kray + 3) // 4 * 4, S)], M))
        ref_x.append(torch.cat([xm, xr[:, :kray].repeat_interleave(S, dim=0)], dim=1).double())
        ref_y.append(dY[:, :N].double())
    split = mlp._ray_split(blocks, N4)
    assert split is not None
    Kp_main, Kp_ray = K.pad32(kmain), K.pad32(kray)
    cm = list(range(kmain)) + [-1] * (Kp_main - kmain) + [kmain + j for j in range(kray)] + [-1] * (Kp_ray - kray)
    lp = types.SimpleNamespace(N=N, col_map=torch.tensor(cm, dtype=torch.int32, device=DEV))
    gW = torch.full((N, kmain + kray), float("nan"), device=DEV)
    gb = torch.full((N,), float("nan"), device=DEV)
    mlp._wgrad_rays(blocks, N4, lp, torch.empty(0, device=DEV), gW, gb, False, split)
    X, Y = torch.cat(ref_x), torch.cat(ref_y)
    refw = Y.T @ X
    bound = 2.0 ** -15 * (Y.abs().T @ X.abs()) + 1e-6
    assert ((gW.cpu().double() - refw).abs() <= bound).all()
    assert torch.allclose(gb.cpu().double(), Y.sum(0), rtol=1e-4, atol=2e-4)


def test_ray_split_refuses_a_block_boundary_inside_a_ray():
    """Two blocks whose rays of 256 samples would start inside a split (block 0 of 384 rows: a
    multiple of 128, not of 256) take the per-sample route instead."""
    from nerf_amd import mlp
    blocks = []
    for B, S in ((6, 64), (4, 256)):
        M = B * S
        blocks.append((torch.zeros(M, 128, device=DEV), [(torch.zeros(M, 256, device=DEV), 256, 1),
                                                         (torch.zeros(B, 24, device=DEV), 24, S)], M))
    assert mlp._ray_split(blocks, 128) is None
    assert mlp._ray_split(blocks[1:], 128) is not None


def test_ray_route_in_a_training_step():
    """A mip NerfInterpolation step with and without the per-ray route: parameter gradients within
    the split-precision spread (only the colour layer's direction columns change summation)."""
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel, mlp
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        g = torch.Generator(device=DEV).manual_seed(2)
        o = torch.randn(1024, 3, device=DEV, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 2.5], device=DEV)
        d = torch.nn.functional.normalize(torch.randn(1024, 3, device=DEV, generator=g) * 0.3
                                          - torch.tensor([0.0, 0.0, 1.0], device=DEV), dim=1)
        pw = torch.full((1024,), 1e-3, device=DEV)
        target = torch.rand(1024, 3, device=DEV, generator=g)
        grads = []
        for on in (False, True):
            torch.manual_seed(0)
            pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
            pos.pixel_width_sigma = 0.0
            dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
            model = NerfModel(4, 256, True, False, 2, pos, dirs).to(DEV)
            ren = NerfInterpolation(2.0, 8.0, model, 128, "stratified_uniform", -1.0, "middle", model, 64).to(DEV)
            saved = mlp.WGRAD_RAYS
            mlp.WGRAD_RAYS = on
            try:
                torch.manual_seed(5)
                fine, coarse = ren(o, d, pw)
                (((fine - target) ** 2).mean() + ((coarse - target) ** 2).mean()).backward()
            finally:
                mlp.WGRAD_RAYS = saved
            torch.cuda.synchronize()
            grads.append({n: p.grad.clone() for n, p in model.named_parameters()})
        for n, a in grads[1].items():
            b = grads[0][n]
            assert (a - b).abs().max() <= 1e-4 * b.abs().max() + 1e-12, n
    finally:
        torch.set_float32_matmul_precision(prev)
