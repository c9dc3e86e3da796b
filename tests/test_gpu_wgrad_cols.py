"""Weight gradient of a layer larger than one 256 x 256 tile — mip-NeRF's skip layer [trunk
activation 256 | encoding] (NerfModel's skip connections, barf/model_mip.py:85-130), GARF's
Linear(1024, 256), Linear(512, 256), Linear(131, 512) (garf/model_radiance.py, model_proposal.py) —
as single-tile launches over row blocks and column groups (mlp._tile_split / _wgrad_tiles; a group
of <= 128 columns runs linear_wgrad_x3_tr_kernel<..., JN = 1> over all four SIMDs).  Against fp64 with the
split-precision bound of test_gpu_parity.py (2^-15 of |dY|^T |X|), one or two row blocks, 256 and
257 output rows, segments padded to 32 columns (widths a multiple of 4, as the kernels require); and
the layer-level switch (NERF_WGRAD_TILESPLIT) on a mip NerfInterpolation step and on GARF's
radiance network."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M0,M1,N,ks", [(50000, 0, 256, (256, 96)), (30000, 70001, 256, (256, 60)),
                                        (65536, 0, 257, (256, 96)), (32768, 20000, 257, (128, 128, 60)),
                                        (4096, 8192, 200, (192, 96, 24)), (20000, 30000, 512, (128, 4)),
                                        (30000, 0, 256, (1024,)), (10000, 20000, 256, (128, 512)),
                                        (20000, 0, 500, (512,))])
def test_wgrad_cols_matches_fp64(M0, M1, N, ks):
    from nerf_amd import kernels as K, mlp
    torch.manual_seed(M0 + M1 + N)
    N4 = (N + 3) // 4 * 4
    nrow = N if N == 257 else N4
    blocks, ref_x, ref_y = [], [], []
    for M in (M0, M1):
        if M == 0:
            continue
        dY = torch.randn(M, N4)
        dY[:, N:] = 0
        xs = [torch.randn(M, k) for k in ks]
        blocks.append((dY.to(DEV), [(x.to(DEV), k, 1) for x, k in zip(xs, ks)], M))
        ref_x.append(torch.cat(xs, dim=1).double())
        ref_y.append(dY[:, :N].double())
    split = mlp._tile_split(blocks[0][1], nrow)
    assert split is not None
    cm, base = [], 0
    for k in ks:
        cm += [base + j for j in range(k)] + [-1] * (K.pad32(k) - k)
        base += k
    lp = types.SimpleNamespace(N=N, col_map=torch.tensor(cm, dtype=torch.int32, device=DEV))
    gW = torch.full((N, sum(ks)), float("nan"), device=DEV)
    gb = torch.full((N,), float("nan"), device=DEV)
    mlp._wgrad_tiles(blocks, nrow, N4, lp, torch.empty(0, device=DEV), gW, gb, False, split, 3)
    X, Y = torch.cat(ref_x), torch.cat(ref_y)
    refw = Y.T @ X
    bound = 2.0 ** -15 * (Y.abs().T @ X.abs()) + 1e-6
    assert ((gW.cpu().double() - refw).abs() <= bound).all()
    assert torch.allclose(gb.cpu().double(), Y.sum(0), rtol=1e-4, atol=2e-4)


def test_tile_split_in_a_training_step():
    """A mip NerfInterpolation step (skip layer [256 | 63-wide integrated encoding]) with and without
    the tile split: parameter gradients within the split-precision spread."""
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel, mlp
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        g = torch.Generator(device=DEV).manual_seed(3)
        o = torch.randn(1024, 3, device=DEV, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 2.5], device=DEV)
        d = torch.nn.functional.normalize(torch.randn(1024, 3, device=DEV, generator=g) * 0.3
                                          - torch.tensor([0.0, 0.0, 1.0], device=DEV), dim=1)
        pw = torch.full((1024,), 1e-3, device=DEV)
        target = torch.rand(1024, 3, device=DEV, generator=g)
        grads, used = [], []
        for on in (False, True):
            torch.manual_seed(0)
            pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
            pos.pixel_width_sigma = 0.0
            dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
            model = NerfModel(4, 256, True, False, 2, pos, dirs).to(DEV)
            ren = NerfInterpolation(2.0, 8.0, model, 128, "stratified_uniform", -1.0, "middle", model, 64).to(DEV)
            saved, saved_fn = mlp.WGRAD_TILESPLIT, mlp._wgrad_tiles
            calls = []
            mlp.WGRAD_TILESPLIT = on
            mlp._wgrad_tiles = lambda *a, **kw: (calls.append(1), saved_fn(*a, **kw))
            try:
                torch.manual_seed(5)
                fine, coarse = ren(o, d, pw)
                (((fine - target) ** 2).mean() + ((coarse - target) ** 2).mean()).backward()
            finally:
                mlp.WGRAD_TILESPLIT, mlp._wgrad_tiles = saved, saved_fn
            torch.cuda.synchronize()
            used.append(len(calls))
            grads.append({n: p.grad.clone() for n, p in model.named_parameters()})
        assert used[0] == 0 and used[1] >= 1, used
        for n, a in grads[1].items():
            b = grads[0][n]
            assert (a - b).abs().max() <= 1e-4 * b.abs().max() + 1e-12, n
    finally:
        torch.set_float32_matmul_precision(prev)


def test_tile_split_garf_radiance():
    """GARF's radiance network forward + backward with and without the tile split: parameter
    gradients within the split-precision spread, and the split route taken."""
    from nerf_amd import RadianceNetwork, mlp
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        g = torch.Generator(device=DEV).manual_seed(4)
        pos = torch.randn(8192, 3, device=DEV, generator=g) * 0.5
        d = torch.nn.functional.normalize(torch.randn(8192, 3, device=DEV, generator=g), dim=1)
        grads, used = [], []
        for on in (False, True):
            torch.manual_seed(0)
            net = RadianceNetwork(0.5, 2.0).to(DEV)
            saved, saved_fn = mlp.WGRAD_TILESPLIT, mlp._wgrad_tiles
            calls = []
            mlp.WGRAD_TILESPLIT = on
            mlp._wgrad_tiles = lambda *a, **kw: (calls.append(1), saved_fn(*a, **kw))
            try:
                rgb, dens = net(pos, d)
                (rgb.square().sum() + dens.sum()).backward()
            finally:
                mlp.WGRAD_TILESPLIT, mlp._wgrad_tiles = saved, saved_fn
            torch.cuda.synchronize()
            used.append(len(calls))
            grads.append({n: p.grad.clone() for n, p in net.named_parameters()})
        assert used[0] == 0 and used[1] >= 3, used
        for n, a in grads[1].items():
            b = grads[0][n]
            assert torch.isfinite(a).all(), n
            assert (a - b).abs().max() <= 1e-4 * b.abs().max() + 1e-12, n
    finally:
        torch.set_float32_matmul_precision(prev)
