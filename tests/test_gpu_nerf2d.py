"""GPU parity for config C1 (2d-reconstruction, nerf_amd.Nerf2d) and the tanh GEMM epilogues
(NERF_EPI_TANH / NERF_EPI_TANH_BWD) it runs on, through the C-ABI.

Tolerances (fp32): tanh epilogue vs torch 2e-6 abs (libm tanh ulps on |y| <= 1; the GEMM part is
compared through the same kernel without the epilogue); Nerf2d forward 2e-5 (fp32 MFMA) / 2e-4
(3 x bf16 split, ~2^-16 per product over K = 40..256) against the reference run in
tests/golden/nerf2d.npz; gradients 1e-4 / 1e-3 relative to the tensor's largest entry; three
Adam steps: parameters within 1e-5 / 1e-4 of the reference's (Adam's first steps move every
weight by ~lr whatever the gradient's size, so parameter error stays at the gradient-sign level).
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import nerf_amd
    nerf_amd._lib.load()
    yield


@pytest.fixture(params=["highest", "high"])
def matmul_precision(request):
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(request.param)
    yield request.param
    torch.set_float32_matmul_precision(old)


def _tol(prec, fp32, x3):
    return fp32 if prec == "highest" else x3


@pytest.mark.parametrize("N", [3, 64, 256, 320])
def test_tanh_epilogues_vs_torch(matmul_precision, N):
    """y = tanh(x W^T + b) and g * (1 - y^2) (+ accumulate) from the GEMM epilogues, against the
    same kernels without the epilogue followed by torch's tanh / tanh_backward formula."""
    from nerf_amd import kernels as K
    from nerf_amd._lib import NERF_EPI_ACCUM, NERF_EPI_BIAS, NERF_EPI_TANH, NERF_EPI_TANH_BWD
    from nerf_amd.mlp import LayerPlan, Source, matmul_precision as prec_of
    torch.manual_seed(N)
    M, Kin = 5003, 96
    lin = torch.nn.Linear(Kin, N).to(DEV)
    lp = LayerPlan(lin, [Source("act", Kin, K.pad32(Kin), 0)], False, tanh=True)
    lp.finalize(torch.device(DEV))
    prec = prec_of()
    lp.pack(prec)
    x = torch.randn(M, Kin, device=DEV)
    segs = [(x, Kin, 1)]
    ld = (N + 3) // 4 * 4
    z = torch.empty(M, ld, device=DEV)
    y = torch.empty(M, ld, device=DEV)
    lp.gemm(prec, segs, M, False, N, lin.bias, z, NERF_EPI_BIAS)
    lp.gemm(prec, segs, M, False, N, lin.bias, y, NERF_EPI_BIAS | NERF_EPI_TANH)
    torch.testing.assert_close(y[:, :N], torch.tanh(z[:, :N]), atol=2e-6, rtol=0)
    # backward epilogue: g * (1 - y^2), then accumulated onto an existing gradient
    g = torch.empty(M, ld, device=DEV)
    lp.gemm(prec, segs, M, False, N, None, g, 0)
    dz = torch.empty(M, ld, device=DEV)
    lp.gemm(prec, segs, M, False, N, None, dz, NERF_EPI_TANH_BWD, aux=y)
    ref = g[:, :N] * (1 - y[:, :N] * y[:, :N])
    torch.testing.assert_close(dz[:, :N], ref, atol=1e-6, rtol=1e-6)
    base = torch.randn(M, ld, device=DEV)
    acc = base.clone()
    lp.gemm(prec, segs, M, False, N, None, acc, NERF_EPI_TANH_BWD | NERF_EPI_ACCUM, aux=y)
    torch.testing.assert_close(acc[:, :N], base[:, :N] + ref, atol=1e-5, rtol=1e-6)


def test_nerf2d_vs_reference(golden, matmul_precision):
    from nerf_amd import Nerf2d
    g = golden("nerf2d")
    torch.manual_seed(0)
    m = Nerf2d(64, 48, 10)
    for k, v in m.state_dict().items():
        ref = g[f"init_sum.{k}"]
        assert abs(v.double().abs().sum().item() - ref[1]) <= 1e-9 * max(1.0, ref[1]), k
    m = m.to(DEV)
    x = torch.from_numpy(g["x"]).to(DEV)
    y = torch.from_numpy(g["y"]).to(DEV)
    pe = m.model[0](x)
    torch.testing.assert_close(pe.cpu(), torch.from_numpy(g["pe"]), atol=2e-6, rtol=0)
    y_hat = m(x)
    tol = _tol(matmul_precision, 2e-5, 2e-4)
    np.testing.assert_allclose(y_hat.detach().cpu().numpy(), g["y_hat"], atol=tol, rtol=0)
    loss = m.training_step((x, y))
    np.testing.assert_allclose(loss.item(), g["loss"][0], rtol=tol)
    loss.backward()
    gtol = _tol(matmul_precision, 1e-4, 1e-3)
    for k, p in m.named_parameters():
        ref = g[f"grad.{k}"]
        np.testing.assert_allclose(p.grad.cpu().numpy(), ref, atol=gtol * np.abs(ref).max(), rtol=0, err_msg=k)
    # three Adam steps (the GPU optimizer is nerf_amd's fused launch)
    m.zero_grad()
    opt = m.configure_optimizers()["optimizer"]
    opt.param_groups[0]["lr"] = 1e-3
    for _ in range(3):
        opt.zero_grad()
        m.training_step((x, y)).backward()
        opt.step()
    ptol = _tol(matmul_precision, 1e-5, 1e-4)
    for k, v in m.state_dict().items():
        np.testing.assert_allclose(v.reshape(-1)[:256].cpu().numpy(), g[f"adam3_head.{k}"], atol=ptol, err_msg=k)
        ref = g[f"adam3_sum.{k}"]
        assert abs(v.double().abs().sum().item() - ref[1]) <= ptol * v.numel(), k


def test_nerf2d_fit_vs_oracle():
    """A 40-step fit of a procedural 48 x 64 image (the reference's SingleImageDataModule
    coordinates: x / width, y / height over an ij meshgrid) on the GPU in fp32 against the CPU
    oracle with torch Adam from the same init: final losses within 1 %."""
    import math
    from nerf_amd import Nerf2d
    H, W = 48, 64
    xs, ys = torch.meshgrid(torch.arange(W), torch.arange(H), indexing="ij")
    xs, ys = xs.flatten(), ys.flatten()
    loc = torch.stack((xs.float() / W, ys.float() / H), dim=1)
    img = torch.stack((0.5 + 0.5 * torch.sin(6 * loc[:, 0]), 0.5 + 0.5 * torch.cos(9 * loc[:, 1]),
                       loc[:, 0] * loc[:, 1]), dim=1)
    torch.manual_seed(0)
    m = Nerf2d(W, H, 10, learning_rate=1e-3)
    sd = {k: v.clone().requires_grad_(True) for k, v in m.state_dict().items()}
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        m = m.to(DEV)
        opt = m.configure_optimizers()["optimizer"]
        xg, yg = loc.to(DEV), img.to(DEV)
        for _ in range(40):
            opt.zero_grad()
            m.training_step((xg, yg)).backward()
            opt.step()
        gpu_loss = m.validation_step((xg, yg)).item()
    finally:
        torch.set_float32_matmul_precision(prev)
    opt_c = torch.optim.Adam(list(sd.values()), lr=1e-3)
    for _ in range(40):
        opt_c.zero_grad()
        torch.nn.functional.mse_loss(O.nerf2d_forward(sd, loc, 10), img).backward()
        opt_c.step()
    with torch.no_grad():
        cpu_loss = torch.nn.functional.mse_loss(O.nerf2d_forward(sd, loc, 10), img).item()
    assert math.isfinite(gpu_loss) and abs(gpu_loss - cpu_loss) <= 0.01 * cpu_loss, (gpu_loss, cpu_loss)
