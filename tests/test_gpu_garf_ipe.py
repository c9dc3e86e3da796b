"""GPU parity for the integrated-encoding backward (a3) and the GARF Gaussian-activation
field MLPs (a8), through the C-ABI, against the reference's golden vectors.

Tolerances (fp32): IPE outputs 2e-6 abs; IPE gradients as the Fourier/BARF d/dx test
(2e-3 abs + 1e-5 rel: sums of ~20 terms up to scale*2^9*|g|); GaussAct 1e-6 rel (libm exp ulps);
GARF networks 1e-4 (fp32 MFMA) / 2e-3 (3 x bf16 split, ~2^-16 per product, deep Gaussian chain).
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def g2d(a):
    return torch.from_numpy(np.asarray(a)).to(DEV)


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


@pytest.mark.parametrize("key", ["ipe_dv1_pws0.0", "ipe_dv1_pws0.5", "ipe_dv0_pws0.0", "ipe_dv0_pws0.5",
                                 "ipebarf_dv1_a6.3", "ipebarf_dv0_a6.3"])
def test_integrated_encoding_grads(golden, key):
    from nerf_amd import IntegratedBarfFourierFeatures, IntegratedFourierFeatures
    g = golden("ipe_grad")
    dv = "_dv1" in key
    if key.startswith("ipebarf"):
        enc = IntegratedBarfFourierFeatures(10, 6.3, 0, 1, True, 1.0, dv).to(DEV)
        enc.pixel_width_sigma = 0.0
    else:
        enc = IntegratedFourierFeatures(10, 2 * np.pi, True, dv)
        enc.pixel_width_sigma = 0.5 if key.endswith("pws0.5") else 0.0
    x = g2d(g["x"]).requires_grad_(True)
    d = g2d(g["dir"]).requires_grad_(True)
    y = enc(x, d, g2d(g["pw"]), g2d(g["t0"]), g2d(g["t1"]))
    np.testing.assert_allclose(y.detach().cpu().numpy(), g[key], atol=2e-6, rtol=0)
    (y * g2d(g[key + "_gy"])).sum().backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), g[key + "_dx"], atol=2e-3, rtol=1e-5)
    np.testing.assert_allclose(d.grad.cpu().numpy(), g[key + "_ddir"], atol=2e-3, rtol=1e-5)


def test_integrated_encoding_grads_random_vs_oracle():
    """Larger batch, per-sample widths and intervals, both variance modes, vs the oracle's autograd."""
    from nerf_amd import IntegratedFourierFeatures
    torch.manual_seed(11)
    N = 5000
    x = torch.rand(N, 3) * 6 - 3
    d = torch.nn.functional.normalize(torch.randn(N, 3), dim=1) * (0.5 + torch.rand(N, 1))
    t0 = 2 + torch.rand(N, 1) * 6
    t1 = t0 + torch.rand(N, 1) * 0.3 + 1e-3
    pw = 1e-3 + torch.rand(N, 1) * 2e-3
    gy = torch.randn(N, 63)
    for dv in (True, False):
        enc = IntegratedFourierFeatures(10, 2 * np.pi, True, dv)
        enc.pixel_width_sigma = 0.7
        xg, dg = x.to(DEV).requires_grad_(True), d.to(DEV).requires_grad_(True)
        y = enc(xg, dg, pw.to(DEV), t0.to(DEV), t1.to(DEV))
        (y * gy.to(DEV)).sum().backward()
        xo, do = x.clone().requires_grad_(True), d.clone().requires_grad_(True)
        yo = O.integrated_pe(xo, do, pw, t0, t1, 10, 2 * np.pi, True, dv, 0.7)
        (yo * gy).sum().backward()
        np.testing.assert_allclose(y.detach().cpu().numpy(), yo.detach().numpy(), atol=2e-6, rtol=0)
        np.testing.assert_allclose(xg.grad.cpu().numpy(), xo.grad.numpy(), atol=2e-3, rtol=1e-5)
        np.testing.assert_allclose(dg.grad.cpu().numpy(), do.grad.numpy(), atol=2e-3, rtol=1e-5)


def test_gauss_act_golden(golden):
    from nerf_amd import GaussAct
    g = golden("garf")
    act = GaussAct(48).to(DEV)
    with torch.no_grad():
        act.inv_standard_deviation.copy_(g2d(g["act.s"]))
    z = g2d(g["act.z"]).requires_grad_(True)
    y = act(z)
    np.testing.assert_allclose(y.detach().cpu().numpy(), g["act.y"], atol=1e-7, rtol=1e-6)
    (y * g2d(g["act.gy"])).sum().backward()
    np.testing.assert_allclose(z.grad.cpu().numpy(), g["act.dz"], atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(act.inv_standard_deviation.grad.cpu().numpy(), g["act.ds"], atol=1e-5, rtol=1e-5)


def test_gauss_act_large_vs_oracle():
    """Many slabs (M > 512 * 1024) and a ragged column count; the inverse-std gradient is
    deterministic (fixed-order slab reduction): two runs are bit-identical."""
    from nerf_amd import GaussAct
    torch.manual_seed(12)
    M, N = 600_000, 37
    z = torch.randn(M, N)
    act = GaussAct(N, 0.5, 2.0).to(DEV)
    s = act.inv_standard_deviation.detach().cpu().clone()
    gy = torch.randn(M, N)
    grads = []
    for _ in range(2):
        act.inv_standard_deviation.grad = None
        zd = z.to(DEV).requires_grad_(True)
        y = act(zd)
        (y * gy.to(DEV)).sum().backward()
        grads.append(act.inv_standard_deviation.grad.clone())
    assert torch.equal(grads[0], grads[1])
    zo, so = z.clone().requires_grad_(True), s.clone().requires_grad_(True)
    yo = O.gauss_act(zo, so)
    (yo * gy).sum().backward()
    np.testing.assert_allclose(y.detach().cpu().numpy(), yo.detach().numpy(), atol=1e-7, rtol=1e-6)
    np.testing.assert_allclose(zd.grad.cpu().numpy(), zo.grad.numpy(), atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(grads[0].cpu().numpy(), so.grad.numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("name", ["radiance", "proposal"])
def test_garf_networks_golden(golden, name, matmul_precision):
    from nerf_amd import ProposalNetwork, RadianceNetwork
    g = golden("garf")
    torch.manual_seed(0)
    m = (RadianceNetwork if name == "radiance" else ProposalNetwork)(0.5, 2.0, 5e-4, 5e-5, 0, 1.0, 0.0)
    for k, v in m.state_dict().items():
        ref = g[f"{name}.sdsum.{k}"]
        assert abs(v.double().abs().sum().item() - ref[1]) <= 1e-9 * max(1.0, ref[1]), k
    m = m.to(DEV)
    tol = 1e-4 if matmul_precision == "highest" else 2e-3
    pos = g2d(g["pos"]).requires_grad_(True)
    if name == "radiance":
        d = g2d(g["dir"]).requires_grad_(True)
        rgb, dens = m(pos, d)
        np.testing.assert_allclose(rgb.detach().cpu().numpy(), g["radiance.rgb"], atol=tol, rtol=tol)
        np.testing.assert_allclose(dens.detach().cpu().numpy(), g["radiance.density"], atol=tol, rtol=tol)
        ((rgb * g2d(g["radiance.gc"])).sum() + (dens * g2d(g["radiance.gd"])).sum()).backward()
        np.testing.assert_allclose(d.grad.cpu().numpy(), g["radiance.ddir"], atol=10 * tol, rtol=10 * tol)
    else:
        dens = m(pos)
        assert dens.shape == (pos.shape[0], 1)
        np.testing.assert_allclose(dens.detach().cpu().numpy(), g["proposal.density"], atol=tol, rtol=tol)
        (dens * g2d(g["proposal.gd"])).sum().backward()
    np.testing.assert_allclose(pos.grad.cpu().numpy(), g[f"{name}.dpos"], atol=10 * tol, rtol=10 * tol)
    for k, prm in m.named_parameters():
        s = g[f"{name}.gradsum.{k}"]
        assert abs(prm.grad.double().abs().sum().item() - s[1]) <= 10 * tol * s[1] + 1e-6, k
        key = f"{name}.grad.{k}"
        if key in g:
            np.testing.assert_allclose(prm.grad.cpu().numpy(), g[key],
                                       atol=10 * tol * max(1.0, np.abs(g[key]).max()), rtol=10 * tol)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["radiance", "proposal"])
def test_garf_gauss_epilogue_matches_separate_passes(name):
    """The Gaussian activation fused into the split-precision GEMM epilogues (forward: z and
    exp(-z^2 v) from one launch; backward: dL/dz and the inverse-std column partials from the
    consumer's input-gradient GEMM) against the separate nerf_gauss_act passes on the same GEMMs:
    outputs and input gradients bit-identical, inverse-std gradients equal up to the fp64 summation
    order, every other parameter gradient bit-identical.  M = 70,001 rows: ragged 256-row tiles, the
    1024- and 512-wide layers in 256-column blocks of the 256-row tile kernel."""
    from nerf_amd import ProposalNetwork, RadianceNetwork
    from nerf_amd import mlp as mlp_mod
    torch.manual_seed(3)
    M = 70_001
    pos = (torch.rand(M, 3) * 2 - 1).to(DEV)
    d = torch.nn.functional.normalize(torch.randn(M, 3), dim=-1).to(DEV)
    gc, gd = torch.randn(M, 3).to(DEV), torch.randn(M, 1).to(DEV)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    results = []
    try:
        for fused in (True, False):
            mlp_mod.GAUSS_EPILOGUE = fused
            torch.manual_seed(0)
            m = (RadianceNetwork if name == "radiance" else ProposalNetwork)(0.5, 2.0).to(DEV)
            p = pos.clone().requires_grad_(True)
            if name == "radiance":
                rgb, dens = m(p, d)
                loss = (rgb * gc).sum() + (dens * gd).sum()
                outs = [rgb.detach(), dens.detach()]
            else:
                dens = m(p)
                loss = (dens * gd).sum()
                outs = [dens.detach()]
            loss.backward()
            results.append((outs, p.grad.clone(), {k: v.grad.clone() for k, v in m.named_parameters()}))
    finally:
        mlp_mod.GAUSS_EPILOGUE = True
        torch.set_float32_matmul_precision(prev)
    (o1, dp1, g1), (o2, dp2, g2) = results
    for a, b in zip(o1, o2):
        assert torch.equal(a, b)
    assert torch.equal(dp1, dp2)
    for k in g1:
        if k.endswith("inv_standard_deviation"):
            torch.testing.assert_close(g1[k], g2[k], rtol=1e-5, atol=1e-6, msg=k)
        else:
            assert torch.equal(g1[k], g2[k]), k


NBLOCK_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {pkg!r})
from nerf_amd import RadianceNetwork
torch.set_float32_matmul_precision("high")
dev = torch.device("cuda", 0)
torch.manual_seed(3)
M = 70_001
pos = (torch.rand(M, 3) * 2 - 1).to(dev).requires_grad_(True)
d = torch.nn.functional.normalize(torch.randn(M, 3), dim=-1).to(dev)
gc, gd = torch.randn(M, 3).to(dev), torch.randn(M, 1).to(dev)
torch.manual_seed(0)
m = RadianceNetwork(0.5, 2.0).to(dev)
rgb, dens = m(pos, d)
((rgb * gc).sum() + (dens * gd).sum()).backward()
out = {{"rgb": rgb.detach().cpu(), "dens": dens.detach().cpu(), "dpos": pos.grad.cpu()}}
out.update({{k: v.grad.cpu() for k, v in m.named_parameters()}})
torch.save(out, sys.argv[1])
"""


@pytest.mark.gpu
def test_wide_layers_column_blocks_match_the_128_tile_kernel(tmp_path):
    """GARF's radiance network with its 1024- and 512-wide layers (forward with the Gaussian epilogue,
    and the input gradients into them) as 256-column blocks of the 256-row tile kernel
    (NERF_NT_NBLOCK=1, the default) against the 128 x 128 tile kernel (NERF_NT_NBLOCK=0; the switch
    is read once per process, so each runs in a child): the two kernels round their 3 x bf16 split
    products differently (each within 2^-16 of scale), so outputs agree within 1e-5 of scale and the
    gradients, through several such layers, within 1e-4."""
    import os
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nerf-experiments_amd")
    res = []
    for on in ("1", "0"):
        f = tmp_path / f"nb{on}.pt"
        r = subprocess.run([sys.executable, "-c", NBLOCK_SCRIPT.format(pkg=pkg), str(f)],
                           env=dict(os.environ, NERF_NT_NBLOCK=on), capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        res.append(torch.load(f, weights_only=True))
    for k, a in res[0].items():
        b = res[1][k]
        assert torch.isfinite(a).all(), k
        tol = 1e-5 if k in ("rgb", "dens") else 1e-4
        assert (a - b).abs().max() <= tol * b.abs().max() + 1e-12, (k, (a - b).abs().max().item())
