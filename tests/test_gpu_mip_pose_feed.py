"""GPU parity of three reference APIs against fixtures produced by the reference itself
(tests/golden/make_golden.py): the older mip_NeRF directory's integrated encoding / MipNerfModel /
MipNerf renderer (mip_NeRF/mip_model.py:11-167), BARF pose gradients through the whole rendering
path (CameraExtrinsics -> _compute_color -> backward; barf/model_barf.py:29-92), and the on-device
training-batch feed (barf/dataset.py:407-637, data_module.py:276-369).

Tolerances: encodings 2e-6 absolute (fp32 sin/cos of the same fp32 argument); field-MLP outputs and
rendered colours 1e-4 absolute in exact-fp32 MFMA ("highest") and 2e-4 in split precision ("high",
three bf16 products per fp32 product, ~2^-17 relative each); pose gradients 1e-3 of their largest
magnitude in exact fp32 ("highest"); in split precision ("high") a conditioning bound: the pose
gradients sum thousands of per-sample position gradients that largely cancel (the translation
gradient's condition number is ~3e3: the reference's own fp32 result sits 1.7e-4 of its magnitude
away from fp64), so the test computes the fp64 value with the CPU oracle and requires the
split-precision error to stay within 2 x 2^9 x the fp32 reference's own error (2^9 = the ratio of
the per-product error bounds, 2^-15 for three bf16 products vs 2^-24; tools/pose_grad_conditioning.py prints the numbers:
translation: fp32 1.7e-4, "highest" 1.8e-4, "high" 5.5e-2;
rotation: fp32 5.0e-6, "highest" 4.9e-6, "high" 2.8e-3 — the reference's TF32 "high" setting, 2^-11 per
product, would be another 32x worse).  The split-precision bounds are stated per quantity
(HIGH_POSE_GRAD_BOUND: rotation 4.5e-3, translation 8e-2 of the largest gradient), and
test_gpu_barf_fit_precision.py shows on a fixed-seed BARF fit that this error leaves PSNR and pose
convergence unchanged within its stated bounds; feed: gathers bit-exact, directions 3e-7
(the kernel recomputes each pixel's direction instead of gathering the reference's batched matmul)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import nerf_amd
    nerf_amd._lib.load()
    prev = torch.get_float32_matmul_precision()
    yield
    torch.set_float32_matmul_precision(prev)


def t(a, dev=DEV):
    return torch.from_numpy(np.asarray(a)).to(dev)


# ------------------------------------------------------------------------------------------- mip_NeRF
@pytest.mark.parametrize("dv", [0, 1])
def test_mipnerf_integrated_encoding(golden, dv):
    from nerf_amd.mip_model import IntegratedFourierFeatures
    g = golden("mipnerf")
    enc = IntegratedFourierFeatures(10, 2 * math.pi, bool(dv))
    y = enc.forward(t(g["x"]), t(g["dir"]), t(g["t0"]), t(g["t1"]), 1 / 1111.1)
    assert y.shape == (g["x"].shape[0], 60)
    np.testing.assert_allclose(y.cpu().numpy(), g[f"ipe_dv{dv}"], atol=2e-6, rtol=0)
    # the same variant pinned in pe.npz (argument given per call, distribute_variance=True)
    p = golden("pe")
    enc2 = IntegratedFourierFeatures(10, 2 * math.pi, False)
    y2 = enc2.forward(t(p["x"]), t(p["dir"]), t(p["t0"]), t(p["t1"]), 1 / 1111.1, distribute_variance=True)
    np.testing.assert_allclose(y2.cpu().numpy(), p["mipnerf_ipe_800"], atol=2e-6, rtol=0)


@pytest.mark.parametrize("precision,tol", [("highest", 1e-4), ("high", 2e-4)])
def test_mipnerf_model_forward_backward(golden, precision, tol):
    from nerf_amd.mip_model import MipNerfModel
    torch.set_float32_matmul_precision(precision)
    g = golden("mipnerf")
    torch.manual_seed(0)
    model = MipNerfModel(4, 256, (True, 10, 4), 2, True)
    for k, v in model.state_dict().items():
        np.testing.assert_allclose([v.double().sum().item(), v.double().abs().sum().item()], g[f"model.sdsum.{k}"],
                                   rtol=1e-12, atol=1e-9)
    model = model.to(DEV)
    dens, rgb = model(t(g["x"]), t(g["dir"]), t(g["t0"]), t(g["t1"]), 1 / 1111.1)
    np.testing.assert_allclose(dens.detach().cpu().numpy(), g["model.density"], atol=tol, rtol=0)
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), g["model.rgb"], atol=tol, rtol=0)
    ((dens * t(g["model.gd"])).sum() + (rgb * t(g["model.gc"])).sum()).backward()
    for k, prm in model.named_parameters():
        want = g[f"model.gradsum.{k}"]
        got = prm.grad.double().abs().sum().item()
        assert abs(got - want[1]) <= 2e-3 * max(want[1], 1e-6), (k, got, want[1])


@pytest.mark.parametrize("precision,tol", [("highest", 1e-4), ("high", 2e-4)])
def test_mipnerf_renderer_coarse_fine(golden, precision, tol):
    from nerf_amd.mip_model import MipNerf
    torch.set_float32_matmul_precision(precision)
    g = golden("mipnerf")
    torch.manual_seed(0)
    ren = MipNerf(1.0, 5.0, 96, 4, (True, 32), (True, 10, 4), 2, distribute_variance=True).to(DEV)
    tc = t(g["ren.tc"])
    ren._sample_t_stratified_uniform = lambda *a, **k: ren._get_intervals(tc.clone())
    rgb_f, rgb_c = ren(t(g["ren.o"]), t(g["ren.d"]), t(g["ren.pw"]))
    np.testing.assert_allclose(rgb_c.detach().cpu().numpy(), g["ren.rgb_coarse"], atol=tol, rtol=0)
    np.testing.assert_allclose(rgb_f.detach().cpu().numpy(), g["ren.rgb_fine"], atol=tol, rtol=0)
    assert int(ren.last_resample_status.item()) & 1 == 0


# ------------------------------------------------------------------------------------ pose gradients
def _oracle_pose_grads_fp64(g):
    """The fixture's pose gradients recomputed by the CPU oracle in float64 (same weights, rays, t)."""
    from oracle import nerf_oracle as O
    from nerf_amd import BarfPositionalEncoding, NerfModel
    dt = torch.float64
    torch.manual_seed(0)
    sd = NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 6.3, 0, 1, True, 1.0),
                   BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0)).state_dict()
    sd = {k: v.to(dt) for k, v in sd.items() if not k.endswith("alpha")}
    rot = torch.tensor(g["rotation"], dtype=dt, requires_grad=True)
    trans = torch.tensor(g["translation"], dtype=dt, requires_grad=True)
    idx = torch.from_numpy(g["idx"])
    R = torch.matrix_exp(torch.cross(-torch.eye(3, dtype=dt).view(1, 3, 3), rot.view(-1, 3, 1), dim=1))
    o2 = torch.tensor(g["o"], dtype=dt) + trans[idx]
    d2 = torch.matmul(R[idx], torch.tensor(g["d"], dtype=dt).unsqueeze(-1)).squeeze(-1)
    t0, t1 = torch.tensor(g["t0"], dtype=dt), torch.tensor(g["t1"], dtype=dt)
    B, S = t0.shape
    pos, dirs = O.compute_positions(o2, d2, t0, t1, "middle")

    def pe(x, L, alpha):
        args = x.repeat_interleave(L, dim=1) * (2.0 ** torch.arange(L, dtype=dt)).repeat(3)
        m = O.barf_mask(alpha, L).to(dt).repeat(3).view(1, -1)
        return torch.cat((x, m * torch.cos(args), m * torch.sin(args)), dim=1)
    dens, rgb = O.nerf_model_forward(sd, pe(pos.reshape(-1, 3), 10, 6.3), pe(dirs.reshape(-1, 3), 4, 4.0), 2, 4,
                                     True, False)
    b = (-dens.view(B, S) * (t1 - t0)) * 3.0 * (1 / 3)
    T = torch.cat((torch.ones(B, 1, dtype=dt), torch.exp(torch.cumsum(b[:, :-1], dim=1))), dim=1)
    out = torch.sum((T * (1 - torch.exp(b))).unsqueeze(-1) * rgb.view(B, S, 3), dim=1)
    (out * torch.tensor(g["grgb"], dtype=dt)).sum().backward()
    return {"drot": rot.grad.numpy(), "dtrans": trans.grad.numpy()}


# split-precision pose-gradient error vs fp64, relative to the largest |gradient|
HIGH_POSE_GRAD_BOUND = {"drot": 4.5e-3, "dtrans": 8e-2}


@pytest.mark.parametrize("precision,tol,gtol", [("highest", 1e-4, 1e-3), ("high", 2e-4, None)])
def test_pose_gradients_through_rendering(golden, precision, tol, gtol):
    from nerf_amd import BarfPositionalEncoding, NerfInterpolation, NerfModel
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    torch.set_float32_matmul_precision(precision)
    g = golden("pose_render")
    torch.manual_seed(0)
    model = NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 6.3, 0, 1, True, 1.0),
                      BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0))
    ren = NerfInterpolation(2.0, 8.0, model, 32, "equidistant", -1.0, "middle").to(DEV)
    extr = CameraExtrinsics(6, 1e-3, 1e-5, 100).to(DEV)
    with torch.no_grad():
        extr.rotation.copy_(t(g["rotation"]))
        extr.translation.copy_(t(g["translation"]))
    B, S = g["t0"].shape
    o2, d2, _, _ = extr(t(g["idx"]), t(g["o"]), t(g["d"]))
    rgb, w, _ = ren._compute_color(model, t(g["t0"]), t(g["t1"]), o2, d2, t(g["pw"]), B, S)
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), g["rgb"], atol=tol, rtol=0)
    np.testing.assert_allclose(w.detach().cpu().numpy(), g["w"], atol=tol, rtol=0)
    (rgb * t(g["grgb"])).sum().backward()
    ref64 = _oracle_pose_grads_fp64(g)
    for name, p in (("drot", extr.rotation), ("dtrans", extr.translation)):
        want, exact = g[name].astype(np.float64), ref64[name]
        got = p.grad.double().cpu().numpy()
        scale = np.abs(exact).max()
        fp32_err = np.abs(want - exact).max() / scale          # the reference's own fp32 error
        err = np.abs(got - exact).max() / scale
        if gtol is not None:
            assert np.abs(got - want).max() <= gtol * np.abs(want).max(), (name, np.abs(got - want).max())
            assert err <= 4 * fp32_err + 1e-6, (name, err, fp32_err)
        else:
            # stated bounds on this fixture (measured 2.8e-3 / 5.5e-2): within the
            # conditioning bound 2^10 x fp32_err above, and shown harmless to pose convergence by the
            # fixed-seed fit of test_gpu_barf_fit_precision.py
            assert err <= HIGH_POSE_GRAD_BOUND[name], (name, err, fp32_err)
            assert err <= 2 * 2 ** 9 * fp32_err + 1e-5, (name, err, fp32_err)


# ------------------------------------------------------------------------------------------------ feed
@pytest.mark.parametrize("sigma", [None, 0.1, 2.0, 5.0, 8.0])
def test_ray_feed_matches_reference_dataset(golden, sigma):
    from nerf_amd.ray_feed import DeviceRayFeed
    g = golden("feed")
    images, c2w, focal = torch.from_numpy(g["images"]), torch.from_numpy(g["c2w"]), float(g["focal"][0])
    sigmas = [float(s) for s in g["sigmas"]]
    feed = DeviceRayFeed(images, c2w, focal, 64, rotation_noise_sigma=0.1, translation_noise_sigma=0.2,
                         noise_seed=3, gaussian_blur_sigmas=sigmas, dataloader_seed=1, device=DEV)
    got = feed.batch(t(g["indices"]), sigma)
    o, on, d, dn, col, img, pw = [x.cpu() for x in got]
    assert torch.equal(o, torch.from_numpy(g["o_raw"])) and torch.equal(on, torch.from_numpy(g["o_noisy"]))
    assert torch.equal(img, torch.from_numpy(g["img_idx"]))
    assert (d - torch.from_numpy(g["d_raw"])).abs().max() <= 3e-7
    assert (dn - torch.from_numpy(g["d_noisy"])).abs().max() <= 3e-7
    want_col = g["colors"] if sigma is None else g[f"blur_{sigma}"]
    assert torch.equal(col, torch.from_numpy(want_col))
    assert torch.equal(pw, torch.from_numpy(g["pw"]))
    feed.check()
