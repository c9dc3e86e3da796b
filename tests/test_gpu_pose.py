"""GPU parity of the camera-pose alignment (nerf_kabsch) against the reference's
CameraCalibrationModel.kabsch_algorithm / compute_pose_error run in tests/golden/kabsch.npz.

Tolerances: R 1e-5 abs, t 1e-4 abs, c 1e-5 rel, pose error 1e-5 rel — the kernel sums in fp64
where the reference sums and decomposes in fp32 (the fixture's noise is far above that, so the
outlier sets agree)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("case", ["noisy", "outliers", "reflect", "small"])
def test_kabsch_and_pose_error_vs_reference(golden, case):
    from nerf_amd.pose import compute_pose_error, kabsch_algorithm, validation_transform_rays
    g = golden("kabsch")
    raw = torch.from_numpy(g[f"{case}.raw"]).to(DEV)
    pred = torch.from_numpy(g[f"{case}.pred"]).to(DEV)
    for ro in (1, 0):
        R, t, c = kabsch_algorithm(raw, pred, remove_outliers=bool(ro))
        np.testing.assert_allclose(R.cpu().numpy(), g[f"{case}.ro{ro}.R"], atol=1e-5)
        np.testing.assert_allclose(t.cpu().numpy(), g[f"{case}.ro{ro}.t"], atol=1e-4)
        np.testing.assert_allclose(float(c), g[f"{case}.ro{ro}.c"][0], rtol=1e-5)
        assert abs(float(torch.linalg.det(R)) - 1.0) < 1e-5       # a rotation, reflections fixed
    err = compute_pose_error(raw, pred)
    np.testing.assert_allclose(float(err), g[f"{case}.pose_error"][0], rtol=1e-5)
    # validation rays through the alignment: origins R o c + t, directions R d
    R, t, c = kabsch_algorithm(raw, pred)
    o2, d2, _ = validation_transform_rays(raw, raw, (R, t, c))
    torch.testing.assert_close(o2, (R @ raw.T).T * c + t)
    torch.testing.assert_close(d2, (R @ raw.T).T)


def test_kabsch_recovers_exact_similarity_and_is_deterministic():
    """Noise-free similarity transform of 1000 points: recovered exactly; two launches agree bitwise."""
    from nerf_amd.pose import kabsch_algorithm
    torch.manual_seed(5)
    a = torch.randn(1000, 3, dtype=torch.float64)
    v = torch.randn(3, dtype=torch.float64)
    Kx = torch.tensor([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]], dtype=torch.float64)
    R0 = torch.linalg.matrix_exp(Kx)
    b = (R0 @ a.T).T * 1.7 + torch.tensor([0.3, -2.0, 5.0], dtype=torch.float64)
    A, B = a.float().to(DEV), b.float().to(DEV)
    R1, t1, c1 = kabsch_algorithm(A, B, remove_outliers=False)
    R2, t2, c2 = kabsch_algorithm(A, B, remove_outliers=False)
    assert torch.equal(R1, R2) and torch.equal(t1, t2) and torch.equal(c1, c2)
    np.testing.assert_allclose(R1.cpu().numpy(), R0.numpy(), atol=2e-6)
    np.testing.assert_allclose(float(c1), 1.7, rtol=2e-6)
    np.testing.assert_allclose(t1.cpu().numpy()[0], [0.3, -2.0, 5.0], atol=5e-5)


# ------------------------------------------------------------------ camera refinement (nerf_pose_rays_*)
def _pose_case(n_img, B, scale, seed):
    g = torch.Generator().manual_seed(seed)
    rot = torch.randn(n_img, 3, generator=g) * scale
    trans = torch.randn(n_img, 3, generator=g)
    idx = torch.randint(0, max(1, n_img - 1), (B,), generator=g)       # the last image gets no rays
    o = torch.randn(B, 3, generator=g) * 2.0
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=1)
    return rot, trans, idx, o, d


def test_camera_extrinsics_vs_reference_fixture(golden):
    """CameraExtrinsics.forward on the HIP kernels vs the reference run (tests/golden/pose.npz):
    rays and rotations 1e-6 abs; parameter gradients as the CPU oracle test bounds them."""
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    g = golden("pose")
    m = CameraExtrinsics(10, 1e-3, 1e-5, 100).to(DEV)
    with torch.no_grad():
        m.rotation.copy_(torch.from_numpy(g["rotation"]))
        m.translation.copy_(torch.from_numpy(g["translation"]))
    idx = torch.from_numpy(g["idx"]).to(DEV)
    new_o, new_d, R, t = m(idx, torch.from_numpy(g["o"]).to(DEV), torch.from_numpy(g["d"]).to(DEV))
    np.testing.assert_allclose(new_o.detach().cpu().numpy(), g["new_o"], atol=1e-6)
    np.testing.assert_allclose(new_d.detach().cpu().numpy(), g["new_d"], atol=1e-6)
    np.testing.assert_allclose(R.detach().cpu().numpy(), g["R"], atol=1e-6)
    ((new_o * torch.from_numpy(g["go"]).to(DEV)).sum() + (new_d * torch.from_numpy(g["gd"]).to(DEV)).sum()).backward()
    np.testing.assert_allclose(m.rotation.grad.cpu().numpy(), g["drot"], atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(m.translation.grad.cpu().numpy(), g["dtrans"], atol=1e-5, rtol=1e-6)


@pytest.mark.parametrize("scale", [0.0, 1e-7, 1e-3, 0.3, 1.5])
def test_pose_rays_vs_fp64_oracle(scale):
    """Rays, R, t and all four gradient inputs (new_o, new_d, R, t) vs the oracle in fp64 at
    rotation magnitudes from 0 (the Taylor branch) to ~2.6 rad; 1e-6 abs on the forward, 2e-6 of
    each gradient's scale (the kernel sums in fp64, the reference's fp32 index_add does not)."""
    from nerf_amd import kernels as K
    from oracle import nerf_oracle as O
    rot, trans, idx, o, d = _pose_case(12, 3000, scale, 7)
    g = torch.Generator().manual_seed(1)
    go, gd, gR, gt = (torch.randn(3000, 3, generator=g), torch.randn(3000, 3, generator=g),
                      torch.randn(3000, 3, 3, generator=g), torch.randn(3000, 3, generator=g))
    r64, t64 = rot.double().requires_grad_(), trans.double().requires_grad_()
    want = O.camera_extrinsics(r64, t64, idx, o.double(), d.double())
    (sum((w * gg.double()).sum() for w, gg in zip(want, (go, gd, gR, gt)))).backward()
    rd, td = rot.to(DEV).requires_grad_(), trans.to(DEV).requires_grad_()
    got = K.pose_rays(rd, td, idx.to(DEV), o.to(DEV), d.to(DEV))
    for w, x in zip(want, got):
        np.testing.assert_allclose(x.detach().cpu().double().numpy(), w.detach().numpy(), atol=1e-6, rtol=0)
    (sum((x * gg.to(DEV)).sum() for x, gg in zip(got, (go, gd, gR, gt)))).backward()
    for p, q in ((rd, r64), (td, t64)):
        scale_g = q.grad.abs().max().item()
        assert (p.grad.cpu().double() - q.grad).abs().max().item() <= 2e-6 * scale_g
    assert torch.equal(rd.grad[-1].cpu(), torch.zeros(3)) and torch.equal(td.grad[-1].cpu(), torch.zeros(3))


def test_pose_rays_partial_gradients_deterministic_and_bad_index():
    """Only new_d used (the others' gradients NULL); two backward passes bitwise equal; an
    out-of-range image index gives NaN rays for that ray only."""
    from nerf_amd import kernels as K
    rot, trans, idx, o, d = _pose_case(100, 4096, 0.1, 3)
    outs = []
    for _ in range(2):
        rd, td = rot.to(DEV).requires_grad_(), trans.to(DEV).requires_grad_()
        _, new_d, _, _ = K.pose_rays(rd, td, idx.to(DEV), o.to(DEV), d.to(DEV))
        new_d.square().sum().backward()
        outs.append((rd.grad.clone(), td.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], torch.zeros_like(outs[0][1]))     # new_o unused: no translation gradient
    bad = idx.clone()
    bad[5] = 100
    new_o, new_d, R, t = K.pose_rays(rot.to(DEV), trans.to(DEV), bad.to(DEV), o.to(DEV), d.to(DEV))
    assert torch.isnan(new_o[5]).all() and torch.isnan(R[5]).all()
    assert torch.isfinite(new_o[torch.arange(4096) != 5]).all()


def test_forward_origins_leaves_rotation_without_gradient():
    """forward_origins (model_camera_extrinsics.py:61-74) involves only the translation."""
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    m = CameraExtrinsics(5, 1e-3, 1e-5, 100).to(DEV)
    idx = torch.tensor([0, 3, 3, 1], device=DEV)
    o = torch.randn(4, 3, device=DEV)
    new_o, t = m.forward_origins(idx, o)
    new_o.sum().backward()
    assert m.rotation.grad is None
    assert torch.equal(m.translation.grad[3].cpu(), torch.full((3,), 2.0))


def test_pose_rays_bucketed_backward_matches_scan():
    """Above POSE_BUCKET_MIN_WORK (image, ray) pairs the backward buckets rays by image (stable
    device argsort + searchsorted) so each workgroup reads only its own rays: same gradients as the
    all-rays scan (fp64 sums in another grouping, rounded to fp32: 1e-6 of scale), deterministic,
    rays with an out-of-range index contribute to no image."""
    from nerf_amd import kernels as K
    rot, trans, idx, o, d = _pose_case(300, 20000, 0.2, 11)
    idx[7] = -1
    idx[8] = 300
    g = torch.Generator().manual_seed(2)
    go, gd = torch.randn(20000, 3, generator=g).to(DEV), torch.randn(20000, 3, generator=g).to(DEV)
    outs = []
    old = K.POSE_BUCKET_MIN_WORK
    try:
        for thr in (1 << 62, 0, 0):
            K.POSE_BUCKET_MIN_WORK = thr
            rd, td = rot.to(DEV).requires_grad_(), trans.to(DEV).requires_grad_()
            new_o, new_d, _, _ = K.pose_rays(rd, td, idx.to(DEV), o.to(DEV), d.to(DEV))
            ((torch.nan_to_num(new_o) * go).sum() + (torch.nan_to_num(new_d) * gd).sum()).backward()
            outs.append((rd.grad.clone(), td.grad.clone()))
    finally:
        K.POSE_BUCKET_MIN_WORK = old
    for a, b in zip(outs[0], outs[1]):
        assert (a - b).abs().max().item() <= 1e-6 * a.abs().max().item()
    assert torch.equal(outs[1][0], outs[2][0]) and torch.equal(outs[1][1], outs[2][1])
    assert torch.equal(outs[1][0][-1].cpu(), torch.zeros(3))      # the last image has no rays
