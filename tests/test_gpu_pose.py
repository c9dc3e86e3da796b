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
