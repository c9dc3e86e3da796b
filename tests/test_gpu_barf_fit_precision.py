"""BARF pose refinement in split precision ("high", 3 x bf16 MFMA products: the bench's C4 setting)
against exact fp32 MFMA ("highest") on one fixed-seed fit (tests/_barf_fit.py; barf/model_barf.py:29-92,
pose error as model_camera_calibration.py:340-346).

Why: the split-precision pose gradient of a single batch is 5.5e-2 (translation) / 2.8e-3
(rotation) of its magnitude away from fp64 (test_gpu_mip_pose_feed.py; the reference's fp32 is at
1.7e-4 / 5e-6 — a sum of thousands of cancelling per-sample terms, condition number ~3e3).  What
BARF needs is that the FIT is unaffected.  Measured on the GPU (2000 steps, seed 0; tools/
barf_precision_fit.py prints the same): PSNR 30.89 dB "high" vs 30.45 dB "highest", pose error
0.0832 vs 0.0848 from 0.1120 at the start.

Stated bounds: both fits refine the poses (final pose error <= 0.85 x initial); |PSNR("high") -
PSNR("highest")| <= 1.0 dB; pose error("high") <= 1.10 x pose error("highest")."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_barf_fit_split_precision_matches_exact_fp32():
    import nerf_amd
    from _barf_fit import run_fit
    nerf_amd._lib.load()
    high = run_fit("high", 2000)
    exact = run_fit("highest", 2000)
    for r in (high, exact):
        assert r["pose_error"] <= 0.85 * r["pose_error_initial"], r
        assert r["loss_curve"][-1] < 0.05 * r["loss_curve"][0], r
    assert abs(high["psnr"] - exact["psnr"]) <= 1.0, (high["psnr"], exact["psnr"])
    assert high["pose_error"] <= 1.10 * exact["pose_error"], (high["pose_error"], exact["pose_error"])
