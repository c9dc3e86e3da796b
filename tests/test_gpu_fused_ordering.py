"""Rows generated inside the fused forward and read back within the same launch.

The fused forward generates both encodings at every 128-sample tile start.  The position rows are
per sample and stored by the wave that owns the samples, which reads them back itself (the skip
layer).  The direction rows are per ray: the HBM row of a ray is stored once, by the wave holding the
ray's first sample.  When the samples per ray S do not divide the tile, that wave belongs to another
workgroup, so the colour layer must not read the row back from HBM.  It takes its direction block
from registers captured at the tile start, from the wave's own LDS rows (csrc/mlp_fused.hip,
seg_gen on a later layer).  The library refuses the HBM read-back (fused_launch's ordering rule).

Every deferred encoding buffer is NaN-filled at allocation here (NERF_POISON_DEFERRED=1, set by
tests/conftest.py), so a read of a row before its store fails every time.

Parity: the renderer's _compute_color at S in {96, 192, 200, 320} against the CPU oracle
(oracle/nerf_oracle.py, reference barf/model_interpolation.py:288-414 with masked IPE and masked PE,
positional_encodings.py:124-148, 266-282), in split precision ("high": three bf16 products per fp32
product).  Bars: rgb and weights 2e-4 absolute, as the reference-fixture renderer tests in
test_gpu_mip_pose_feed.py use for "high"."""
import math
import os

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
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    yield
    torch.set_float32_matmul_precision(prev)


def _setup(S, B, seed=5):
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel
    torch.manual_seed(0)
    pos = IntegratedBarfFourierFeatures(10, 7.3, 0, 1, True, 1.0, True)
    pos.pixel_width_sigma = 0.0
    model = NerfModel(4, 256, True, False, 2, pos, BarfPositionalEncoding(4, 2.6, 0, 1, True, 1.0))
    sd = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith("alpha")}
    ren = NerfInterpolation(2.0, 8.0, model, S, "stratified_uniform", -1.0, "middle").to(DEV)
    g = torch.Generator().manual_seed(seed)
    o = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=1) * 4.03
    d = torch.nn.functional.normalize(-o + 0.5 * torch.randn(B, 3, generator=g), dim=1)
    pw = torch.full((B,), 1 / 1111.1)
    t = torch.sort(2 + torch.rand(B, S, generator=g) * 6, dim=1).values
    t0, t1 = O.intervals(t, 8.0)
    return ren, sd, o, d, pw, t0.contiguous(), t1.contiguous()


def _oracle(sd, o, d, pw, t0, t1):
    B, S = t0.shape
    pos, dirs = O.compute_positions(o, d, t0, t1, "middle")
    n = B * S
    pos_pe = O.integrated_pe(pos.reshape(-1, 3), dirs.reshape(-1, 3), torch.full((n, 1), float(pw[0])),
                             t0.reshape(-1, 1), t1.reshape(-1, 1), 10, 1.0, True, True, 0.0,
                             mask=O.barf_mask(7.3, 10))
    dir_pe = O.barf_pe(dirs.reshape(-1, 3), 4, 2.6, True, 1.0)
    dens, col = O.nerf_model_forward(sd, pos_pe, dir_pe, 2, 4, True, False)
    return O.render_rays(dens.view(B, S), col.view(B, S, 3), t1 - t0, 3.0, 1 / 3)


def _spy(monkeypatch):
    """Record the fused forward launches and the generated encodings each one received."""
    from nerf_amd import mlp_fused
    calls = []
    real = mlp_fused.FusedForward.run

    def run(self, M, pos, dirs, dir_rd, acts, masks, col_outs, gens=(None, None), comp=None, **kw):
        calls.append((M, dir_rd, gens[0] is not None, gens[1] is not None))
        return real(self, M, pos, dirs, dir_rd, acts, masks, col_outs, gens, comp, **kw)
    monkeypatch.setattr(mlp_fused.FusedForward, "run", run)
    return calls


@pytest.mark.parametrize("S", [96, 192, 200, 320])
def test_fused_forward_per_ray_directions_vs_oracle(S, monkeypatch):
    assert os.environ.get("NERF_POISON_DEFERRED") == "1"
    B = 333                                   # several workgroups; the last tile partial
    ren, sd, o, d, pw, t0, t1 = _setup(S, B)
    calls = _spy(monkeypatch)
    rgb, w, _ = ren._compute_color(ren.model_radiance, t0.to(DEV), t1.to(DEV), o.to(DEV), d.to(DEV), pw.to(DEV),
                                   B, S)
    torch.cuda.synchronize()
    # the fused forward ran, generating both encodings in-kernel with per-ray directions (divisor S)
    assert calls and calls[-1] == (B * S, S, True, True)
    ref_rgb, ref_w = _oracle(sd, o, d, pw, t0, t1)
    assert torch.isfinite(rgb).all() and torch.isfinite(w).all()
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), ref_rgb.numpy(), atol=2e-4, rtol=0)
    np.testing.assert_allclose(w.detach().cpu().numpy(), ref_w.numpy(), atol=2e-4, rtol=0)
    # the backward reads the stored rows (every ray's direction row, every sample's position row)
    rgb.square().sum().backward()
    for p in ren.parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all()


def test_fused_forward_refuses_per_ray_rows_read_back(monkeypatch):
    """Without the register capture a later layer would read the per-ray rows back from HBM, which
    another workgroup may not have stored yet: the library refuses that launch."""
    from nerf_amd import mlp_fused
    monkeypatch.setattr(mlp_fused, "CAPTURE_PER_RAY", False)
    B, S = 64, 96
    ren, sd, o, d, pw, t0, t1 = _setup(S, B)
    with pytest.raises(RuntimeError):
        ren._compute_color(ren.model_radiance, t0.to(DEV), t1.to(DEV), o.to(DEV), d.to(DEV), pw.to(DEV), B, S)
    torch.cuda.synchronize()
