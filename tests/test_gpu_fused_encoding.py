"""Encodings generated inside the fused field-MLP kernel (mlp_fused.hip gen_block, VERDICT r02
"PE fused into the MLP prologue") against the stand-alone encoding kernel (nerf_encode_fwd, pinned
to the reference's pe.npz / mipnerf.npz golden vectors by test_gpu_parity.py /
test_gpu_mip_pose_feed.py).

The kernel evaluates the same encode_common.h functions with fp contraction off, so the bar is
BITWISE: the rows it stores for the weight gradients equal nerf_encode_fwd's, and every head,
layer output and gradient of a render_raw step is bitwise that of the unfused step.  Encoders: the
C3 mip workload's masked integrated encoding (pixel width as 800^2 / per-sample, sigma 0 and the
> 0.25 branch, distributed and per-axis variance), BARF's masked Fourier features at a fractional
alpha, plain Fourier features (n2v) and 3d-ingp's scale-1 features as the direction encoder;
BASELINE's 4096 x 64 batch and ragged ray x sample counts (M not a multiple of the 128-sample
workgroup tile), query at the interval start and midpoint."""
import math

import pytest
import torch

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


def _model(kind):
    from nerf_amd import (BarfPositionalEncoding, FourierFeatures, IntegratedBarfFourierFeatures,
                          IntegratedFourierFeatures, NerfModel)
    from nerf_amd.model_ingp import FourierFeatures as IngpFourier
    torch.manual_seed(0)
    if kind == "mip":
        pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
        pos.pixel_width_sigma = 0.0
        dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
    elif kind == "ipe_axis":
        pos = IntegratedFourierFeatures(10, 1.0, True, False)
        pos.pixel_width_sigma = 0.5                      # the > 0.25 branch (positional_encodings.py:204)
        dirs = FourierFeatures(4, 1.0)
    elif kind == "barf":
        pos = BarfPositionalEncoding(10, 3.7, 0, 1, True, 1.0)       # fractional alpha: a ramped level
        dirs = BarfPositionalEncoding(4, 1.5, 0, 1, True, 1.0)
    elif kind == "n2v":
        pos = FourierFeatures(10, 2 * math.pi)
        dirs = FourierFeatures(4, 1.0)
    else:                                               # 3d-ingp's direction features
        pos = FourierFeatures(10, 2 * math.pi)
        dirs = IngpFourier(4)
    return NerfModel(4, 256, True, kind == "n2v", 2, pos, dirs).to(DEV)


def _rays(n_rays, S, seed=3):
    g = torch.Generator(device=DEV).manual_seed(seed)
    o = torch.randn(n_rays, 3, device=DEV, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 2.5], device=DEV)
    d = torch.nn.functional.normalize(torch.randn(n_rays, 3, device=DEV, generator=g) * 0.3
                                      - torch.tensor([0.0, 0.0, 1.0], device=DEV), dim=1)
    t = torch.sort(torch.rand(n_rays, S + 1, device=DEV, generator=g) * 4 + 0.5, dim=1).values
    t0, t1 = t[:, :-1].contiguous(), t[:, 1:].contiguous()
    pw = torch.rand(n_rays, device=DEV, generator=g) * 2e-3 + 5e-4
    return o, d, t0, t1, pw


def _encode(model, o, d, t0, t1, pw, S, query, pw_mode, defer):
    pe = model.position_encoder.encode_rays(o, d, t0, t1, pw, S, query, pw_mode, defer=defer)
    de = model.direction_encoder.encode_padded(d, defer=defer)
    return pe, de


@pytest.mark.parametrize("kind,n_rays,S,query,pw_mode", [
    ("mip", 4096, 64, 1, 0), ("mip", 37, 65, 1, 2), ("ipe_axis", 300, 17, 1, 1), ("barf", 4096, 64, 0, 0),
    ("barf", 129, 3, 1, 0), ("n2v", 1000, 7, 0, 0), ("ingp_dirs", 64, 64, 0, 0)])
def test_generated_encodings_bitwise(kind, n_rays, S, query, pw_mode):
    from nerf_amd import kernels as K, mlp_fused
    model = _model(kind)
    o, d, t0, t1, pw = _rays(n_rays, S)
    if pw_mode == 2:
        pw = pw[:, None].expand(n_rays, S).contiguous()
    M = n_rays * S
    assert mlp_fused.eligible(model._get_plan(), M)
    with torch.no_grad():
        pe_ref, de_ref = _encode(model, o, d, t0, t1, pw, S, query, pw_mode, False)
        z_ref, h_ref, c_ref = model._run_mlp(pe_ref, de_ref, S)
        pe, de = _encode(model, o, d, t0, t1, pw, S, query, pw_mode, True)
        assert K.deferred(pe) is not None and K.deferred(de) is not None
        z, h, c = model._run_mlp(pe, de, S)
        torch.cuda.synchronize()
    assert K.deferred(pe) is None and K.deferred(de) is None
    assert torch.equal(pe, pe_ref)                   # the stored rows, pad columns (zero) included
    assert torch.equal(de, de_ref)
    assert torch.equal(h[:, :3], h_ref[:, :3])
    if c_ref is not None:
        assert torch.equal(c, c_ref)


@pytest.mark.parametrize("kind", ["mip", "barf"])
def test_generated_encodings_training_step_bitwise(kind):
    """A render_raw forward + backward (pose gradients to the rays, weight gradients through the
    stored encoding rows) with and without in-kernel encodings: every gradient bitwise equal."""
    from nerf_amd import model_interpolation_architecture as A
    n_rays, S = 512, 64
    o, d, t0, t1, pw = _rays(n_rays, S, seed=5)
    results = []
    for fuse in (False, True):
        model = _model(kind)
        oo, dd = o.clone().requires_grad_(True), d.clone().requires_grad_(True)
        saved = A.FUSE_ENCODINGS
        A.FUSE_ENCODINGS = fuse
        try:
            heads = model.render_raw(oo, dd, pw, t0, t1, S, 1, 0)
        finally:
            A.FUSE_ENCODINGS = saved
        rgb = heads.color_base[:, :3]
        sigma = heads.dens_base[:, heads.dens_col]
        loss = rgb.square().sum() + (sigma * torch.linspace(-1, 1, sigma.shape[0], device=DEV)).sum()
        loss.backward()
        torch.cuda.synchronize()
        results.append((oo.grad.clone(), dd.grad.clone(), [p.grad.clone() for p in model.parameters()]))
    (go0, gd0, gp0), (go1, gd1, gp1) = results
    assert torch.equal(go0, go1) and torch.equal(gd0, gd1)
    assert all(torch.equal(a, b) for a, b in zip(gp0, gp1))


def test_deferred_encodings_filled_on_the_layerwise_path():
    """Exact fp32 ("highest") runs the layer-by-layer GEMMs: MLPFunction fills deferred rows itself."""
    from nerf_amd import kernels as K
    model = _model("barf")
    o, d, t0, t1, pw = _rays(200, 16)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        with torch.no_grad():
            pe_ref, de_ref = _encode(model, o, d, t0, t1, pw, 16, 1, 0, False)
            _, h_ref, c_ref = model._run_mlp(pe_ref, de_ref, 16)
            pe, de = _encode(model, o, d, t0, t1, pw, 16, 1, 0, True)
            _, h, c = model._run_mlp(pe, de, 16)
    finally:
        torch.set_float32_matmul_precision(prev)
    assert K.deferred(pe) is None and torch.equal(pe, pe_ref) and torch.equal(de, de_ref)
    # (the layer-by-layer head leaves its pad column unwritten: rgb columns and the density column)
    assert torch.equal(h[:, :3], h_ref[:, :3]) and torch.equal(c, c_ref)
