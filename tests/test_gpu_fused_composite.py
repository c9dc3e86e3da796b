"""Alpha compositing fused into the field MLP's launches (nerf_mlp_fused_render, VERDICT r02
"compositing fused into the head epilogue / the chain's prologue") against the stand-alone
compositing kernels (nerf_composite_fwd/bwd, pinned to the reference's composite golden vectors by
test_gpu_parity.py) on the same raw heads.

Forward: the tile-end compositing evaluates the same composite_common.h instructions, so rgb and
weights are BITWISE those of render_raw + composite_raw.  Backward: the chain forms the head /
density gradient rows from the forward's per-sample coefficients (linear in grad_rgb: no scan), a
different fp32 rounding order than nerf_composite_bwd — bar 2e-5 relative to each gradient's scale
(the compositing tolerance of test_gpu_parity.py).  Covers the C3 mip workload's S = 64 / 128,
S = 16 / 32 (8 / 4 rays per tile), S = 256 (one ray over two tiles run back to back: 3d-ingp's
fine pass), ragged ray counts (the last tile partial), the density as a
column output (NerfModel) and as head row 3 (delayed density), pose gradients to the rays, and the
torch fallback taken when the chain cannot form the rows."""
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


def _model(delayed_density=False):
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfModel
    torch.manual_seed(0)
    pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
    pos.pixel_width_sigma = 0.0
    dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
    return NerfModel(4, 256, True, delayed_density, 2, pos, dirs).to(DEV)


def _rays(n_rays, S, seed=3):
    g = torch.Generator(device=DEV).manual_seed(seed)
    o = torch.randn(n_rays, 3, device=DEV, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 2.5], device=DEV)
    d = torch.nn.functional.normalize(torch.randn(n_rays, 3, device=DEV, generator=g) * 0.3
                                      - torch.tensor([0.0, 0.0, 1.0], device=DEV), dim=1)
    t = torch.sort(torch.rand(n_rays, S + 1, device=DEV, generator=g) * 4 + 0.5, dim=1).values
    t0, t1 = t[:, :-1].contiguous(), t[:, 1:].contiguous()
    pw = torch.rand(n_rays, device=DEV, generator=g) * 2e-3 + 5e-4
    return o, d, t0, t1, pw


def _step(model, o, d, t0, t1, pw, S, fused, target, scales=(3.0, 7.0), grad=True):
    """rgb, weights and (grads of o, d, params) of one compositing pass, fused or not."""
    from nerf_amd.model_interpolation import composite_raw
    oo = o.clone().requires_grad_(grad)
    dd = d.clone().requires_grad_(grad)
    dist = (t1 - t0).contiguous()
    n_rays = o.shape[0]
    if fused:
        assert model.fused_composite_ok(n_rays * S, S)
        rgb, w = model.render_composite(oo, dd, pw, t0, t1, S, 1, 1, dist, *scales)
    else:
        heads = model.render_raw(oo, dd, pw, t0, t1, S, 1, 1)
        rgb, w = composite_raw(heads, dist, n_rays, S, *scales)
    if not grad:
        return rgb, w, None
    model.zero_grad(set_to_none=True)
    loss = ((rgb - target) ** 2).mean()
    loss.backward()
    torch.cuda.synchronize()
    return rgb.detach(), w.detach(), (oo.grad.clone(), dd.grad.clone(),
                                      [p.grad.clone() if p.grad is not None else None for p in model.parameters()])


def _close(a, b, rel=2e-5):
    scale = b.abs().max().item()
    err = (a - b).abs().max().item()
    assert err <= rel * max(scale, 1e-30), f"max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("n_rays,S,delayed", [(4096, 64, False), (4096, 128, False), (37, 64, False),
                                              (301, 32, False), (75, 16, False), (203, 128, True),
                                              (1024, 256, False), (37, 256, False), (45, 256, True)])
def test_fused_composite_forward_bitwise_and_gradients(n_rays, S, delayed):
    model = _model(delayed)
    o, d, t0, t1, pw = _rays(n_rays, S)
    target = torch.rand(n_rays, 3, device=DEV, generator=torch.Generator(device=DEV).manual_seed(9))
    rgb0, w0, g0 = _step(model, o, d, t0, t1, pw, S, False, target)
    rgb1, w1, g1 = _step(model, o, d, t0, t1, pw, S, True, target)
    assert torch.equal(rgb0, rgb1)
    assert torch.equal(w0, w1)
    _close(g1[0], g0[0])
    _close(g1[1], g0[1])
    for a, b in zip(g1[2], g0[2]):
        assert (a is None) == (b is None)
        if a is not None:
            _close(a, b)


def test_fused_composite_inference_matches():
    """Without autograd (render mode): no coefficient rows, rgb and weights bitwise as above."""
    model = _model()
    o, d, t0, t1, pw = _rays(640, 64, seed=11)
    with torch.no_grad():
        rgb0, w0, _ = _step(model, o, d, t0, t1, pw, 64, False, None, grad=False)
        rgb1, w1, _ = _step(model, o, d, t0, t1, pw, 64, True, None, grad=False)
    assert torch.equal(rgb0, rgb1) and torch.equal(w0, w1)


def test_fused_composite_torch_fallback(monkeypatch):
    """When the fused chain cannot take the compositing's gradient (here: no chain layout), the
    rows are formed from the coefficients in torch and the layer-by-layer backward runs."""
    from nerf_amd import mlp_fused
    model = _model()
    n_rays, S = 300, 64
    o, d, t0, t1, pw = _rays(n_rays, S, seed=4)
    target = torch.rand(n_rays, 3, device=DEV)
    _, _, g0 = _step(model, o, d, t0, t1, pw, S, False, target)
    monkeypatch.setattr(mlp_fused.FusedInputGrad, "layout", staticmethod(lambda plan, a, b: None))
    runs = mlp_fused.FusedInputGrad.runs
    _, _, g1 = _step(model, o, d, t0, t1, pw, S, True, target)
    assert mlp_fused.FusedInputGrad.runs == runs            # the chain did not run
    _close(g1[0], g0[0])
    for a, b in zip(g1[2], g0[2]):
        _close(a, b)


def test_fused_composite_in_the_renderer():
    """NerfInterpolation (mip: shared field, 64 coarse + 128 fine, pdf resample) with and without
    the fused compositing: both passes' rgb bitwise equal (so the resampled t too), gradients close."""
    from nerf_amd import NerfInterpolation, mlp
    o, d, _, _, pw = _rays(1024, 8, seed=21)
    target = torch.rand(1024, 3, device=DEV)
    out = []
    for fuse in (False, True):
        model = _model()
        ren = NerfInterpolation(2.0, 8.0, model, 128, "stratified_uniform", -1.0, "middle", model, 64).to(DEV)
        saved = mlp.FUSE_COMPOSITE
        mlp.FUSE_COMPOSITE = fuse
        try:
            torch.manual_seed(5)
            fine, coarse = ren(o, d, pw)
            loss = ((fine - target) ** 2).mean() + ((coarse - target) ** 2).mean()
            loss.backward()
        finally:
            mlp.FUSE_COMPOSITE = saved
        torch.cuda.synchronize()
        out.append((fine.detach(), coarse.detach(), [p.grad.clone() for p in model.parameters()]))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    for a, b in zip(out[1][2], out[0][2]):
        _close(a, b)


@pytest.mark.parametrize("S", [96, 200])
def test_renderer_falls_back_for_rays_that_do_not_fill_a_tile(S):
    """Samples per ray that do not divide the 128-sample tile (or exceed it) take render_raw + the
    stand-alone compositing kernels: the renderer's output is the same with the fused switch on or off."""
    from nerf_amd import NerfInterpolation, mlp
    model = _model()
    assert not model.fused_composite_ok(64 * S, S)
    o, d, _, _, pw = _rays(64, 8, seed=31)
    ren = NerfInterpolation(2.0, 8.0, model, S, "stratified_uniform", -1.0, "middle").to(DEV)
    outs = []
    for fuse in (True, False):
        saved = mlp.FUSE_COMPOSITE
        mlp.FUSE_COMPOSITE = fuse
        try:
            torch.manual_seed(3)
            fine, _ = ren(o, d, pw)
            model.zero_grad(set_to_none=True)
            fine.square().sum().backward()
        finally:
            mlp.FUSE_COMPOSITE = saved
        torch.cuda.synchronize()
        outs.append((fine.detach(), [p.grad.clone() for p in model.parameters()]))
    assert torch.equal(outs[0][0], outs[1][0])
    assert all(torch.equal(a, b) for a, b in zip(outs[0][1], outs[1][1]))
