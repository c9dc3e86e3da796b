"""GPU checks at BASELINE.json's full per-GPU sizes (4096 rays x 64 / 64+128 / 128 samples),
where the CPU oracle cannot run the whole batch in seconds: size-independent properties of
the outputs plus oracle parity on a seeded subset of rays of the same full-size launch.

Properties: compositing weights are a sub-partition of unity (0 <= w, sum_s w <= 1 + 1e-6)
and rgb lies in [0, 1]; resampled t are sorted within each ray, start at the first coarse
t, stay inside [near - one coarse interval (the -1 offset), far], and t_end is the next
t_start (far for the last); every gradient
is finite; a fixed seed reproduces the training step bit for bit (all reductions in this
path run in a fixed order); encodings of the full batch equal the per-sample oracle on a
subset of rows (2e-6 abs), the full-size field MLP matches the oracle on a subset of rows
(1e-4, fp32 MFMA)."""
import math

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


def _lego_rays(n, seed, radius=4.03, image=800):
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(n, 2, generator=g)
    th = u[:, 0] * 2 * math.pi
    z = u[:, 1] * 0.9 + 0.1
    r = torch.sqrt(1 - z * z)
    o = torch.stack((r * torch.cos(th), r * torch.sin(th), z), dim=1) * radius
    d = torch.nn.functional.normalize(-o + (torch.rand(n, 3, generator=g) - 0.5) * 0.5, dim=1)
    pw = torch.full((n,), 1.0 / (image / 2 / math.tan(0.6911112 / 2)))
    return o, d, pw


def _mip_renderer():
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel
    torch.manual_seed(0)
    pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
    pos.pixel_width_sigma = 0.0
    model = NerfModel(4, 256, True, False, 2, pos, BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0))
    return NerfInterpolation(2.0, 8.0, model, 128, "stratified_uniform", -1.0, "middle", model, 64).to(DEV)


def test_full_size_coarse_fine_properties():
    """mip config (BASELINE configs[2]): 4096 rays, 64 coarse + 128 fine through the resample."""
    ren = _mip_renderer()
    B = 4096
    o, d, pw = _lego_rays(B, 1)
    o, d, pw = o.to(DEV), d.to(DEV), pw.to(DEV)
    t0c, t1c = ren._sample_t_stratified_uniform(B, 64, "stratified_uniform", -1.0)
    rgb_c, w, dist = ren._compute_color(ren.model_proposal, t0c, t1c, o, d, pw, B, 64)
    assert torch.all(w >= 0) and torch.all(w.sum(1) <= 1 + 1e-6)
    assert torch.all(rgb_c >= 0) and torch.all(rgb_c <= 1)
    t0, t1 = ren._sample_t_pdf_weighted(t0c, w, dist, 128)
    assert int(ren.last_resample_status.item()) == 0
    assert torch.all(t0[:, 1:] >= t0[:, :-1])
    assert torch.equal(t0[:, 0], t0c[:, 0])
    # offset -1 shifts every coarse ray back by up to one interval (model_interpolation.py:177-178)
    assert torch.all(t0 >= 2.0 - 6.0 / 64 - 1e-5) and torch.all(t1 <= 8.0)
    assert torch.equal(t1[:, :-1], t0[:, 1:]) and torch.all(t1[:, -1] == 8.0)
    # the fine t of a subset of rays equal the oracle's allocation + fill (bit-exact)
    idx = torch.arange(0, B, 97)
    r0, r1, ok = O.sample_t_pdf_weighted(t0c[idx].cpu(), w[idx].cpu(), dist[idx].cpu(), 128, 8.0, 0)
    assert ok
    np.testing.assert_array_equal(t0[idx].cpu().numpy(), r0.numpy())
    rgb_f, _, _ = ren._compute_color(ren.model_radiance, t0, t1, o, d, pw, B, 128)
    assert torch.all(rgb_f >= 0) and torch.all(rgb_f <= 1)


def test_full_size_encoding_subset_parity():
    """Full-size ray-mode encodings (4096 x 128 samples, BARF L10 + identity and masked IPE at
    800^2) against the oracle on every 61st sample row."""
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures
    B, S = 4096, 128
    o, d, pw = _lego_rays(B, 2)
    g = torch.Generator().manual_seed(3)
    t = torch.sort(2 + torch.rand(B, S, generator=g) * 6, dim=1).values
    t0, t1 = O.intervals(t, 8.0)
    rows = torch.arange(0, B * S, 61)
    pos, dirs = O.compute_positions(o, d, t0, t1, "middle")
    pos, dirs = pos.reshape(-1, 3)[rows], dirs.reshape(-1, 3)[rows]
    barf = BarfPositionalEncoding(10, 7.3, 0, 1, True, 1.0).to(DEV)
    out = barf.encode_rays(o.to(DEV), d.to(DEV), t0.to(DEV), t1.to(DEV), None, S, 1, 0)
    np.testing.assert_allclose(out[rows.to(DEV), :63].cpu().numpy(), O.barf_pe(pos, 10, 7.3, True, 1.0).numpy(),
                               atol=2e-6, rtol=0)
    ipe = IntegratedBarfFourierFeatures(10, 7.3, 0, 1, True, 1.0, False).to(DEV)
    ipe.pixel_width_sigma = 0.0
    out = ipe.encode_rays(o.to(DEV), d.to(DEV), t0.to(DEV), t1.to(DEV), pw.to(DEV), S, 1, 0)
    n = rows.numel()
    ref = O.integrated_pe(pos, dirs, torch.full((n, 1), float(pw[0])), t0.reshape(-1, 1)[rows],
                          t1.reshape(-1, 1)[rows], 10, 1.0, True, False, 0.0, mask=O.barf_mask(7.3, 10))
    np.testing.assert_allclose(out[rows.to(DEV), :63].cpu().numpy(), ref.numpy(), atol=2e-6, rtol=0)


def test_full_size_mlp_subset_parity():
    """The bench's NerfModel (naive-to-vanilla) on all 262 144 samples of a step; rows of a
    seeded subset against the oracle's MLP (fp32 MFMA, 1e-4)."""
    from nerf_amd import FourierFeatures, NerfModel
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        torch.manual_seed(0)
        m = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0))
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        m = m.to(DEV)
        N = 4096 * 64
        g = torch.Generator().manual_seed(4)
        pos = torch.rand(N, 3, generator=g) * 0.6 - 0.3
        d = torch.nn.functional.normalize(torch.randn(N, 3, generator=g), dim=1)
        with torch.no_grad():
            dens, rgb = m(pos.to(DEV), d.to(DEV), None, None, None)
        rows = torch.arange(5, N, 1013)
        rd, rr = O.nerf_model_forward(sd, O.fourier_features(pos[rows], 10, 2 * math.pi),
                                      O.fourier_features(d[rows], 4, 1.0), 2, 4, True, True)
        np.testing.assert_allclose(dens[rows.to(DEV)].cpu().numpy(), rd.numpy(), atol=1e-4, rtol=1e-4)
        np.testing.assert_allclose(rgb[rows.to(DEV)].cpu().numpy(), rr.numpy(), atol=1e-4, rtol=1e-4)
    finally:
        torch.set_float32_matmul_precision(old)


def test_full_size_training_step_deterministic_and_finite():
    """Two full-size bench steps (4096 x 64, split precision) from the same seed: bit-identical
    loss and gradients (fixed-order reductions everywhere), all finite."""
    from nerf_amd import FourierFeatures, NerfInterpolation, NerfModel

    def run():
        torch.manual_seed(0)
        model = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0))
        ren = NerfInterpolation(0.1, 1 / 3, model, 64, "stratified_uniform", density_factor=(3.0, 7.0)).to(DEV)
        B = 4096
        o = (torch.nn.functional.normalize(torch.randn(B, 3), dim=1) * 0.168).to(DEV)
        d = torch.nn.functional.normalize(-o.cpu() + torch.randn(B, 3) * 0.1, dim=1).to(DEV)
        pw = torch.full((B,), 1 / 555.56, device=DEV)
        target = torch.rand(B, 3).to(DEV)
        torch.manual_seed(7)
        loss, _ = ren.training_loss(o, d, pw, target)
        loss.backward()
        return float(loss.detach()), [p.grad.clone() for p in ren.parameters()]

    l1, g1 = run()
    l2, g2 = run()
    assert math.isfinite(l1) and l1 == l2
    for a, b in zip(g1, g2):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


def _mip_oracle_pass(sd, o, d, pw, t0, t1, dt):
    """The bench's mip field on explicit t (masked IPE at alpha = L, masked PE of the directions,
    NerfModel, compositing with 3 * MAGIC) in dtype dt: (rgb, weights)."""
    B, S = t0.shape
    o, d, t0, t1 = o.to(dt), d.to(dt), t0.to(dt), t1.to(dt)
    pos, dirs = O.compute_positions(o, d, t0, t1, "middle")
    n = B * S
    pos_pe = O.integrated_pe(pos.reshape(-1, 3), dirs.reshape(-1, 3), torch.full((n, 1), float(pw[0]), dtype=dt),
                             t0.reshape(-1, 1), t1.reshape(-1, 1), 10, 1.0, True, True, 0.0,
                             mask=O.barf_mask(10.0, 10).to(dt))
    dir_pe = O.barf_pe(dirs.reshape(-1, 3), 4, 4.0, True, 1.0).to(dt)
    dens, col = O.nerf_model_forward(sd, pos_pe, dir_pe, 2, 4, True, False)
    b = (-dens.view(B, S) * (t1 - t0)) * 3.0 * (1 / 3)
    T = torch.cat((torch.ones(B, 1, dtype=dt), torch.exp(torch.cumsum(b[:, :-1], dim=1))), dim=1)
    w = T * (1 - torch.exp(b))
    return torch.sum(w.unsqueeze(-1) * col.view(B, S, 3), dim=1), w


def test_full_size_mip_step_subset_parity_high():
    """C3 as bench.py times it: 4096 rays x (64 coarse + 128 fine) on the fused
    split-precision path ("high": the fused forward generating both encodings and compositing in its
    launches, the fused input-gradient chain, the weight gradients), against the CPU oracle on a
    seeded subset of 48 rays: coarse rgb / weights on the coarse t, fine rgb / weights on the GPU's
    resampled fine t (2e-4 absolute, the split-precision renderer bar of test_gpu_mip_pose_feed.py),
    and every parameter's gradient of one step's loss restricted to those rays (the other rays get
    zero grad_rgb but run through the same full-size launches) against the oracle in float64, under
    the per-tensor conditioning bound of test_gpu_parity.py's split-precision NerfModel test (2 x the
    spread of the exact gradient under relative 2^-15 weight perturbations + 2 x 2^9 x the fp32
    oracle's own error; 2^-15 = the per-product bound of three bf16 products)."""
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        torch.manual_seed(0)
        pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
        pos.pixel_width_sigma = 0.0
        model = NerfModel(4, 256, True, False, 2, pos, BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0),
                          5e-4, 1e-4, 200000)
        sd = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith("alpha")}
        ren = NerfInterpolation(2.0, 8.0, model, 128, "stratified_uniform", -1.0, "middle", model, 64).to(DEV)
        B = 4096
        o, d, pw = _lego_rays(B, 11)
        target = torch.rand(B, 3, generator=torch.Generator().manual_seed(12))
        idx = torch.arange(7, B, 85)                          # 48 rays spread over the batch
        mask = torch.zeros(B, 1)
        mask[idx] = 1.0
        og, dg, pwg = o.to(DEV), d.to(DEV), pw.to(DEV)
        torch.manual_seed(13)
        t0c, t1c = ren._sample_t_stratified_uniform(B, 64, "stratified_uniform", -1.0)
        rgb_c, w_c, dist = ren._compute_color(ren.model_proposal, t0c, t1c, og, dg, pwg, B, 64)
        t0, t1 = ren._sample_t_pdf_weighted(t0c, w_c, dist, 128)
        rgb_f, w_f, _ = ren._compute_color(ren.model_radiance, t0, t1, og, dg, pwg, B, 128)
        loss = (((rgb_f - target.to(DEV)) ** 2 + (rgb_c - target.to(DEV)) ** 2) * mask.to(DEV)).sum()
        model.zero_grad(set_to_none=True)
        loss.backward()
        torch.cuda.synchronize()
        # forward parity on the subset
        r_c, r_wc = _mip_oracle_pass(sd, o[idx], d[idx], pw, t0c[idx].cpu(), t1c[idx].cpu(), torch.float32)
        np.testing.assert_allclose(rgb_c[idx.to(DEV)].detach().cpu().numpy(), r_c.numpy(), atol=2e-4, rtol=0)
        np.testing.assert_allclose(w_c[idx.to(DEV)].detach().cpu().numpy(), r_wc.numpy(), atol=2e-4, rtol=0)
        r_f, r_wf = _mip_oracle_pass(sd, o[idx], d[idx], pw, t0[idx].cpu(), t1[idx].cpu(), torch.float32)
        np.testing.assert_allclose(rgb_f[idx.to(DEV)].detach().cpu().numpy(), r_f.numpy(), atol=2e-4, rtol=0)
        np.testing.assert_allclose(w_f[idx.to(DEV)].detach().cpu().numpy(), r_wf.numpy(), atol=2e-4, rtol=0)
        # one step's gradients: the conditioning bound of test_gpu_parity.py's split-precision
        # NerfModel test (exact fp64 gradient; its spread under relative 2^-15 weight perturbations,
        # three draws; the fp32 oracle's own error)
        def grads(dt, perturb=None):
            sdx = {k: v.detach().to(dt).clone() for k, v in sd.items()}
            if perturb is not None:
                gen = torch.Generator().manual_seed(perturb)
                sdx = {k: v * (1 + (torch.rand(v.shape, generator=gen, dtype=dt) * 2 - 1) * 2.0 ** -15)
                       for k, v in sdx.items()}
            sdx = {k: v.requires_grad_(True) for k, v in sdx.items()}
            c, _ = _mip_oracle_pass(sdx, o[idx], d[idx], pw, t0c[idx].cpu(), t1c[idx].cpu(), dt)
            f, _ = _mip_oracle_pass(sdx, o[idx], d[idx], pw, t0[idx].cpu(), t1[idx].cpu(), dt)
            tg = target[idx].to(dt)
            (((f - tg) ** 2).sum() + ((c - tg) ** 2).sum()).backward()
            return {k: v.grad.double() for k, v in sdx.items() if v.grad is not None}
        exact, fp32 = grads(torch.float64), grads(torch.float32)
        spread = {k: torch.zeros((), dtype=torch.float64) for k in exact}
        for seed in range(3):
            pert = grads(torch.float64, seed)
            for k in exact:
                spread[k] = torch.maximum(spread[k], (pert[k] - exact[k]).abs().max())
        for k, p in model.named_parameters():
            e = exact[k]                                    # every parameter has an oracle gradient
            scale = e.abs().max().item()
            err = (p.grad.detach().cpu().double() - e).abs().max().item() / scale
            fp32_err = (fp32[k] - e).abs().max().item() / scale
            bound = 2 * spread[k].item() / scale + 2 * 2 ** 9 * max(fp32_err, 2 ** -22)
            print(f"{k}: err {err:.2e} bound {bound:.2e} (spread {spread[k].item() / scale:.2e}, fp32 {fp32_err:.2e})")
            assert err <= bound, (k, err, bound)
    finally:
        torch.set_float32_matmul_precision(old)
