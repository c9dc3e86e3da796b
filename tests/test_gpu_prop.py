"""GPU checks of the nerfacc-equivalent proposal sampler (nerf_prop_cdf / _sample / _loss,
nerf_amd.prop_sampler) against oracle/nerfacc_oracle.py.  nerfacc itself is absent (version
unpinned, not vendored): PARITY UNPINNED — these tests pin the kernels to the restatement only.

Tolerances: cdf 1e-6 abs (fp64 prefix sums on both sides); inverse-cdf edges 2e-6 abs in s
(fp32 interpolation, same formula); t edges 1e-5 relative (lindisp reciprocal); interlevel loss
1e-5 relative per ray; its gradient 1e-5 of its scale (fp64 gathers vs autograd); end-to-end
estimator + rendering 1e-5 (edges), 1e-4 relative (loss, sigma gradients)."""
import numpy as np
import pytest
import torch

from oracle import nerfacc_oracle as NO

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _weights(R, K, seed, zeros=True):
    g = torch.Generator().manual_seed(seed)
    w = torch.rand(R, K, generator=g) ** 3
    if zeros:
        w[:, K // 3:K // 2] = 0.0          # a flat stretch of the cdf
        w[0] = 0.0                          # a ray with no mass at all
    return w / (w.sum(dim=1, keepdim=True) * 1.3 + 1e-6)


@pytest.mark.parametrize("K", [1, 64, 300])
def test_prop_cdf_vs_oracle(K):
    from nerf_amd import kernels as Kn
    w = _weights(37, K, K, zeros=K > 2)
    cdf = Kn.prop_cdf(w.to(DEV)).cpu()
    torch.testing.assert_close(cdf, NO.prop_cdf(w), atol=1e-6, rtol=0)


@pytest.mark.parametrize("S", [1, 64, 192])
def test_prop_cdf_of_composite_weights_is_one_minus_trans(S):
    """nerfacc forms the proposal cdf as 1 - [trans, 0] from the renderer's exclusive transmittance
    (garf/model_garf.py:210-230,257 call sites); here it is built from the compositing kernel's
    weights.  The two agree within 1e-6: trans from the same sigma, delta in fp64 (the compositing
    kernel's own fp64 scan), weights from nerf_composite_fwd, cdf from nerf_prop_cdf."""
    from nerf_amd import kernels as Kn
    R = 53
    g = torch.Generator().manual_seed(S)
    sigma = torch.nn.functional.softplus(torch.randn(R, S, generator=g) * 2)
    sigma[3] = 0.0                                   # an empty ray: trans 1 everywhere
    sigma[4, S // 2:] = 1e4                          # an opaque one: trans 0 past the wall
    t = torch.sort(torch.rand(R, S + 1, generator=g), dim=1).values * 5 + 2
    delta = (t[:, 1:] - t[:, :-1]).contiguous()
    col = torch.rand(R * S, 4, generator=g)
    _, w = Kn.composite_fwd(sigma.reshape(-1).to(DEV), 1, col.to(DEV), 4, delta.to(DEV), R, S, 1.0, 1.0, False)
    cdf = Kn.prop_cdf(w.view(R, S)).cpu().double()
    trans = torch.exp(-torch.cumsum(torch.cat([torch.zeros(R, 1, dtype=torch.float64),
                                               (sigma.double() * delta.double())[:, :-1]], 1), dim=1))
    want = 1.0 - torch.cat([trans, torch.zeros(R, 1, dtype=torch.float64)], dim=1)
    assert (cdf - want).abs().max().item() <= 1e-6


def test_prop_loss_and_compute_loss_validate_inputs():
    from nerf_amd import kernels as Kn
    from nerf_amd.prop_sampler import PropNetEstimator
    R, n, Kb = 8, 16, 12
    q_vals = torch.linspace(0, 1, n + 1).expand(R, n + 1).contiguous().to(DEV)
    k_vals = torch.linspace(0, 1, Kb + 1).expand(R, Kb + 1).contiguous().to(DEV)
    q_cdf, k_cdf = q_vals.clone(), k_vals.clone()
    Kn.prop_loss(q_vals, q_cdf, k_vals, k_cdf, 1e-7)                       # well-formed: fine
    with pytest.raises(ValueError):
        Kn.prop_loss(q_vals, q_cdf[:, :-1], k_vals, k_cdf, 1e-7)           # cdf / edges mismatch
    with pytest.raises(ValueError):
        Kn.prop_loss(q_vals, q_cdf, k_vals[:4], k_cdf[:4], 1e-7)           # different ray counts
    with pytest.raises(ValueError):
        Kn.prop_loss(q_vals.t().contiguous().t(), q_cdf, k_vals, k_cdf, 1e-7)   # column-major edges
    with pytest.raises(ValueError):
        Kn.prop_loss(q_vals.cpu(), q_cdf, k_vals, k_cdf, 1e-7)             # host tensor
    est = PropNetEstimator()
    est.prop_cache = [(k_vals, torch.rand(R, Kb, device=DEV), k_cdf), (q_vals, None, None)]
    with pytest.raises(ValueError):
        est.compute_loss(torch.rand(R, n + 3, device=DEV))                 # trans of another sample count


@pytest.mark.parametrize("transform", ["uniform", "lindisp"])
@pytest.mark.parametrize("K,n", [(1, 64), (64, 192), (300, 100)])
def test_prop_sample_deterministic_vs_oracle(transform, K, n):
    from nerf_amd import kernels as Kn
    R = 29
    g = torch.Generator().manual_seed(K + n)
    vals = torch.sort(torch.rand(R, K + 1, generator=g), dim=1).values
    vals[:, 0], vals[:, -1] = 0.0, 1.0
    cdf = NO.prop_cdf(_weights(R, K, 7, zeros=K > 2))
    s, t = Kn.prop_sample(vals.to(DEV), cdf.to(DEV), n, False, 0, 0 if transform == "uniform" else 1, 2.0, 7.0)
    s_ref = NO.invert_cdf(vals, cdf, NO.quantiles(R, n))
    torch.testing.assert_close(s.cpu(), s_ref, atol=2e-6, rtol=0)
    torch.testing.assert_close(t.cpu(), NO.stot(s.cpu(), transform, 2.0, 7.0), rtol=1e-5, atol=0)
    assert torch.all(s[:, 1:] >= s[:, :-1])


def test_prop_sample_stratified_properties():
    from nerf_amd import kernels as Kn
    R, K, n = 64, 64, 192
    vals = torch.linspace(0, 1, K + 1).expand(R, K + 1).contiguous()
    cdf = NO.prop_cdf(_weights(R, K, 3, zeros=False))
    s, _ = Kn.prop_sample(vals.to(DEV), cdf.to(DEV), n, True, 1234, 1, 2.0, 7.0)
    s2, _ = Kn.prop_sample(vals.to(DEV), cdf.to(DEV), n, True, 1234, 1, 2.0, 7.0)
    s3, _ = Kn.prop_sample(vals.to(DEV), cdf.to(DEV), n, True, 99, 1, 2.0, 7.0)
    assert torch.equal(s, s2) and not torch.equal(s, s3)
    s = s.cpu()
    assert torch.all(s[:, 1:] >= s[:, :-1]) and torch.all(s[:, 0] == 0) and torch.all(s[:, -1] == 1)
    # each interior quantile lies in [(i - 1/2)/n, (i + 1/2)/n): its edge between those quantiles' inverses
    lo = NO.invert_cdf(vals, cdf, ((torch.arange(n + 1) - 0.5).clamp(min=0) / n).expand(R, n + 1))
    hi = NO.invert_cdf(vals, cdf, ((torch.arange(n + 1) + 0.5).clamp(max=n) / n).expand(R, n + 1))
    assert torch.all(s >= lo - 1e-6) and torch.all(s <= hi + 1e-6)


@pytest.mark.parametrize("K,n", [(64, 192), (32, 32), (200, 64)])
def test_prop_loss_and_grad_vs_oracle(K, n):
    from nerf_amd import kernels as Kn
    R = 41
    g = torch.Generator().manual_seed(K * n)
    k_vals = torch.sort(torch.rand(R, K + 1, generator=g), dim=1).values
    k_vals[:, 0], k_vals[:, -1] = 0.0, 1.0
    # query edges: sorted, one of them exactly on a key edge
    q_vals = torch.sort(torch.cat([torch.rand(R, n - 2, generator=g), k_vals[:, 7:8]], dim=1), dim=1).values
    q_vals = torch.cat([torch.zeros(R, 1), q_vals, torch.ones(R, 1)], dim=1)
    kw = _weights(R, K, 11, zeros=False)
    k_cdf = NO.prop_cdf(kw)
    q_cdf = NO.prop_cdf(_weights(R, n, 12))
    lr, gw = Kn.prop_loss(q_vals.to(DEV), q_cdf.to(DEV), k_vals.to(DEV), k_cdf.to(DEV), 1e-7, 1.0 / (R * n),
                          want_grad=True)
    ref = NO.pdf_loss(q_vals, q_cdf, k_vals, k_cdf).double().sum(dim=1)
    torch.testing.assert_close(lr.cpu().double(), ref, rtol=1e-5, atol=1e-12)
    kwr = kw.clone().requires_grad_(True)
    NO.interlevel_loss(q_vals, q_cdf, k_vals, kwr).backward()
    scale = kwr.grad.abs().max().item()
    np.testing.assert_allclose(gw.cpu().numpy(), kwr.grad.numpy(), atol=1e-5 * scale, rtol=0)


def test_estimator_rendering_loss_vs_oracle():
    """PropNetEstimator.sampling (one proposal level of 64, 192 final intervals, lindisp, not
    stratified) -> rendering -> compute_loss with an analytic density, against the oracle pipeline;
    the loss gradient reaches the proposal densities."""
    from nerf_amd.prop_sampler import PropNetEstimator, rendering
    R, P, S, near, far = 33, 64, 192, 2.0, 7.0
    g = torch.Generator().manual_seed(5)
    o = torch.randn(R, 3, generator=g)
    d = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1)
    prop_scale = torch.tensor(3.0, requires_grad=True)

    def density(o_, d_, t0, t1, scale):
        p = o_[:, None] + d_[:, None] * ((t0 + t1) / 2)[..., None]
        return scale * torch.exp(-(p * p).sum(-1) / 4.0)

    od, dd = o.to(DEV), d.to(DEV)
    ps = prop_scale.detach().to(DEV).requires_grad_(True)
    est = PropNetEstimator()
    t0, t1 = est.sampling([lambda a, b: density(od, dd, a, b, ps)], [P], S, R, near, far, "lindisp", False, True)
    w_k_dev = est.prop_cache[0][1].detach().cpu()
    colors, opac, depth, extras = rendering(
        t0, t1, rgb_sigma_fn=lambda a, b, _: (torch.sigmoid(density(od, dd, a, b, 1.0))[..., None].expand(*a.shape, 3),
                                              density(od, dd, a, b, 5.0)))
    loss = est.compute_loss(extras["trans"])
    loss.backward()
    # oracle
    s_k = NO.invert_cdf(torch.tensor([[0.0, 1.0]]).expand(R, 2), torch.tensor([[0.0, 1.0]]).expand(R, 2),
                        NO.quantiles(R, P))
    t_k = NO.stot(s_k, "lindisp", near, far)
    sig_k = density(o, d, t_k[:, :-1], t_k[:, 1:], prop_scale)
    w_k = NO.render_weights(sig_k, t_k[:, 1:] - t_k[:, :-1])
    torch.testing.assert_close(w_k_dev, w_k.detach(), atol=2e-6, rtol=0)
    # inverse-cdf sampling is discontinuous where the cdf is flat: each stage is checked on the
    # device's own inputs (an ulp in a zero-mass stretch may move an edge across it)
    s_q = NO.invert_cdf(s_k, NO.prop_cdf(w_k_dev), NO.quantiles(R, S))
    t_q = NO.stot(s_q, "lindisp", near, far)
    torch.testing.assert_close(t0.cpu(), t_q[:, :-1], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(t1.cpu(), t_q[:, 1:], rtol=1e-5, atol=1e-5)
    w_q = NO.render_weights(density(o, d, t_q[:, :-1], t_q[:, 1:], 5.0), t_q[:, 1:] - t_q[:, :-1])
    w_q_dev = extras["weights"].detach().cpu()
    torch.testing.assert_close(w_q_dev, w_q, atol=2e-6, rtol=0)
    torch.testing.assert_close(opac.detach().cpu()[:, 0], w_q.sum(-1), atol=2e-5, rtol=0)   # 192 terms
    ref = NO.interlevel_loss(s_q, NO.prop_cdf(w_q_dev), s_k, w_k)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-4)
    np.testing.assert_allclose(ps.grad.item(), prop_scale.grad.item(), rtol=1e-4, atol=1e-9)
    assert abs(ps.grad.item()) > 0
