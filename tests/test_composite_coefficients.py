"""The fused compositing's backward coefficients (oracle.composite_coefficients, the formula the
fused forward evaluates: include/nerf_amd.h nerf_fused_composite) reproduce the gradient of the
reference's quadrature (oracle.render_rays on the NerfModel head activations, pinned to the
reference's composite golden vectors by tests/test_oracle_golden.py) taken by autograd, in fp64:
d rgb_raw = cc * g and d sigma_raw = <cs, g> for a ray's grad_rgb g.  CPU only."""
import pytest
import torch

from oracle import nerf_oracle as O


@pytest.mark.parametrize("S,sa,sb,shift", [(64, 3.0, 7.0, 0.0), (128, 3.0, 1 / 3, 0.0), (16, 1.0, 1.0, 1.0)])
def test_coefficients_match_autograd(S, sa, sb, shift):
    g = torch.Generator().manual_seed(S)
    B = 23
    sig_raw = (torch.randn(B, S, generator=g, dtype=torch.float64) * 3).requires_grad_(True)
    sig_raw.data[0, :4] = 9.0                     # the threshold branch of Softplus(threshold=8)
    rgb_raw = torch.randn(B, S, 3, generator=g, dtype=torch.float64).requires_grad_(True)
    dist = torch.rand(B, S, generator=g, dtype=torch.float64) * 0.1
    grad_rgb = torch.randn(B, 3, generator=g, dtype=torch.float64)
    sig = torch.where(sig_raw - shift > 8, sig_raw - shift, torch.log1p(torch.exp(sig_raw - shift)))
    b = (-sig * dist) * sa * sb
    T = torch.cat((torch.ones(B, 1, dtype=b.dtype), torch.exp(torch.cumsum(b[:, :-1], dim=1))), dim=1)
    w = T * (1 - torch.exp(b))
    rgb = (w.unsqueeze(-1) * torch.sigmoid(rgb_raw)).sum(1)
    (rgb * grad_rgb).sum().backward()
    cc, cs = O.composite_coefficients(sig_raw.detach(), rgb_raw.detach(), dist, sa, sb, shift)
    d_rgb = cc * grad_rgb.unsqueeze(1)
    d_sig = (cs * grad_rgb.unsqueeze(1)).sum(-1)
    assert torch.allclose(d_rgb, rgb_raw.grad, rtol=1e-10, atol=1e-13)
    assert torch.allclose(d_sig, sig_raw.grad, rtol=1e-9, atol=1e-12)


def test_oracle_render_rays_matches_restatement():
    """The oracle's fp32 render_rays (the pinned quadrature) agrees with the fp64 form used above."""
    g = torch.Generator().manual_seed(1)
    sig = torch.rand(5, 64, generator=g) * 4
    col = torch.rand(5, 64, 3, generator=g)
    dist = torch.rand(5, 64, generator=g) * 0.05
    rgb, w = O.render_rays(sig, col, dist, 3.0, 7.0)
    b = (-sig.double() * dist.double()) * 3.0 * 7.0
    T = torch.exp(torch.cumsum(b, 1) - b)
    w64 = T * (1 - torch.exp(b))
    assert torch.allclose(w.double(), w64, atol=2e-6)
    assert torch.allclose(rgb.double(), (w64.unsqueeze(-1) * col.double()).sum(1), atol=2e-6)
