"""CPU properties of the nerfacc restatement (oracle/nerfacc_oracle.py; parity unpinned — nerfacc
is absent): the cdf is 0 .. exclusive sums .. 1, inverse-cdf sampling of a uniform cdf is the
identity, lindisp maps the ends to near / far and is uniform in 1/t, and the interlevel loss is
non-negative and zero when the proposal equals the final distribution."""
import torch

from oracle import nerfacc_oracle as NO


def test_cdf_and_inverse():
    w = torch.rand(5, 16)
    w = w / w.sum(1, keepdim=True) * 0.8
    cdf = NO.prop_cdf(w)
    assert torch.all(cdf[:, 0] == 0) and torch.all(cdf[:, -1] == 1) and torch.all(cdf[:, 1:] >= cdf[:, :-1])
    torch.testing.assert_close(cdf[:, 1:-1], torch.cumsum(w, 1)[:, :-1], atol=1e-6, rtol=0)
    vals = torch.linspace(0, 1, 17).expand(5, 17)
    u = NO.quantiles(5, 33)
    torch.testing.assert_close(NO.invert_cdf(vals, vals, u), u, atol=1e-6, rtol=0)


def test_lindisp():
    s = torch.linspace(0, 1, 11)
    t = NO.stot(s, "lindisp", 2.0, 7.0)
    torch.testing.assert_close(t[[0, -1]], torch.tensor([2.0, 7.0]))
    torch.testing.assert_close(1 / t, 0.5 + s * (1 / 7 - 0.5), atol=1e-6, rtol=0)


def test_interlevel_loss_zero_at_match_and_nonnegative():
    R, K = 4, 32
    vals = torch.sort(torch.rand(R, K + 1), 1).values
    vals[:, 0], vals[:, -1] = 0, 1
    w = torch.rand(R, K)
    w = w / w.sum(1, keepdim=True)
    cdf = NO.prop_cdf(w)
    assert NO.pdf_loss(vals, cdf, vals, cdf).abs().max() < 1e-6
    q = torch.sort(torch.rand(R, 65), 1).values
    q[:, 0], q[:, -1] = 0, 1
    qw = torch.rand(R, 64)
    assert torch.all(NO.pdf_loss(q, NO.prop_cdf(qw / qw.sum(1, keepdim=True)), vals, cdf) >= 0)
