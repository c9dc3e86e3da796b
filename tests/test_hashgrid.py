"""Hash-grid encoding (a9, config C5; 3d-ingp/model.py:14-121 as SURVEY.md §8(a) describes it;
the arithmetic it shares with the reference's readable 2-D copy, 2d-ingp/model.py:13-115, is pinned
by tests/golden/hashgrid2d.npz — see oracle/hashgrid_oracle.py).  CPU: the oracle's own invariants and the survey's
stated facts.  GPU: nerf_hashgrid_fwd bit-exact against the oracle (indices are integer arithmetic,
the interpolation the same fp32 operations in the same order), the deterministic fixed-point table
gradient against the oracle's fp64 scatter, and NerfModelINGP on the fused MLP against a
torch composition of the oracle features."""
import numpy as np
import pytest

from conftest import gpu_available
from oracle import hashgrid_oracle as H

gpu = pytest.mark.gpu


def test_resolutions_and_bijective_levels():
    res = H.resolutions()
    # 16 levels 16 .. 1600, levels 0-2 bijective at T = 2^16
    assert res[:4] == [16, 21, 29, 40] and res[-1] == 1600 and len(res) == 16
    assert [(r + 1) ** 3 <= 2 ** 16 for r in res[:4]] == [True, True, True, False]


def test_hash_low_bits_equal_int64_remainder():
    """SURVEY: with T = 2^16 the int64 product-xor remainder equals the low 16 bits of the uint32
    product-xor, negative corners included."""
    rng = np.random.default_rng(0)
    c = rng.integers(-5000, 5000, size=(4096, 3))
    idx = H.corner_index(c, 1600, 2 ** 16)
    u = (c.astype(np.uint64) & 0xffffffff).astype(np.uint64)
    h32 = ((u[:, 0] * 1) ^ (u[:, 1] * 2654435761) ^ (u[:, 2] * 805459861)) & 0xffffffff
    assert np.array_equal(idx, (h32 & 0xffff).astype(np.int64))
    assert (idx >= 0).all() and (idx < 2 ** 16).all()


def test_trilinear_weights_partition_unity():
    rng = np.random.default_rng(1)
    x = rng.uniform(-4, 4, size=(1000, 3)).astype(np.float32)
    for r in (16, 137, 1600):
        _, w = H.level_corners(x, r, 2 ** 16)
        assert np.allclose(w.sum(axis=1), 1.0, atol=2e-6)
        assert (w >= -1e-7).all()


def test_constant_table_gives_constant_features():
    table = np.full((3, 256, 2), 0.25, dtype=np.float32)
    x = np.random.default_rng(2).uniform(-3, 3, size=(64, 3)).astype(np.float32)
    out = H.encode(x, table, [4, 5, 9])
    assert np.allclose(out, 0.25, atol=1e-6)


# ----------------------------------------------------------------------------- GPU
def _table(L, T, F, seed=3):
    return (np.random.default_rng(seed).standard_normal((L, T, F)) * 0.1).astype(np.float32)


@gpu
@pytest.mark.parametrize("T,F,L", [(2 ** 16, 2, 16), (2 ** 14, 4, 8), (1000, 2, 4)])
def test_hashgrid_fwd_bit_exact_vs_oracle(T, F, L):
    import torch
    from nerf_amd import kernels as K
    res = H.resolutions(L)
    table = _table(L, T, F)
    rng = np.random.default_rng(4)
    x = rng.uniform(-6, 6, size=(3001, 3)).astype(np.float32)      # includes positions outside [-4, 4]
    ref = H.encode(x, table, res)
    dev = torch.device("cuda", 0)
    out = torch.full((x.shape[0], K.pad32(L * F)), float("nan"), device=dev)
    K.hashgrid_fwd(K.make_hashgrid_params(L, T, F, res), torch.from_numpy(table).to(dev), out,
                   x=torch.from_numpy(x).to(dev), n_samples=x.shape[0])
    got = out[:, :L * F].cpu().numpy()
    assert np.array_equal(got, ref)


@gpu
def test_hashgrid_fwd_ray_mode():
    """Positions generated from rays (o + t_mid d) as the fused encodings do."""
    import torch
    from nerf_amd import kernels as K
    L, T, F = 16, 2 ** 16, 2
    res = H.resolutions(L)
    table = _table(L, T, F, 5)
    g = torch.Generator().manual_seed(6)
    B, S = 37, 19
    o = torch.randn(B, 3, generator=g) * 2
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=1)
    t0 = torch.sort(torch.rand(B, S, generator=g) * 5 + 2, dim=1).values
    t1 = torch.cat([t0[:, 1:], torch.full((B, 1), 7.0)], dim=1)
    tq = (t0 + t1) / 2
    pos = (o.unsqueeze(1) + tq.unsqueeze(2) * d.unsqueeze(1)).reshape(-1, 3).numpy()
    ref = H.encode(pos, table, res)
    dev = torch.device("cuda", 0)
    out = torch.empty(B * S, 32, device=dev)
    K.hashgrid_fwd(K.make_hashgrid_params(L, T, F, res, query=1), torch.from_numpy(table).to(dev), out,
                   ray_o=o.to(dev), ray_d=d.to(dev), t_start=t0.to(dev), t_end=t1.to(dev), n_samples=B * S,
                   samples_per_ray=S)
    assert np.array_equal(out.cpu().numpy(), ref)


@gpu
def test_hashgrid_bwd_vs_oracle_and_deterministic():
    import torch
    from nerf_amd import kernels as K
    L, T, F = 16, 2 ** 16, 2
    res = H.resolutions(L)
    rng = np.random.default_rng(7)
    x = rng.uniform(-4.5, 4.5, size=(20000, 3)).astype(np.float32)
    g = (rng.standard_normal((x.shape[0], L * F)) * 1e-3).astype(np.float32)
    ref = H.encode_backward(x, g, (L, T, F), res)
    dev = torch.device("cuda", 0)
    p = K.make_hashgrid_params(L, T, F, res)
    ws = torch.zeros((K.hashgrid_workspace_bytes(p) + 7) // 8, dtype=torch.int64, device=dev)
    outs = []
    for _ in range(2):
        gt = torch.empty(L, T, F, device=dev)
        K.hashgrid_bwd(p, torch.from_numpy(g).to(dev), gt, ws, x=torch.from_numpy(x).to(dev), n_samples=x.shape[0])
        outs.append(gt.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])                      # order-independent fixed point
    assert int(ws[32:].abs().sum().item()) == 0                    # accumulators left zero (past the 256-B header)
    scale = np.abs(ref).max()
    assert np.abs(outs[0] - ref).max() <= 1e-6 * scale + 1e-12
    # accumulate mode adds onto the existing gradient
    gt = torch.from_numpy(outs[0]).to(dev)
    K.hashgrid_bwd(p, torch.from_numpy(g).to(dev), gt, ws, x=torch.from_numpy(x).to(dev), n_samples=x.shape[0],
                   accumulate=True)
    assert np.allclose(gt.cpu().numpy(), 2 * outs[0], rtol=1e-6, atol=1e-12)


@gpu
def test_hashgrid_bwd_nonfinite_gradient_gives_nan():
    import torch
    from nerf_amd import kernels as K
    L, T, F = 4, 1024, 2
    res = H.resolutions(L)
    dev = torch.device("cuda", 0)
    p = K.make_hashgrid_params(L, T, F, res)
    ws = torch.zeros((K.hashgrid_workspace_bytes(p) + 7) // 8, dtype=torch.int64, device=dev)
    x = torch.rand(100, 3, device=dev)
    g = torch.ones(100, 8, device=dev)
    g[5, 3] = float("inf")
    gt = torch.zeros(L, T, F, device=dev)
    K.hashgrid_bwd(p, g, gt, ws, x=x, n_samples=100)
    assert torch.isnan(gt).all()
    assert int(ws[32:].abs().sum().item()) == 0


@gpu
def test_nerf_model_ingp_forward_backward_vs_oracle_features():
    """NerfModelINGP (fused MLP over the hash features) against torch fp64 on the oracle's
    features: densities/colours, and the table gradient through the fused backward."""
    import torch
    from nerf_amd import NerfModelINGP
    torch.manual_seed(0)
    model = NerfModelINGP()
    with torch.no_grad():
        model.position_encoder.table.normal_(0, 0.5)            # features large enough to matter
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    dev = torch.device("cuda", 0)
    model = model.to(dev)
    g = torch.Generator().manual_seed(8)
    N = 4096
    pos = torch.rand(N, 3, generator=g) * 8 - 4
    dirs = torch.nn.functional.normalize(torch.randn(N, 3, generator=g), dim=1)
    dens, rgb = model(pos.to(dev), dirs.to(dev))
    w = torch.randn(N, 4, generator=g)
    loss = (rgb * w[:, :3].to(dev)).sum() + (dens * w[:, 3].to(dev)).sum()
    loss.backward()
    # reference: oracle features, torch fp64 MLP with the same weights
    enc = H.encode(pos.numpy(), sd["position_encoder.table"].numpy(), model.position_encoder.resolutions)
    fe = torch.from_numpy(enc).double().requires_grad_(True)
    k = torch.arange(4, dtype=torch.float64)
    args = dirs.double().repeat_interleave(4, dim=1) * (2.0 ** k).repeat(3)
    dpe = torch.cat([torch.cos(args), torch.sin(args)], dim=1)
    z = fe
    for j in range(9):
        lin = f"model_segments.0.{2 * j}"
        z = z @ sd[lin + ".weight"].double().T + sd[lin + ".bias"].double()
        if j < 8:
            z = torch.relu(z)
    h = torch.relu(torch.cat([z[:, :256], dpe], 1) @ sd["model_color.0.weight"].double().T + sd["model_color.0.bias"].double())
    h = h @ sd["model_color.2.weight"].double().T + sd["model_color.2.bias"].double()
    ref_d = torch.nn.functional.softplus(z[:, 256] - 1.0, beta=1, threshold=8)
    ref_c = torch.sigmoid(h[:, :3])
    assert (dens.detach().cpu().double() - ref_d).abs().max() <= 1e-4 * max(1.0, ref_d.abs().max().item())
    assert (rgb.detach().cpu().double() - ref_c).abs().max() <= 1e-4
    ref_loss = (ref_c * w[:, :3].double()).sum() + (ref_d * w[:, 3].double()).sum()
    ref_loss.backward()
    ref_gt = H.encode_backward(pos.numpy(), fe.grad.numpy(), tuple(sd["position_encoder.table"].shape),
                               model.position_encoder.resolutions)
    got = model.position_encoder.table.grad.cpu().double().numpy()
    scale = np.abs(ref_gt).max()
    # the split-precision backward through 10 ReLU layers: within 1e-2 of the gradient's scale, the
    # bound of the fused input-gradient chain's own tests (tests/test_gpu_fused.py)
    assert np.abs(got - ref_gt).max() <= 1e-2 * scale, (np.abs(got - ref_gt).max(), scale)


# ------------------------------------------------------- pinned by the reference's 2-D hash grid
def test_oracle_matches_reference_2d_hash_grid(golden):
    """2d-ingp/model.py:13-115 (tests/golden/hashgrid2d.npz): resolution schedule, bijective flags,
    corner indices (int64, exact), bilinear weights (exact) and features."""
    g = golden("hashgrid2d")
    T = 2 ** 14
    res = H.resolutions(8, 16, 4096)
    assert res == g["res"].tolist()
    assert [int((r + 1) ** 2 <= T) for r in res] == g["bijective"].tolist()
    u = g["u"]
    for l, r in enumerate(res):
        idx, w = H.level_corners_2d(u, r, T)
        assert np.array_equal(idx, g[f"idx{l}"]), l
        assert np.array_equal(w, g[f"w{l}"]), l
    feat = H.encode_2d(u, [g[f"table{l}"] for l in range(8)], res, T)
    np.testing.assert_allclose(feat, g["features"], rtol=1e-6, atol=1e-12)


def test_3d_oracle_reduces_to_the_reference_2d_grid(golden):
    """The 3-D restatement at z = -4 (x_hat_z = 0: the z = 1 corners weigh 0, the z = 0 corners
    hash as 2-D) on x = 8u - 4 (x/8 + 0.5 = u exactly) gives the 2-D reference's features on every
    level where both are hashed or both bijective."""
    g = golden("hashgrid2d")
    T, F = 2 ** 14, 2
    res = g["res"].tolist()
    lv = [l for l, r in enumerate(res) if ((r + 1) ** 3 <= T) == ((r + 1) ** 2 <= T)]
    assert lv == [0, 3, 4, 5, 6, 7]
    u = g["u"]
    x = np.concatenate([8 * u - 4, np.full((u.shape[0], 1), -4.0, np.float32)], axis=1).astype(np.float32)
    table = np.zeros((len(lv), T, F), np.float32)
    for i, l in enumerate(lv):
        t = g[f"table{l}"]
        table[i, :t.shape[0]] = t
    out = H.encode(x, table, [res[l] for l in lv])
    want = np.concatenate([g["features"][:, l * F:(l + 1) * F] for l in lv], axis=1)
    # corners summed in another order than the reference's: fp32 rounding of a 4-term sum
    np.testing.assert_allclose(out, want, rtol=0, atol=2e-7 * np.abs(want).max())


@gpu
def test_hashgrid_kernel_vs_reference_2d_grid(golden):
    """nerf_hashgrid_fwd on the same reduction: the kernel reproduces the reference's 2-D
    features (2d-ingp/model.py) on the shared levels."""
    import torch
    from nerf_amd import kernels as K
    g = golden("hashgrid2d")
    T, F = 2 ** 14, 2
    res = g["res"].tolist()
    lv = [0, 3, 4, 5, 6, 7]
    u = g["u"]
    x = np.concatenate([8 * u - 4, np.full((u.shape[0], 1), -4.0, np.float32)], axis=1).astype(np.float32)
    table = np.zeros((len(lv), T, F), np.float32)
    for i, l in enumerate(lv):
        t = g[f"table{l}"]
        table[i, :t.shape[0]] = t
    dev = torch.device("cuda", 0)
    out = torch.zeros(x.shape[0], 32, device=dev)
    K.hashgrid_fwd(K.make_hashgrid_params(len(lv), T, F, [res[l] for l in lv]), torch.from_numpy(table).to(dev),
                   out, x=torch.from_numpy(x).to(dev), n_samples=x.shape[0])
    want = np.concatenate([g["features"][:, l * F:(l + 1) * F] for l in lv], axis=1)
    np.testing.assert_allclose(out[:, :len(lv) * F].cpu().numpy(), want, rtol=0, atol=2e-7 * np.abs(want).max())
