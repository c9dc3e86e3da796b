"""GPU parity: the HIP path (through the C-ABI) against the reference's golden
vectors and the CPU oracle.  Stated tolerances (fp32):
  encodings 2e-6 abs (same op order; ocml vs SLEEF sin/cos ulps),
  compositing 2e-6 abs on rgb / weights, 2e-5 on input gradients,
  resampling bit-exact, linear layers / field MLP 1e-4 (MFMA vs BLAS summation order).
"""
import math

import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def g2d(a):
    return torch.from_numpy(np.asarray(a)).to(DEV)


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import nerf_amd
    nerf_amd._lib.load()  # fail loudly if the HIP library is missing
    yield


# ----------------------------------------------------------------------------- encodings
def test_fourier_golden(golden):
    from nerf_amd import FourierFeatures
    g = golden("pe")
    x, d = g2d(g["x"]), g2d(g["dir"])
    np.testing.assert_allclose(FourierFeatures(10, 2 * math.pi)(x).cpu().numpy(), g["fourier_L10_2pi"], atol=2e-6,
                               rtol=0)
    np.testing.assert_allclose(FourierFeatures(4, 1.0)(d).cpu().numpy(), g["fourier_L4_1"], atol=2e-6, rtol=0)


@pytest.mark.parametrize("alpha", [0.0, 3.4, 10.0])
@pytest.mark.parametrize("ident", [True, False])
@pytest.mark.parametrize("sname", ["1", "2pi"])
def test_barf_golden_fwd_bwd(golden, alpha, ident, sname):
    from nerf_amd import BarfPositionalEncoding
    g = golden("pe")
    scale = 1.0 if sname == "1" else 2 * math.pi
    key = f"barf_L10_a{alpha}_id{int(ident)}_s{sname}"
    enc = BarfPositionalEncoding(10, alpha, 0, 1, ident, scale).to(DEV)
    x = g2d(g["x"]).requires_grad_(True)
    y = enc(x)
    np.testing.assert_allclose(y.detach().cpu().numpy(), g[key], atol=2e-6, rtol=0)
    (y * g2d(g[key + "_gy"])).sum().backward()
    # d/dx sums ~20 terms of magnitude up to scale*2^9*|g|: relative tolerance on that scale
    np.testing.assert_allclose(x.grad.cpu().numpy(), g[key + "_dx"], atol=2e-3, rtol=1e-5)


def test_barf_update_alpha_no_sync(golden):
    from nerf_amd import BarfPositionalEncoding
    enc = BarfPositionalEncoding(10, 0.0, 10.0, 20.0, True, 1.0).to(DEV)
    enc.update_alpha(13.7)
    assert abs(enc._alpha_host - float(golden("pe")["barf_update_alpha_13.7"][0])) == 0.0
    assert abs(float(enc.alpha) - enc._alpha_host) == 0.0


@pytest.mark.parametrize("pwname", ["400", "800"])
@pytest.mark.parametrize("dv", [True, False])
@pytest.mark.parametrize("pws", [0.0, 0.5])
def test_ipe_golden(golden, pwname, dv, pws):
    from nerf_amd import IntegratedFourierFeatures
    g = golden("pe")
    enc = IntegratedFourierFeatures(10, 2 * math.pi, True, dv)
    enc.pixel_width_sigma = pws
    y = enc(g2d(g["x"]), g2d(g["dir"]), g2d(g[f"pw_{pwname}"]), g2d(g["t0"]), g2d(g["t1"]))
    np.testing.assert_allclose(y.cpu().numpy(), g[f"ipe_{pwname}_dv{int(dv)}_pws{pws}"], atol=2e-6, rtol=0)


def test_ipe_barf_golden(golden):
    from nerf_amd import IntegratedBarfFourierFeatures
    g = golden("pe")
    enc = IntegratedBarfFourierFeatures(10, 3.4, 0, 1, True, 1.0, True).to(DEV)
    enc.pixel_width_sigma = 0.0
    for pwname in ("400", "800"):
        y = enc(g2d(g["x"]), g2d(g["dir"]), g2d(g[f"pw_{pwname}"]), g2d(g["t0"]), g2d(g["t1"]))
        np.testing.assert_allclose(y.cpu().numpy(), g[f"ipebarf_{pwname}_a3.4"], atol=2e-6, rtol=0)


def test_encode_rays_matches_oracle():
    from nerf_amd import BarfPositionalEncoding
    torch.manual_seed(0)
    B, S = 37, 70
    o = torch.randn(B, 3) * 4
    d = torch.nn.functional.normalize(torch.randn(B, 3), dim=1)
    t0 = torch.sort(2 + torch.rand(B, S) * 6, dim=1).values
    t1 = torch.cat((t0[:, 1:], torch.full((B, 1), 8.0)), dim=1)
    enc = BarfPositionalEncoding(10, 6.3, 0, 1, True, 1.0).to(DEV)
    for query, strat in ((0, "left"), (1, "middle")):
        out = enc.encode_rays(o.to(DEV), d.to(DEV), t0.to(DEV), t1.to(DEV), None, S, query, 0)
        pos, _ = O.compute_positions(o, d, t0, t1, strat)
        ref = O.barf_pe(pos.view(-1, 3), 10, 6.3, True, 1.0)
        got = out.cpu()
        np.testing.assert_allclose(got[:, :63].numpy(), ref.numpy(), atol=2e-6, rtol=0)
        assert torch.all(got[:, 63:] == 0)


@pytest.mark.parametrize("kind", [0, 1])
def test_encode_layouts_agree(kind):
    """The LDS-staged kernel (16-byte aligned rows of <= 128 columns) and the per-quad kernel
    (wider or unaligned rows) write identical encodings; pad columns are zero."""
    from nerf_amd import kernels as K
    torch.manual_seed(5)
    B, S = 29, 67
    o = (torch.randn(B, 3) * 2).to(DEV)
    d = torch.nn.functional.normalize(torch.randn(B, 3), dim=1).to(DEV)
    t0 = torch.sort(2 + torch.rand(B, S) * 6, dim=1).values
    t1 = torch.cat((t0[:, 1:], torch.full((B, 1), 8.0)), dim=1)
    pw = torch.full((B,), 1 / 555.56, device=DEV)
    p = K.make_pe_params(kind, 10, True, 1.0, query=1, pixel_width_sigma=0.0, distribute_variance=False,
                         pw_mode=0, mask=[1.0] * 7 + [0.3, 0.0, 0.0])
    outs = [K.encode_fwd(p, 63, ray_o=o, ray_d=d, t_start=t0.to(DEV), t_end=t1.to(DEV), pixel_width=pw,
                         n_samples=B * S, samples_per_ray=S, n_rays=B, out_ld=ld, device=DEV) for ld in (64, 67, 160)]
    for out in outs[1:]:
        assert torch.equal(out[:, :63], outs[0][:, :63])
        assert torch.all(out[:, 63:] == 0)
    assert torch.all(outs[0][:, 63] == 0)


# ----------------------------------------------------------------------------- compositing
@pytest.mark.parametrize("S", [64, 128, 192])
@pytest.mark.parametrize("magic", [1 / 3, 7.0])
def test_render_rays_golden_and_grad(golden, S, magic):
    from nerf_amd.model_interpolation import _RenderRaysFn
    g = golden("composite")
    k = f"S{S}"
    sig = g2d(g[f"{k}_sigma"]).requires_grad_(True)
    col = g2d(g[f"{k}_color"]).requires_grad_(True)
    dist = g2d(g[f"{k}_dist"])
    rgb, w = _RenderRaysFn.apply(sig, col, dist, 3.0, magic)
    if magic == 1 / 3:
        np.testing.assert_allclose(rgb.detach().cpu().numpy(), g[f"{k}_rgb"], atol=2e-6, rtol=0)
        np.testing.assert_allclose(w.detach().cpu().numpy(), g[f"{k}_w"], atol=2e-6, rtol=0)
    # gradients against the oracle's autograd (itself pinned to the golden gradients)
    so = torch.from_numpy(g[f"{k}_sigma"]).requires_grad_(True)
    co = torch.from_numpy(g[f"{k}_color"]).requires_grad_(True)
    rr, ww = O.render_rays(so, co, torch.from_numpy(g[f"{k}_dist"]), 3.0, magic)
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), rr.detach().numpy(), atol=2e-6, rtol=0)
    gr, gw = torch.from_numpy(g[f"{k}_grgb"]), torch.from_numpy(g[f"{k}_gw"])
    ((rr * gr).sum() + (ww * gw).sum()).backward()
    ((rgb * gr.to(DEV)).sum() + (w * gw.to(DEV)).sum()).backward()
    np.testing.assert_allclose(sig.grad.cpu().numpy(), so.grad.numpy(), atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(col.grad.cpu().numpy(), co.grad.numpy(), atol=2e-6, rtol=0)


@pytest.mark.parametrize("width,S", [(32, 128), (4, 128), (4, 64), (4, 100), (4, 257)])
def test_composite_raw_heads_fused_activation(width, S):
    """act = 1: softplus(thr 8) / sigmoid applied in-kernel on strided raw head buffers.
    width 4 is the [rgb | sigma] head row the kernels load and store as one 16-byte access."""
    from nerf_amd.model_interpolation import composite_raw
    from nerf_amd.model_interpolation_architecture import RawHeads
    torch.manual_seed(1)
    B = 50
    head = (torch.randn(B * S, width) * 3)
    head[:, 4:] = 0
    dist = torch.rand(B, S) * 0.05
    hd = head.to(DEV).requires_grad_(True)
    rgb, w = composite_raw(RawHeads(hd, hd, 3), dist.to(DEV), B, S, 3.0, 7.0)
    hc = head.clone().requires_grad_(True)
    rr, ww = O.render_rays(O.softplus8(hc[:, 3]).view(B, S), torch.sigmoid(hc[:, :3]).view(B, S, 3), dist, 3.0, 7.0)
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), rr.detach().numpy(), atol=2e-6, rtol=0)
    np.testing.assert_allclose(w.cpu().numpy(), ww.detach().numpy(), atol=2e-6, rtol=0)
    gr = torch.randn(B, 3)
    (rr * gr).sum().backward()
    (rgb * gr.to(DEV)).sum().backward()
    np.testing.assert_allclose(hd.grad.cpu().numpy(), hc.grad.numpy(), atol=2e-5, rtol=1e-5)


# ----------------------------------------------------------------------------- sampling
@pytest.mark.parametrize("N", [128, 256])
def test_resample_barf_bitexact(golden, N):
    from nerf_amd import kernels as K
    g = golden("resample")
    k = f"barf_N{N}"
    t0, t1, st = K.resample_pdf(g2d(g[f"{k}_tc"]), g2d(g[f"{k}_w"]), g2d(g[f"{k}_dist"]), N, 0, 2.0, 8.0, 1, 0)
    assert int(st.item()) == 0
    np.testing.assert_array_equal(t0.cpu().numpy(), g[f"{k}_t0"])
    np.testing.assert_array_equal(t1.cpu().numpy(), g[f"{k}_t1"])


def test_resample_n2v_bitexact(golden):
    from nerf_amd import kernels as K
    g = golden("resample")
    t0, t1, st = K.resample_pdf(g2d(g["n2v_tc"]), g2d(g["n2v_w"]), g2d(g["n2v_dist"]), 256, 1, 0.1, 1 / 3, 1, 0)
    assert int(st.item()) == 0
    np.testing.assert_array_equal(t0.cpu().numpy(), g["n2v_t0"])
    np.testing.assert_array_equal(t1.cpu().numpy(), g["n2v_t1"])


def test_resample_random_vs_oracle():
    from nerf_amd import kernels as K
    torch.manual_seed(7)
    B, Kb, N = 300, 64, 192
    tc = torch.sort(2 + torch.rand(B, Kb) * 6, dim=1).values
    dist = torch.diff(tc, dim=1, append=torch.full((B, 1), 8.0))
    w = torch.nn.functional.softplus(torch.randn(B, Kb) * 2) * (torch.rand(B, Kb) < 0.5)
    w[:, 0] += 1e-3
    t0, t1, st = K.resample_pdf(tc.to(DEV), w.to(DEV), dist.to(DEV), N, 0, 2.0, 8.0, 3, 0)
    r0, r1, ok = O.sample_t_pdf_weighted(tc, w, dist, N, 8.0, 0)
    assert ok and int(st.item()) == 0
    # the oracle and the kernel both form sum(w) in fp64: bit-exact
    np.testing.assert_array_equal(t0.cpu().numpy(), r0.numpy())
    np.testing.assert_array_equal(t1.cpu().numpy(), r1.numpy())


def test_resample_fallback_batchwide():
    """A ray with all-zero weights makes the reference fall back, batch-wide, to
    equidistant sampling with a per-ray offset in (-D, 0] (model_interpolation.py:273-275)."""
    from nerf_amd import kernels as K
    torch.manual_seed(8)
    B, Kb, N = 9, 64, 128
    tc = torch.sort(2 + torch.rand(B, Kb) * 6, dim=1).values
    dist = torch.diff(tc, dim=1, append=torch.full((B, 1), 8.0))
    w = torch.rand(B, Kb)
    w[4] = 0
    t0, t1, st = K.resample_pdf(tc.to(DEV), w.to(DEV), dist.to(DEV), N, 0, 2.0, 8.0, 11, 0)
    assert int(st.item()) & 1
    base = O.linspace_t(2.0, 8.0, N)
    delta = (8.0 - 2.0) / N
    off = t0.cpu() - base.unsqueeze(0)
    assert torch.all(off <= 1e-5) and torch.all(off >= -delta - 1e-5)
    assert torch.allclose(off, off[:, :1].expand_as(off), atol=2e-6)
    assert torch.all(t1.cpu()[:, -1] == 8.0)


def test_sample_uniform():
    from nerf_amd import kernels as K
    B, S = 33, 64
    t0, t1 = K.sample_uniform(B, S, 2.0, 8.0, False, 0.0, 5, 0, DEV)
    ref = O.linspace_t(2.0, 8.0, S)
    np.testing.assert_allclose(t0.cpu().numpy(), ref.expand(B, S).numpy(), atol=1e-6, rtol=0)
    assert torch.equal(t1[:, :-1], t0[:, 1:]) and torch.all(t1[:, -1] == 8.0)
    t0, t1 = K.sample_uniform(B, S, 2.0, 8.0, True, 0.0, 5, 0, DEV)
    u = (t0.cpu() - ref) / ((8.0 - 2.0) / S)
    assert torch.all(u >= -1e-5) and torch.all(u < 1 + 1e-5) and u.std() > 0.2
    assert torch.equal(t1[:, :-1], t0[:, 1:])
    t0b, _ = K.sample_uniform(B, S, 2.0, 8.0, True, 0.0, 5, 0, DEV)
    assert torch.equal(t0, t0b)  # deterministic for a fixed (seed, counter)


# ----------------------------------------------------------------------------- linear layers
@pytest.mark.parametrize("M,N,ks,rd", [(1000, 256, (256, 64), (1, 1)), (777, 257, (256,), (1,)),
                                       (4096, 128, (256, 32), (1, 64)), (300, 4, (128,), (1,)),
                                       (129, 300, (32, 32, 64), (1, 3, 1)), (1000, 128, (4,), (1,)),
                                       (333, 20, (260, 12), (1, 7))])
def test_linear_fwd_wgrad(M, N, ks, rd):
    """Packed layout: segment j occupies pad32(k_j) weight columns; columns past k_j are zero."""
    from nerf_amd import kernels as K
    from nerf_amd._lib import NERF_EPI_ACCUM, NERF_EPI_BIAS, NERF_EPI_MASK, NERF_EPI_RELU
    torch.manual_seed(M + N)
    segs_cpu = [torch.randn((M + r - 1) // r, k) for k, r in zip(ks, rd)]
    Kv = sum(ks)
    Kp = sum(K.pad32(k) for k in ks)
    W = torch.randn(N, Kv) / math.sqrt(Kv)
    b = torch.randn(N)
    X = torch.cat([s.repeat_interleave(r, dim=0)[:M] for s, r in zip(segs_cpu, rd)], dim=1)
    cm = []
    off = 0
    for k in ks:
        cm += [off + j for j in range(k)] + [-1] * (K.pad32(k) - k)
        off += k
    Wp = torch.zeros(K.pad128(N), Kp)
    for j, c in enumerate(cm):
        if c >= 0:
            Wp[:N, j] = W[:, c]
    segs = [(s.to(DEV), k, r) for s, k, r in zip(segs_cpu, ks, rd)]
    ldo = (N + 3) // 4 * 4
    out = torch.empty(M, ldo, device=DEV)
    K.linear_fwd(segs, M, Wp.to(DEV), Kp, N, b.to(DEV), out, NERF_EPI_BIAS | NERF_EPI_RELU)
    ref = torch.relu(X @ W.T + b)
    np.testing.assert_allclose(out[:, :N].cpu().numpy(), ref.numpy(), atol=1e-4, rtol=1e-4)
    # ReLU-mask + accumulate epilogue
    aux = torch.randn(M, ldo)
    out2 = torch.randn(M, ldo)
    o2 = out2.clone().to(DEV)
    K.linear_fwd(segs, M, Wp.to(DEV), Kp, N, None, o2, NERF_EPI_MASK | NERF_EPI_ACCUM, aux=aux.to(DEV))
    ref2 = out2[:, :N] + (X @ W.T) * (aux[:, :N] > 0)
    np.testing.assert_allclose(o2[:, :N].cpu().numpy(), ref2.numpy(), atol=1e-4, rtol=1e-4)
    _check_mask_bits(lambda *a, **k: K.linear_fwd(segs, M, Wp.to(DEV), Kp, *a, **k), M, N, ldo, b, aux, out2)
    # weight gradient, scattered through the column map
    dY = torch.randn(M, ldo)
    dY[:, N:] = 0
    N4 = ldo
    ws = torch.empty((K.linear_wgrad_workspace_bytes(M, N4, Kp) + 3) // 4, device=DEV)
    K.linear_wgrad(dY.to(DEV), N4, segs, M, ws)
    dW = torch.empty(N, Kv, device=DEV)
    db = torch.empty(N, device=DEV)
    K.linear_wgrad_reduce(M, N4, Kp, N, ws, torch.tensor(cm, dtype=torch.int32, device=DEV), dW, db)
    np.testing.assert_allclose(dW.cpu().numpy(), (dY[:, :N].T.double() @ X.double()).float().numpy(), atol=2e-4,
                               rtol=1e-4)
    np.testing.assert_allclose(db.cpu().numpy(), dY[:, :N].sum(0).numpy(), atol=2e-4, rtol=1e-4)


def _check_mask_bits(fwd, M, N, ldo, b, aux, out2):
    """NERF_EPI_MASKOUT writes (out > 0) as bits — row m = 8 uint32 words, bit b of word
    2e + h <-> column 4(32h + b) + e; a MASK epilogue reading those bits (NERF_EPI_MASKBITS)
    equals the one reading the fp32 activation."""
    from nerf_amd._lib import NERF_EPI_ACCUM, NERF_EPI_BIAS, NERF_EPI_MASK, NERF_EPI_MASKBITS, NERF_EPI_MASKOUT, \
        NERF_EPI_RELU
    if N > 256:
        return
    act = torch.empty(M, ldo, device=DEV)
    bits = torch.full((M, 32), 0xA5, dtype=torch.uint8, device=DEV)
    fwd(N, b.to(DEV), act, NERF_EPI_BIAS | NERF_EPI_RELU | NERF_EPI_MASKOUT, aux=bits)
    pos = torch.zeros(M, 256, dtype=torch.int64)
    pos[:, :N] = (act[:, :N] > 0).cpu().long()
    q = pos.view(M, 64, 4)                                  # [m][quad][e]
    want = torch.zeros(M, 8, dtype=torch.int64)
    for e in range(4):
        for h in range(2):
            want[:, 2 * e + h] = (q[:, 32 * h:32 * h + 32, e] << torch.arange(32)).sum(1)
    got = bits.cpu().view(torch.int32).long() & 0xFFFFFFFF
    nq = (N + 3) // 4                                       # bits of quads past N are unspecified
    for h in range(2):
        nb = min(max(nq - 32 * h, 0), 32)
        valid = (1 << nb) - 1
        for e in range(4):
            assert torch.equal(got[:, 2 * e + h] & valid, want[:, 2 * e + h] & valid), (e, h)
    # the same masked + accumulated product through float aux and through the bits
    act_aux = act.clone()
    o_f = out2.clone().to(DEV)
    o_b = out2.clone().to(DEV)
    fwd(N, None, o_f, NERF_EPI_MASK | NERF_EPI_ACCUM, aux=act_aux)
    fwd(N, None, o_b, NERF_EPI_MASK | NERF_EPI_MASKBITS | NERF_EPI_ACCUM, aux=bits)
    assert torch.equal(o_f[:, :N], o_b[:, :N])


def _split_bf16(W):
    hi = W.bfloat16()
    return hi, (W - hi.float()).bfloat16()


@pytest.mark.parametrize("M,N,ks,rd", [(1000, 256, (256, 64), (1, 1)), (777, 257, (256,), (1,)),
                                       (4096, 128, (256, 32), (1, 64)), (300, 4, (128,), (1,)),
                                       (129, 300, (32, 32, 64), (1, 3, 1)), (1000, 128, (4,), (1,)),
                                       (333, 20, (260, 12), (1, 7)), (70000, 256, (256,), (1,)),
                                       # one 256 x 256 weight-gradient tile (LDS-DMA kernel): ragged
                                       # splits, per-ray rows, fewer chunks than ring slots
                                       (5003, 256, (200, 24), (1, 7)), (777, 200, (128, 60), (1, 3)),
                                       (50, 256, (256,), (1,)), (10, 160, (64,), (1,)),
                                       # 257 rows by their true count: the 256 x 256 tile + row 256
                                       (70000, 257, (256,), (1,)), (40, 257, (200,), (3,)),
                                       # N <= 16: the vector-ALU small-N weight gradient (exact fp32
                                       # products, well inside the split-precision bound)
                                       (100003, 4, (128,), (1,)), (999, 16, (64, 32), (1, 5)),
                                       (77, 12, (512, 32), (1, 7)), (5000, 8, (1024,), (1,))])
def test_linear_x3_fwd_wgrad(M, N, ks, rd):
    """3 x bf16 split-precision GEMMs (hi*hi + hi*lo + lo*hi, fp32 accumulate).

    Tolerance: each product misses lo_x*lo_w and the residual rounding of lo, both
    <= 2^-16 |x||w|, so |err| <= 2^-15 * (|X| @ |W|^T) bounds the result elementwise."""
    from nerf_amd import kernels as K
    from nerf_amd._lib import NERF_EPI_ACCUM, NERF_EPI_BIAS, NERF_EPI_MASK, NERF_EPI_RELU
    torch.manual_seed(M + N + 1)
    segs_cpu = [torch.randn((M + r - 1) // r, k) for k, r in zip(ks, rd)]
    Kv = sum(ks)
    Kp = sum(K.pad32(k) for k in ks)
    W = torch.randn(N, Kv) / math.sqrt(Kv)
    b = torch.randn(N)
    X = torch.cat([s.repeat_interleave(r, dim=0)[:M] for s, r in zip(segs_cpu, rd)], dim=1)
    cm = []
    off = 0
    for k in ks:
        cm += [off + j for j in range(k)] + [-1] * (K.pad32(k) - k)
        off += k
    cmd = torch.tensor(cm, dtype=torch.int32, device=DEV)
    ldwt = K.pad32(N)
    Wpx = torch.empty(K.pad128(N), 2 * Kp, dtype=torch.bfloat16, device=DEV)
    Wtx = torch.empty(K.pad128(Kp) + 128, 2 * ldwt, dtype=torch.bfloat16, device=DEV)
    K.pack_weight_x3(W.to(DEV), cmd, Kp, Wpx, Wtx, ldwt)
    # packing is bit-exact against torch's round-to-nearest-even split, interleaved per 32 columns
    Wp = torch.zeros(K.pad128(N), Kp)
    for j, c in enumerate(cm):
        if c >= 0:
            Wp[:N, j] = W[:, c]
    h, lo = _split_bf16(Wp)
    assert torch.equal(Wpx.cpu().view(torch.int16), K.interleave_x3(h, lo).view(torch.int16))
    Wt = torch.zeros(K.pad128(Kp) + 128, ldwt)
    Wt[:Kp, :N] = Wp[:N].T
    ht, lt = _split_bf16(Wt)
    assert torch.equal(Wtx.cpu().view(torch.int16), K.interleave_x3(ht, lt).view(torch.int16))

    segs = [(s.to(DEV), k, r) for s, k, r in zip(segs_cpu, ks, rd)]
    ldo = (N + 3) // 4 * 4
    Xd, Wd = X.double(), W.double()
    bound = 2.0 ** -15 * (Xd.abs() @ Wd.abs().T) + 1e-6
    out = torch.empty(M, ldo, device=DEV)
    K.linear_fwd_x3(segs, M, Wpx, Kp, N, b.to(DEV), out, NERF_EPI_BIAS | NERF_EPI_RELU)
    ref = torch.relu(Xd @ Wd.T + b.double())
    err = (out[:, :N].cpu().double() - ref).abs()
    assert (err <= bound + 1e-6).all(), float((err - bound).max())
    # ReLU-mask + accumulate epilogue
    aux = torch.randn(M, ldo)
    out2 = torch.randn(M, ldo)
    o2 = out2.clone().to(DEV)
    K.linear_fwd_x3(segs, M, Wpx, Kp, N, None, o2, NERF_EPI_MASK | NERF_EPI_ACCUM, aux=aux.to(DEV))
    ref2 = out2[:, :N].double() + (Xd @ Wd.T) * (aux[:, :N] > 0)
    err = (o2[:, :N].cpu().double() - ref2).abs()
    assert (err <= bound + 1e-6).all(), float((err - bound).max())
    _check_mask_bits(lambda *a, **k: K.linear_fwd_x3(segs, M, Wpx, Kp, *a, **k), M, N, ldo, b, aux, out2)
    # transposed (input-gradient) direction through Wt planes: dX = dY @ W
    dY = torch.randn(M, ldo)
    dY[:, N:] = 0
    dX = torch.empty(M, Kp, device=DEV)
    K.linear_fwd_x3([(dY.to(DEV), ldo, 1)], M, Wtx, ldwt, Kp, None, dX, 0)
    refx = dY[:, :N].double() @ Wp[:N].double()
    bx = 2.0 ** -15 * (dY[:, :N].double().abs() @ Wp[:N].double().abs()) + 1e-6
    assert ((dX.cpu().double() - refx).abs() <= bx).all()
    # weight gradient, scattered through the column map (fp64 split reduction)
    N4 = ldo
    ws = torch.empty((K.linear_wgrad_workspace_bytes(M, N4, Kp) + 3) // 4, device=DEV)
    K.linear_wgrad_x3(dY.to(DEV), N4, segs, M, ws)
    dW = torch.empty(N, Kv, device=DEV)
    db = torch.empty(N, device=DEV)
    K.linear_wgrad_reduce(M, N4, Kp, N, ws, cmd, dW, db)
    refw = dY[:, :N].T.double() @ Xd
    bw = 2.0 ** -15 * (dY[:, :N].T.double().abs() @ Xd.abs()) + 1e-6
    assert ((dW.cpu().double() - refw).abs() <= bw).all()
    np.testing.assert_allclose(db.cpu().numpy(), dY[:, :N].sum(0).numpy(), atol=2e-4, rtol=1e-4)
    if N == 257:
        # the true row count (nerf_linear_wgrad_x3 with N = 257: one 256 x 256 tile per split, row 256
        # as fp32 FMAs on the vector ALUs); a NaN-filled workspace: every slab entry the reduce reads
        # is written, rows past N are never read
        ws.fill_(float("nan"))
        K.linear_wgrad_x3(dY.to(DEV), N, segs, M, ws)
        K.linear_wgrad_reduce(M, N4, Kp, N, ws, cmd, dW, db)
        assert ((dW.cpu().double() - refw).abs() <= bw).all()
        np.testing.assert_allclose(db.cpu().numpy(), dY[:, :N].sum(0).numpy(), atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize("M0,M1,N,ks,rd0,rd1", [(3000, 5000, 256, (256,), (1,), (1,)),
                                                (70000, 33333, 257, (256,), (1,), (1,)),
                                                (2000, 1500, 256, (256, 64), (1, 1), (1, 1)),
                                                (4096, 2048, 128, (256, 32), (1, 64), (1, 32)),
                                                (1000, 37, 260, (200,), (1,), (3,)),
                                                (131072, 65536, 3, (128,), (1,), (1,)),
                                                (3000, 77, 16, (64, 32), (1, 1), (1, 64))])
def test_linear_x3_wgrad_two_row_blocks(M0, M1, N, ks, rd0, rd1):
    """nerf_linear_wgrad_x3_rows: the weight gradient of two passes' rows (own dY / X pointers,
    row strides and row divisors) in one launch and one reduce, against fp64 over the
    concatenated rows with the split-precision bound; the row-256 path (N = 257) included."""
    from nerf_amd import kernels as K
    torch.manual_seed(M0 + M1 + N)
    N4 = (N + 3) // 4 * 4
    Kp = sum(K.pad32(k) for k in ks)
    blocks, Xs, Ys = [], [], []
    for M, rd, ld_extra in ((M0, rd0, 0), (M1, rd1, 8)):
        segs_cpu = [torch.randn((M + r - 1) // r, k) for k, r in zip(ks, rd)]
        dY = torch.randn(M, N4 + ld_extra)
        dY[:, N:] = 0
        Xs.append(torch.cat([sg.repeat_interleave(r, dim=0)[:M] for sg, r in zip(segs_cpu, rd)], dim=1))
        Ys.append(dY[:, :N])
        blocks.append((dY.to(DEV), [(sg.to(DEV), k, r) for sg, k, r in zip(segs_cpu, ks, rd)], M))
    ws = torch.full(((K.linear_wgrad_workspace_bytes(M0 + M1, N4, Kp) + 3) // 4,), float("nan"), device=DEV)
    K.linear_wgrad_x3_rows(blocks, N, ws)
    cm = []
    for k in ks:
        cm += [len([c for c in cm if c >= 0]) + j for j in range(k)] + [-1] * (K.pad32(k) - k)
    dW = torch.empty(N, sum(ks), device=DEV)
    db = torch.empty(N, device=DEV)
    K.linear_wgrad_reduce(M0 + M1, N4, Kp, N, ws, torch.tensor(cm, dtype=torch.int32, device=DEV), dW, db)
    X = torch.cat(Xs).double()
    Y = torch.cat(Ys).double()
    refw = Y.T @ X
    bw = 2.0 ** -15 * (Y.abs().T @ X.abs()) + 1e-6
    assert ((dW.cpu().double() - refw).abs() <= bw).all()
    np.testing.assert_allclose(db.cpu().numpy(), Y.sum(0).numpy(), atol=2e-4, rtol=1e-4)


# ----------------------------------------------------------------------------- field MLP
def _make_models():
    from nerf_amd import BarfPositionalEncoding, FourierFeatures, NerfModel
    torch.manual_seed(0)
    barf = NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0),
                     BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0))
    torch.manual_seed(0)
    n2v = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0))
    torch.manual_seed(0)
    small = NerfModel(2, 64, False, False, 3, BarfPositionalEncoding(6, 3.4, 0, 1, True, 1.0),
                      BarfPositionalEncoding(2, 1.5, 0, 1, False, 1.0))
    return {"barf": barf, "n2v": n2v, "small": small}


@pytest.fixture(params=["highest", "high"])
def matmul_precision(request):
    """Both MLP GEMM precisions: "highest" -> fp32 MFMA, "high" -> 3 x bf16 split MFMA."""
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(request.param)
    yield request.param
    torch.set_float32_matmul_precision(old)


@pytest.mark.parametrize("name", ["barf", "n2v", "small"])
def test_nerf_model_golden(golden, name, matmul_precision):
    g = golden("model")
    m = _make_models()[name]
    # identical initial weights to the reference's th.manual_seed(0) construction
    for k, v in m.state_dict().items():
        ref = g[f"{name}.sdsum.{k}"]
        assert abs(v.double().sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), k
        assert abs(v.double().abs().sum().item() - ref[1]) <= 1e-9 * max(1.0, ref[1]), k
    m = m.to(DEV)
    pos = g2d(g["pos"]).requires_grad_(True)
    d = g2d(g["dir"])
    dens, rgb = m(pos, d, None, None, None)
    np.testing.assert_allclose(dens.detach().cpu().numpy(), g[f"{name}.density"], atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), g[f"{name}.rgb"], atol=1e-4, rtol=1e-4)
    ((dens * g2d(g[f"{name}.gd"])).sum() + (rgb * g2d(g[f"{name}.gc"])).sum()).backward()
    if matmul_precision == "highest":
        tol = 1e-4
        np.testing.assert_allclose(pos.grad.cpu().numpy(), g[f"{name}.dpos"], atol=10 * tol, rtol=10 * tol)
        for k, prm in m.named_parameters():
            s = g[f"{name}.gradsum.{k}"]
            assert abs(prm.grad.double().abs().sum().item() - s[1]) <= tol * s[1] + 1e-6, k
            key = f"{name}.grad.{k}"
            if key in g:
                np.testing.assert_allclose(prm.grad.cpu().numpy(), g[key],
                                           atol=tol * max(1.0, np.abs(g[key]).max()), rtol=10 * tol)
        return
    # split precision: a per-tensor conditioning bound.  Gradients of the deep first segment pass
    # ~10 ReLU masks whose pre-activations sit arbitrarily close to zero, so how far ANY finite
    # precision lands from the exact value differs per tensor, and mask flips make it non-linear in
    # the precision.  The CPU oracle (pinned to the reference by the "highest" branch above and
    # tests/test_oracle_golden.py) gives the exact (fp64) gradient, the spread of that exact gradient
    # when every weight is perturbed by a relative 2^-15 (the per-product error bound of three bf16
    # products; four random draws), and the reference's own fp32 error.  Each
    # tensor's split-precision error must stay within 2 x that spread + 2 x 2^9 x the fp32 error
    # (2^9 = 2^-15 / 2^-24; floored at fp32's well-conditioned 2^-22).
    exact = _oracle_model_grads(m, name, g, torch.float64)
    fp32 = _oracle_model_grads(m, name, g, torch.float32)
    spread = {k: torch.zeros(()) for k in exact}
    for seed in range(4):
        pert = _oracle_model_grads(m, name, g, torch.float64, perturb=(seed, 2.0 ** -15))
        for k in exact:
            spread[k] = torch.maximum(spread[k], (pert[k] - exact[k]).abs().max())
    got = {k: p.grad.double().cpu() for k, p in m.named_parameters()}
    got["dpos"] = pos.grad.double().cpu()
    for k, e in exact.items():
        scale = e.abs().max().item()
        if scale == 0:
            continue
        fp32_err = (fp32[k].double() - e).abs().max().item() / scale
        err = (got[k] - e).abs().max().item() / scale
        bound = 2 * spread[k].item() / scale + 2 * 2 ** 9 * max(fp32_err, 2 ** -22)
        assert err <= bound, (k, err, spread[k].item() / scale, fp32_err)


def _oracle_model_grads(m, name, g, dtype, perturb=None):
    """Parameter and position gradients of the golden NerfModel config by the CPU oracle in dtype;
    perturb = (seed, r): every weight and bias multiplied by (1 + U(-r, r)) first."""
    cfg = {"barf": (lambda x: O.barf_pe(x, 10, 10.0, True, 1.0), lambda x: O.barf_pe(x, 4, 4.0, True, 1.0),
                    2, 4, True, False),
           "n2v": (lambda x: O.fourier_features(x, 10, 2 * math.pi), lambda x: O.fourier_features(x, 4, 1.0),
                   2, 4, True, True),
           "small": (lambda x: O.barf_pe(x, 6, 3.4, True, 1.0), lambda x: O.barf_pe(x, 2, 1.5, False, 1.0),
                     3, 2, False, False)}[name]
    pe, de, nseg, nhid, dd, dden = cfg
    sd = {k: v.detach().cpu().to(dtype) for k, v in m.state_dict().items() if not k.endswith("alpha")}
    if perturb is not None:
        gen = torch.Generator().manual_seed(perturb[0])
        sd = {k: v * (1 + (torch.rand(v.shape, generator=gen, dtype=dtype) * 2 - 1) * perturb[1])
              for k, v in sd.items()}
    sd = {k: v.requires_grad_(True) for k, v in sd.items()}
    pos = torch.from_numpy(g["pos"]).to(dtype).requires_grad_(True)
    d = torch.from_numpy(g["dir"]).to(dtype)
    dens, rgb = O.nerf_model_forward(sd, pe(pos).to(dtype), de(d).to(dtype), nseg, nhid, dd, dden)
    ((dens * torch.from_numpy(g[f"{name}.gd"]).to(dtype)).sum()
     + (rgb * torch.from_numpy(g[f"{name}.gc"]).to(dtype)).sum()).backward()
    out = {k: v.grad.double() for k, v in sd.items()}
    out["dpos"] = pos.grad.double()
    return out


def test_compute_color_and_forward_golden(golden, matmul_precision):
    """_compute_color with explicit t and the coarse+fine forward with injected coarse t."""
    from nerf_amd import BarfPositionalEncoding, NerfInterpolation, NerfModel
    g = golden("color")
    torch.manual_seed(0)
    model = NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0),
                      BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0)).to(DEV)
    ren = NerfInterpolation(2.0, 8.0, model, 128, "stratified_uniform", 0.0, "middle", model, 64).to(DEV)
    o, d, pw, tc = g2d(g["o"]), g2d(g["d"]), g2d(g["pw"]), g2d(g["tc"])
    B = o.shape[0]
    t0, t1 = ren._get_intervals(tc)
    rgb, w, dist = ren._compute_color(model, t0, t1, o, d, pw, B, 64)
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), g["rgb"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(w.detach().cpu().numpy(), g["w"], atol=1e-4, rtol=0)
    ren._sample_t_stratified_uniform = lambda *a, **k: ren._get_intervals(tc.clone())
    rf, rc = ren(o, d, pw)
    np.testing.assert_allclose(rc.detach().cpu().numpy(), g["fwd_rgb_coarse"], atol=1e-4, rtol=0)
    # the fine t depends on floor() of the coarse weights: compare rays whose allocation is not
    # within MLP rounding of an integer boundary (all of them, for this fixture)
    np.testing.assert_allclose(rf.detach().cpu().numpy(), g["fwd_rgb_fine"], atol=2e-4, rtol=0)


@pytest.mark.parametrize("enc", ["barf", "ipe"])
def test_ray_gradients_fused_vs_reference_shaped(enc):
    """Pose refinement: gradients w.r.t. ray origins and directions.  The fused path (positions
    generated in the encoding kernel, nerf_encode_bwd_rays; direction encoding per ray) against
    the reference-shaped composition of the same kernels (positions and repeated directions in
    torch, NerfModel.forward, _render_rays — model_interpolation.py:288-414), fp32 GEMMs.  The
    ray gradients sum ~100 per-sample terms: 1e-4 relative to their scale."""
    from nerf_amd import (BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel)
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        torch.manual_seed(3)
        if enc == "barf":
            pe = BarfPositionalEncoding(10, 7.5, 0, 1, True, 1.0)
        else:
            pe = IntegratedBarfFourierFeatures(10, 7.5, 0, 1, True, 1.0, False)
            pe.pixel_width_sigma = 0.0
        model = NerfModel(4, 256, True, False, 2, pe, BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0)).to(DEV)
        S, B = 96, 64
        ren = NerfInterpolation(2.0, 8.0, model, S, "equidistant", 0.0, "middle").to(DEV)
        o = (torch.nn.functional.normalize(torch.randn(B, 3), dim=1) * 4).to(DEV)
        d = torch.nn.functional.normalize(-o.cpu() + torch.randn(B, 3) * 0.2, dim=1).to(DEV)
        pw = torch.full((B,), 1 / 555.56, device=DEV)
        t0, t1 = ren._sample_t_stratified_uniform(B, S, "equidistant", 0.0)
        gr = torch.randn(B, 3, device=DEV)
        of, df = o.clone().requires_grad_(True), d.clone().requires_grad_(True)
        rgb_f, _, _ = ren._compute_color(model, t0, t1, of, df, pw, B, S)
        (rgb_f * gr).sum().backward()
        og, dg = o.clone().requires_grad_(True), d.clone().requires_grad_(True)
        pos, dirs = ren._compute_positions(og, dg, t0, t1)
        n = B * S
        dens, col = model(pos.reshape(n, 3), dirs.reshape(n, 3), pw.repeat(1, S).view(n, 1), t0.reshape(n, 1),
                          t1.reshape(n, 1))
        rgb_g, _ = ren._render_rays(dens.view(B, S), col.view(B, S, 3), t1 - t0)
        (rgb_g * gr).sum().backward()
        np.testing.assert_allclose(rgb_f.detach().cpu().numpy(), rgb_g.detach().cpu().numpy(), atol=1e-5)
        for a, b in ((of.grad, og.grad), (df.grad, dg.grad)):
            assert a is not None and torch.isfinite(a).all()
            scale = float(b.abs().max())
            np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=1e-4 * scale, rtol=1e-4)
    finally:
        torch.set_float32_matmul_precision(old)


def test_fused_adam_matches_torch_adam():
    """FusedAdam (one nerf_adam_step launch) against torch.optim.Adam on the same parameters and
    gradients: two groups (different lr, one with weight decay), 6 steps, a LR change mid-way,
    a parameter without gradient.  fp32 update formula in torch's order: 1e-6 relative."""
    from nerf_amd import FusedAdam
    torch.manual_seed(21)
    shapes = [(256, 319), (256,), (3, 128), (4,), (1000, 7)]
    base = [torch.randn(s) for s in shapes]
    pf = [torch.nn.Parameter(b.clone().to(DEV)) for b in base]
    pt = [torch.nn.Parameter(b.clone().to(DEV)) for b in base]
    groups = lambda ps: [{"params": ps[:3], "lr": 5e-4}, {"params": ps[3:], "lr": 1e-3, "weight_decay": 0.01}]
    of = FusedAdam(groups(pf), eps=1e-5)
    ot = torch.optim.Adam(groups(pt), eps=1e-5)
    assert isinstance(of, torch.optim.Adam)
    for step in range(6):
        for i, (a, b) in enumerate(zip(pf, pt)):
            if i == 2 and step == 3:
                a.grad = b.grad = None          # skipped this step, as torch skips it
                continue
            g = torch.randn(a.shape, device=DEV) * (10.0 ** (i - 2))
            a.grad, b.grad = g.clone(), g.clone()
        if step == 4:
            for o in (of, ot):
                o.param_groups[0]["lr"] = 2e-4
        of.step()
        ot.step()
    for a, b in zip(pf, pt):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(), rtol=1e-6, atol=1e-7)
    sa, sb = of.state[pf[0]], ot.state[pt[0]]
    assert float(sa["step"]) == float(sb["step"]) == 6
    np.testing.assert_allclose(sa["exp_avg_sq"].cpu().numpy(), sb["exp_avg_sq"].cpu().numpy(), rtol=1e-6, atol=1e-12)


def test_training_steps_reduce_loss():
    from nerf_amd import FourierFeatures, NerfInterpolation, NerfModel
    torch.manual_seed(0)
    model = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0)).to(DEV)
    ren = NerfInterpolation(0.1, 1 / 3, model, 64, "stratified_uniform", density_factor=(3.0, 7.0)).to(DEV)
    opt = ren.configure_optimizers()["optimizer"]
    B = 1024
    o = (torch.nn.functional.normalize(torch.randn(B, 3), dim=1) * 0.168).to(DEV)
    d = torch.nn.functional.normalize(-o.cpu() + torch.randn(B, 3) * 0.1, dim=1).to(DEV)
    pw = torch.full((B,), 1 / 555.56, device=DEV)
    target = torch.full((B, 3), 0.3, device=DEV)   # learnable: a constant colour
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss, _ = ren.training_loss(o, d, pw, target)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert all(math.isfinite(x) for x in losses)
    assert losses[-1] < 0.3 * losses[0]
