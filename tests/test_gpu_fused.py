"""Fused field-MLP forward (csrc/mlp_fused.hip, one launch for the whole NerfModel) against
the layer-by-layer split-precision path it replaces (mlp.py, pinned to the reference's golden
vectors by test_gpu_parity.py) on the same inputs, and against the CPU oracle on a subset.

Every layer output (these are the backward's saved activations), the density column and the
ReLU mask bits are compared.  Tolerance: 1e-4 of the layer's max |value| (both paths form each
product with ~2^-17 relative error, in different summation orders); mask bits must agree
wherever the activation is not within 1e-5 of the max of zero.  Sizes: BASELINE's 4096 x 64
samples, a ragged M (not a multiple of the 64-sample tile), the per-ray direction rows of the
ray-mode encoder, and one-tile batches."""
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
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    yield
    torch.set_float32_matmul_precision(prev)


def _model(name):
    from nerf_amd import BarfPositionalEncoding, FourierFeatures, NerfModel
    torch.manual_seed(0)
    if name == "n2v":
        return NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0))
    return NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0),
                     BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0))


def _run(model, pos_pe, dir_pe, rd, fused):
    from nerf_amd import mlp, mlp_fused
    from nerf_amd.mlp import MLPFunction
    plan = model._get_plan()
    saved = mlp_fused.ENABLED
    mlp_fused.ENABLED = fused
    mlp.CAPTURE = []
    try:
        outs = MLPFunction.apply(plan, pos_pe.shape[0], pos_pe, dir_pe, rd, *plan.params())
        torch.cuda.synchronize()
        acts, masks = mlp.CAPTURE[0]
    finally:
        mlp_fused.ENABLED = saved
        mlp.CAPTURE = None
    assert len(acts) == len(plan.layers)
    return outs, acts, masks, plan


@pytest.mark.parametrize("name,M,rd", [("n2v", 4096 * 64, 64), ("n2v", 1000, 1), ("barf", 4096 * 8 + 37, 1),
                                       ("barf", 64, 64), ("n2v", 3 * 64 + 5, 1)])
def test_fused_forward_matches_layerwise(name, M, rd):
    from nerf_amd import mlp_fused
    model = _model(name).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(11)
    pd = model.position_encoder.output_dim
    dd = model.direction_encoder.output_dim
    pos_pe = torch.zeros(M, (pd + 31) // 32 * 32, device=DEV)
    pos_pe[:, :pd] = torch.rand(M, pd, device=DEV, generator=g) * 2 - 1
    nd = (M + rd - 1) // rd
    dir_pe = torch.zeros(nd, (dd + 31) // 32 * 32, device=DEV)
    dir_pe[:, :dd] = torch.rand(nd, dd, device=DEV, generator=g) * 2 - 1
    plan = model._get_plan()
    plan.to_device(torch.device(DEV))
    assert mlp_fused.eligible(plan, M)
    o_ref, a_ref, m_ref, _ = _run(model, pos_pe, dir_pe, rd, False)
    o_fus, a_fus, m_fus, _ = _run(model, pos_pe, dir_pe, rd, True)
    assert len(o_ref) == len(o_fus)
    errs = []
    for li, (x, y) in enumerate(zip(a_ref, a_fus)):
        n = plan.layers[li].N
        scale = max(1.0, x[:, :n].abs().max().item())
        err = (x[:, :n] - y[:, :n]).abs().max().item()
        bad = ((x[:, :n] - y[:, :n]).abs() > 1e-4 * scale).nonzero()
        errs.append((li, err, scale, bad[:4].tolist(), int(bad.shape[0])))
    for li, err, scale, bad, nbad in errs:
        assert err <= 1e-4 * scale, errs
        # padding columns of the output rows are zero in the fused path
        if y.shape[1] > n:
            assert (y[:, n:] == 0).all()
    widths = [plan.layers[i].N for i in plan.outputs] + [1] * len(plan.column_outputs)
    for x, y, n in zip(o_ref, o_fus, widths):
        x, y = x.reshape(x.shape[0], -1)[:, :n], y.reshape(y.shape[0], -1)[:, :n]   # padding columns: unspecified
        scale = max(1.0, x.abs().max().item())
        assert (x - y).abs().max().item() <= 1e-4 * scale
    # inference (no autograd): the kernel stores only the exposed outputs; same bits
    from nerf_amd.mlp import MLPFunction
    with torch.no_grad():
        o_inf = MLPFunction.apply(plan, M, pos_pe, dir_pe, rd, *plan.params())
    for x, y, n in zip(o_fus, o_inf, widths):
        assert torch.equal(x.reshape(x.shape[0], -1)[:, :n], y.reshape(y.shape[0], -1)[:, :n])
    for li, (ma, mb) in enumerate(zip(m_ref, m_fus)):
        assert (ma is None) == (mb is None)
        if ma is None:
            continue
        n = plan.layers[li].N
        # both layouts mapped to columns: NERF_EPI_MASKOUT (layer by layer) and NERF_FUSED_MASK
        bits_a = np.unpackbits(ma.cpu().numpy(), axis=1, bitorder="little")[:, _maskout_order()]
        bits_b = 1 - np.unpackbits(mb.cpu().numpy(), axis=1, bitorder="little")[:, _fused_mask_order()]   # dead bits
        act = a_ref[li][:, :n].cpu().numpy()
        near0 = np.abs(act) <= 1e-5 * max(1.0, np.abs(act).max())
        diff = (bits_a[:, :n] != bits_b[:, :n]) & ~near0
        assert not diff.any(), (li, int(diff.sum()))
        # and the bits are the activations' signs (away from zero)
        sign = act > 0
        assert not ((bits_b[:, :n] != sign) & ~near0).any()


def _maskout_order():
    """row bit index of column n in the NERF_EPI_MASKOUT layout: bit b of word 2e+h <-> column 4(32h+b)+e"""
    order = np.empty(256, dtype=np.int64)
    for w in range(8):
        e, h = w // 2, w % 2
        for b in range(32):
            order[4 * (32 * h + b) + e] = 32 * w + b
    return order


def _fused_mask_order():
    """row bit index of column n in the NERF_FUSED_MASK layout (include/nerf_amd.h): column
    16 c + 4 g + r is bit 4 (7 - (c & 7)) + r of word 2 g + (c >> 3) (set: a dead unit)"""
    order = np.empty(256, dtype=np.int64)
    for c in range(16):
        for g in range(4):
            for r in range(4):
                order[16 * c + 4 * g + r] = 32 * (2 * g + (c >> 3)) + 4 * (7 - (c & 7)) + r
    return order


def test_mask_layout_orders_are_permutations():
    assert sorted(_maskout_order().tolist()) == list(range(256))
    assert sorted(_fused_mask_order().tolist()) == list(range(256))


def test_fused_forward_vs_oracle_subset():
    """Fused NerfModel forward (n2v config) against the CPU oracle on 512 rows."""
    model = _model("n2v")
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(DEV)
    g = torch.Generator().manual_seed(5)
    M = 64 * 512
    x = torch.rand(M, 3, generator=g) * 2 - 1
    d = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=1)
    from nerf_amd import mlp_fused
    assert mlp_fused.ENABLED
    dens, rgb = model(x.to(DEV), d.to(DEV), None, None, None)
    idx = torch.arange(0, M, 61)
    pe = O.fourier_features(x[idx], 10, 2 * math.pi)
    de = O.fourier_features(d[idx], 4, 1.0)
    od, oc = O.nerf_model_forward(sd, pe, de, 2, 4, True, True)
    assert (dens.cpu()[idx] - od).abs().max().item() < 2e-4
    assert (rgb.cpu()[idx] - oc).abs().max().item() < 2e-4


@pytest.mark.parametrize("fused", [True, False])
def test_weight_updates_outside_autograd_reach_the_kernels(fused):
    """p.data updates do not bump a parameter's version counter; the packed weight images must
    still follow them: after p.data.add_, the fused and layer-by-layer forwards equal a
    fresh model built from the updated state_dict."""
    model = _model("n2v").to(DEV)
    g = torch.Generator().manual_seed(9)
    M = 2048
    pe = torch.rand(M, 64, generator=g).to(DEV)
    pe[:, 60:] = 0
    de = torch.rand(M // 64, 32, generator=g).to(DEV)
    de[:, 24:] = 0
    _run(model, pe, de, 64, fused)                       # packs the images once
    with torch.no_grad():
        for p in model.parameters():
            p.data.add_(0.01 * torch.randn(p.shape, generator=g).to(DEV))
    outs, acts, _, _ = _run(model, pe, de, 64, fused)
    fresh = _model("n2v").to(DEV)
    fresh.load_state_dict(model.state_dict())
    outs2, acts2, _, _ = _run(fresh, pe, de, 64, fused)
    for a, b in zip(acts, acts2):
        assert torch.equal(a, b)


def _fp64_param_grads(pos_pe, dir_pe, rd, w_out):
    """fp64 torch reference of the same NerfModel plan (dense cat + linear + ReLU)."""
    model = _model("n2v").to(DEV).double()
    plan = model._get_plan()
    acts = []
    pe64, de64 = pos_pe.double(), dir_pe.double().repeat_interleave(rd, dim=0)[:pos_pe.shape[0]]
    for lp in plan.layers:
        parts = []
        for s in lp.sources:
            src = acts[s.layer] if s.kind == "act" else (pe64 if s.kind == "pos" else de64)
            parts.append(src[:, :s.k_valid])
        y = torch.nn.functional.linear(torch.cat(parts, 1), lp.module.weight, lp.module.bias)
        acts.append(torch.relu(y) if lp.relu else y)
    (acts[-1][:, :4] * w_out.double()).sum().backward()
    return {n: p.grad.detach() for n, p in model.named_parameters()}


@pytest.mark.parametrize("M,rd", [(4096 * 64, 64), (1000, 1), (3 * 64 + 5, 1)])
def test_fused_input_gradient_chain_matches_layerwise(M, rd):
    """The backward's input-gradient chain in one launch (n2v NerfModel: only the head output
    feeds the loss, no encoding gradients): every parameter gradient against an fp64 reference,
    as accurate as the layer-by-layer backward it replaces: both paths' errors are 1e-3..9e-3 of
    the tensor's max |gradient| (split precision through ~10 ReLU layers whose masks flip under
    2^-17 perturbations; ~2e-2 for the encoding gradients at the bottom of the
    chain), so the bound is the layerwise error + 1e-2 and < 5e-2
    (an indexing or routing error shows as O(0.1..1))."""
    from nerf_amd import mlp_fused
    from nerf_amd.mlp import MLPFunction
    g = torch.Generator(device=DEV).manual_seed(7)
    pos_pe = torch.zeros(M, 64, device=DEV)
    pos_pe[:, :60] = torch.rand(M, 60, device=DEV, generator=g) * 2 - 1
    nd = (M + rd - 1) // rd
    dir_pe = torch.zeros(nd, 32, device=DEV)
    dir_pe[:, :24] = torch.rand(nd, 24, device=DEV, generator=g) * 2 - 1
    w_out = torch.randn(M, 4, device=DEV, generator=g)
    grads = {}
    for fused in (False, True):
        model = _model("n2v").to(DEV)
        plan = model._get_plan()
        saved = mlp_fused.ENABLED
        mlp_fused.ENABLED = fused
        runs = mlp_fused.FusedInputGrad.runs
        try:
            outs = MLPFunction.apply(plan, M, pos_pe, dir_pe, rd, *plan.params())
            (outs[1][:, :4] * w_out).sum().backward()
            torch.cuda.synchronize()
        finally:
            mlp_fused.ENABLED = saved
        assert (mlp_fused.FusedInputGrad.runs > runs) == fused
        grads[fused] = {n: p.grad.detach().double() for n, p in model.named_parameters()}
    ref = _fp64_param_grads(pos_pe, dir_pe, rd, w_out)
    for n, r in ref.items():
        scale = max(r.abs().max().item(), 1e-12)
        e_layer = (grads[False][n] - r).abs().max().item() / scale
        e_fused = (grads[True][n] - r).abs().max().item() / scale
        assert e_fused <= e_layer + 1e-2 and e_fused < 5e-2, (n, e_fused, e_layer)


def test_fused_forward_with_layerwise_backward(monkeypatch):
    """A fused forward whose backward cannot run the chain (forced here) takes the layer-by-layer
    input-gradient GEMMs: they must not read the fused NERF_FUSED_MASK bits as NERF_EPI_MASKOUT
    words (mlp.py uses the stored activations instead).  Gradients against the all-layerwise
    run and fp64 (bound as in the chain test above)."""
    from nerf_amd import mlp_fused
    from nerf_amd.mlp import MLPFunction
    M, rd = 4096 * 4 + 7, 1
    g = torch.Generator(device=DEV).manual_seed(17)
    pos_pe = torch.zeros(M, 64, device=DEV)
    pos_pe[:, :60] = torch.rand(M, 60, device=DEV, generator=g) * 2 - 1
    dir_pe = torch.zeros(M, 32, device=DEV)
    dir_pe[:, :24] = torch.rand(M, 24, device=DEV, generator=g) * 2 - 1
    w_out = torch.randn(M, 4, device=DEV, generator=g)
    monkeypatch.setattr(mlp_fused, "dgrad_eligible", lambda plan, M: False)
    grads = {}
    for fused in (False, True):
        model = _model("n2v").to(DEV)
        plan = model._get_plan()
        saved = mlp_fused.ENABLED
        mlp_fused.ENABLED = fused
        runs = mlp_fused.FusedInputGrad.runs
        try:
            outs = MLPFunction.apply(plan, M, pos_pe, dir_pe, rd, *plan.params())
            (outs[1][:, :4] * w_out).sum().backward()
            torch.cuda.synchronize()
        finally:
            mlp_fused.ENABLED = saved
        assert mlp_fused.FusedInputGrad.runs == runs
        grads[fused] = {n: p.grad.detach().double() for n, p in model.named_parameters()}
    ref = _fp64_param_grads(pos_pe, dir_pe, rd, w_out)
    for n, r in ref.items():
        scale = max(r.abs().max().item(), 1e-12)
        e_layer = (grads[False][n] - r).abs().max().item() / scale
        e_fused = (grads[True][n] - r).abs().max().item() / scale
        assert e_fused <= e_layer + 1e-2 and e_fused < 5e-2, (n, e_fused, e_layer)


def test_fused_input_gradient_chain_density_column():
    """mip / barf-shaped NerfModel without delayed density: the density column's gradient joins
    the chain as an HBM-fed k-block; parameter gradients against the layer-by-layer backward and
    fp64 (tolerance as above)."""
    from nerf_amd import mlp_fused
    from nerf_amd.mlp import MLPFunction
    M, rd = 4096 * 16 + 3, 1
    g = torch.Generator(device=DEV).manual_seed(9)
    pos_pe = torch.zeros(M, 64, device=DEV)
    pos_pe[:, :63] = torch.rand(M, 63, device=DEV, generator=g) * 2 - 1
    dir_pe = torch.zeros(M, 32, device=DEV)
    dir_pe[:, :27] = torch.rand(M, 27, device=DEV, generator=g) * 2 - 1
    w_rgb = torch.randn(M, 3, device=DEV, generator=g)
    w_sig = torch.randn(M, device=DEV, generator=g)
    grads = {}
    for fused in (False, True):
        model = _model("barf").to(DEV)
        plan = model._get_plan()
        saved = mlp_fused.ENABLED
        mlp_fused.ENABLED = fused
        runs = mlp_fused.FusedInputGrad.runs
        try:
            outs = MLPFunction.apply(plan, M, pos_pe, dir_pe, rd, *plan.params())
            ((outs[1][:, :3] * w_rgb).sum() + (outs[2] * w_sig).sum()).backward()
            torch.cuda.synchronize()
        finally:
            mlp_fused.ENABLED = saved
        assert (mlp_fused.FusedInputGrad.runs > runs) == fused
        grads[fused] = {n: p.grad.detach().double() for n, p in model.named_parameters()}
    # fp64 reference
    model = _model("barf").to(DEV).double()
    plan = model._get_plan()
    acts = []
    for lp in plan.layers:
        parts = []
        for s in lp.sources:
            src = acts[s.layer] if s.kind == "act" else (pos_pe.double() if s.kind == "pos" else dir_pe.double())
            parts.append(src[:, :s.k_valid])
        y = torch.nn.functional.linear(torch.cat(parts, 1), lp.module.weight, lp.module.bias)
        acts.append(torch.relu(y) if lp.relu else y)
    z_last, head = plan.outputs
    ((acts[head][:, :3] * w_rgb.double()).sum() + (acts[z_last][:, 256] * w_sig.double()).sum()).backward()
    for n, p in model.named_parameters():
        r = p.grad.detach()
        scale = max(r.abs().max().item(), 1e-12)
        e_layer = (grads[False][n] - r).abs().max().item() / scale
        e_fused = (grads[True][n] - r).abs().max().item() / scale
        assert e_fused <= e_layer + 1e-2 and e_fused < 5e-2, (n, e_fused, e_layer)


@pytest.mark.parametrize("rd", [1, 128])
def test_fused_input_gradient_chain_encoding_grads(rd):
    """BARF pose refinement: the chain also returns the gradients w.r.t. the position and
    (per-ray) direction encodings (second kernel output, summed over layers / rays on the host).
    Against the layer-by-layer backward and fp64 (tolerance as above)."""
    from nerf_amd import mlp_fused
    from nerf_amd.mlp import MLPFunction
    M = 128 * 300 + (0 if rd > 1 else 5)
    g = torch.Generator(device=DEV).manual_seed(13)
    base_pos = torch.zeros(M, 64, device=DEV)
    base_pos[:, :63] = torch.rand(M, 63, device=DEV, generator=g) * 2 - 1
    nd = (M + rd - 1) // rd
    base_dir = torch.zeros(nd, 32, device=DEV)
    base_dir[:, :27] = torch.rand(nd, 27, device=DEV, generator=g) * 2 - 1
    w_rgb = torch.randn(M, 3, device=DEV, generator=g)
    w_sig = torch.randn(M, device=DEV, generator=g)
    res = {}
    for fused in (False, True):
        model = _model("barf").to(DEV)
        plan = model._get_plan()
        pos_pe = base_pos.clone().requires_grad_(True)
        dir_pe = base_dir.clone().requires_grad_(True)
        saved = mlp_fused.ENABLED
        mlp_fused.ENABLED = fused
        runs = mlp_fused.FusedInputGrad.runs
        try:
            outs = MLPFunction.apply(plan, M, pos_pe, dir_pe, rd, *plan.params())
            ((outs[1][:, :3] * w_rgb).sum() + (outs[2] * w_sig).sum()).backward()
            torch.cuda.synchronize()
        finally:
            mlp_fused.ENABLED = saved
        assert (mlp_fused.FusedInputGrad.runs > runs) == fused
        res[fused] = {n: p.grad.detach().double() for n, p in model.named_parameters()}
        res[fused]["pos"] = pos_pe.grad.detach().double()
        res[fused]["dir"] = dir_pe.grad.detach().double()
    model = _model("barf").to(DEV).double()
    plan = model._get_plan()
    p64 = base_pos.double().requires_grad_(True)
    d64 = base_dir.double().requires_grad_(True)
    dexp = d64.repeat_interleave(rd, dim=0)[:M]
    acts = []
    for lp in plan.layers:
        parts = []
        for s in lp.sources:
            src = acts[s.layer] if s.kind == "act" else (p64 if s.kind == "pos" else dexp)
            parts.append(src[:, :s.k_valid])
        y = torch.nn.functional.linear(torch.cat(parts, 1), lp.module.weight, lp.module.bias)
        acts.append(torch.relu(y) if lp.relu else y)
    z_last, head = plan.outputs
    ((acts[head][:, :3] * w_rgb.double()).sum() + (acts[z_last][:, 256] * w_sig.double()).sum()).backward()
    ref = {n: p.grad.detach() for n, p in model.named_parameters()}
    ref["pos"] = p64.grad.detach()
    ref["dir"] = d64.grad.detach()
    for n, r in ref.items():
        scale = max(r.abs().max().item(), 1e-12)
        e_layer = (res[False][n] - r).abs().max().item() / scale
        e_fused = (res[True][n] - r).abs().max().item() / scale
        assert e_fused <= e_layer + 1e-2 and e_fused < 5e-2, (n, e_fused, e_layer)
