"""Host-side logic that needs no GPU: MLP lowering, packing maps, encoder
bookkeeping, schedules, state_dict layout, and that the product path refuses
CPU tensors (no silent fallback)."""
import math

import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O


def _models():
    from nerf_amd import BarfPositionalEncoding, FourierFeatures, NerfModel
    torch.manual_seed(0)
    barf = NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0),
                     BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0))
    torch.manual_seed(0)
    n2v = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0))
    torch.manual_seed(0)
    small = NerfModel(2, 64, False, False, 3, BarfPositionalEncoding(6, 3.4, 0, 1, True, 1.0),
                      BarfPositionalEncoding(2, 1.5, 0, 1, False, 1.0))
    torch.manual_seed(0)
    flat = NerfModel(0, 32, False, True, 2, FourierFeatures(2, 1.0), FourierFeatures(1, 1.0))
    return {"barf": barf, "n2v": n2v, "small": small, "flat": flat}


@pytest.mark.parametrize("name", ["barf", "n2v", "small", "flat"])
def test_state_dict_layout_and_init_match_reference(golden, name):
    m = _models()[name]
    if name == "flat":
        assert [k for k in m.state_dict()] == ["model_segments.0.weight", "model_segments.0.bias",
                                              "model_segments.1.weight", "model_segments.1.bias",
                                              "model_color.0.weight", "model_color.0.bias",
                                              "model_color.2.weight", "model_color.2.bias"]
        return
    g = golden("model")
    keys = sorted(k.split(".sdsum.", 1)[1] for k in g if k.startswith(f"{name}.sdsum."))
    assert sorted(m.state_dict().keys()) == keys
    for k, v in m.state_dict().items():
        ref = g[f"{name}.sdsum.{k}"]
        assert abs(v.double().sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), k


@pytest.mark.parametrize("name", ["barf", "n2v", "small", "flat"])
def test_mlp_lowering(name):
    from nerf_amd.mlp import nerf_model_plan
    m = _models()[name]
    plan, z_last, head = nerf_model_plan(m.n_segments, m.model_segments, m.model_color, m.hidden_dim,
                                         m.position_encoder.output_dim, m.direction_encoder.output_dim,
                                         m.delayed_direction, m.delayed_density)
    linears = [mod for mod in m.modules() if isinstance(mod, torch.nn.Linear)]
    assert len(plan.layers) == len(linears)
    assert {id(lp.module) for lp in plan.layers} == {id(x) for x in linears}
    assert plan.outputs == [z_last, head] and head == len(plan.layers) - 1
    for i, lp in enumerate(plan.layers):
        lp.finalize("cpu")
        # the column map is a bijection onto the Linear's input columns
        cm = lp.col_map.tolist()
        assert sorted(c for c in cm if c >= 0) == list(range(lp.module.in_features))
        assert lp.Kp % 32 == 0 and lp.Kp == len(cm)
        # relu everywhere except the last layer of the last segment and the colour output
        assert lp.relu == (i not in (z_last, head))
    # the head reads z_last without its density column and the direction encoding (if delayed)
    srcs = plan.layers[head - 1].sources
    assert srcs[0].kind == "act" and srcs[0].layer == z_last and srcs[0].k_valid == m.hidden_dim
    assert (len(srcs) == 2) == m.delayed_direction
    # segment inputs follow the reference order [z, dir, pos]
    first = [lp for lp in plan.layers if any(s.kind == "pos" for s in lp.sources)]
    assert len(first) == m.n_segments
    for i, lp in enumerate(first):
        kinds = [s.kind for s in lp.sources]
        expect = (["act"] if i > 0 else []) + ([] if m.delayed_direction else ["dir"]) + ["pos"]
        assert kinds == expect


@pytest.mark.parametrize("name", ["radiance", "proposal"])
def test_garf_lowering_and_state_dict(golden, name):
    """GARF networks: reference key names and init (checksums), one plan layer per Linear, a
    Gaussian activation on every Linear followed by GaussAct, the z1 + z2 residual."""
    from nerf_amd.model_garf import GaussAct, ProposalNetwork, RadianceNetwork, strip_compile_prefix
    g = golden("garf")
    torch.manual_seed(0)
    m = (RadianceNetwork if name == "radiance" else ProposalNetwork)(0.5, 2.0, 5e-4, 5e-5, 0, 1.0, 0.0)
    keys = sorted(k.split(".sdsum.", 1)[1] for k in g if k.startswith(f"{name}.sdsum."))
    assert sorted(m.state_dict().keys()) == keys
    assert len(m.param_groups) == 2
    assert len(list(m.parameters_gaussian())) == sum(isinstance(x, GaussAct) for x in m.modules())
    plan = m._get_plan()
    linears = [x for x in m.modules() if isinstance(x, torch.nn.Linear)]
    assert [id(lp.module) for lp in plan.layers] == [id(x) for x in linears]
    n_gauss = sum(lp.gauss is not None for lp in plan.layers)
    assert n_gauss == len(list(m.parameters_gaussian()))
    assert len(plan.params()) == 2 * len(linears) + n_gauss
    for lp in plan.layers:
        lp.finalize("cpu")
        assert sorted(c for c in lp.col_map.tolist() if c >= 0) == list(range(lp.module.in_features))
    if name == "radiance":
        assert plan.outputs == [7, 9]
        assert plan.layers[7].residual == 3 and plan.layers[7].residual_cols == 128
        assert plan.layers[7].gauss is None and plan.layers[9].gauss is None
        assert [s.kind for s in plan.layers[4].sources] == ["act", "pos"]
        assert [s.kind for s in plan.layers[8].sources] == ["act", "dir"]
        assert plan.layers[8].sources[0].layer == 7 and plan.layers[8].sources[0].k_valid == 128
        assert plan.consumed[3] and plan.consumed[7]
    else:
        assert plan.outputs == [3]
    sd = {k.replace("model", "model._orig_mod", 1): v for k, v in m.state_dict().items()}
    assert strip_compile_prefix(sd).keys() == m.state_dict().keys()
    # garf's two-argument constructor (no learning rates): no param groups
    assert (RadianceNetwork if name == "radiance" else ProposalNetwork)(0.5, 2.0).param_groups == []


def test_col_map_follows_reference_concatenation():
    """Packed column j of a segment maps to the Linear input column of the same feature."""
    from nerf_amd.mlp import LayerPlan, Source
    lin = torch.nn.Linear(256 + 63, 256)
    lp = LayerPlan(lin, [Source("act", 256, 256, 0), Source("pos", 63, 64)], True)
    lp.finalize("cpu")
    cm = lp.col_map.tolist()
    assert cm[:256] == list(range(256)) and cm[256:319] == list(range(256, 319)) and cm[319] == -1


@pytest.mark.parametrize("alpha", [0.0, 0.5, 3.4, 9.99, 10.0, 12.0])
def test_barf_mask_values(alpha):
    from nerf_amd.positional_encodings import barf_mask_values
    assert barf_mask_values(alpha, 10) == O.barf_mask(alpha, 10).tolist()


def test_barf_alpha_schedule_and_state_dict():
    from nerf_amd import BarfPositionalEncoding
    enc = BarfPositionalEncoding(10, 1.0, 2.0, 6.0, True, 1.0)
    for epoch, want in ((0.0, 1.0), (2.0, 1.0), (4.0, 5.5), (6.0, 10.0), (100.0, 10.0)):
        enc.update_alpha(epoch)
        assert abs(enc._alpha_host - want) < 1e-6 and abs(float(enc.alpha) - want) < 1e-6
    enc2 = BarfPositionalEncoding(10, 0.0, 2.0, 6.0, True, 1.0)
    enc2.load_state_dict(enc.state_dict())
    assert enc2._alpha_host == enc._alpha_host
    assert enc.output_dim == 63 and enc.padded_dim == 64


def test_barf_alpha_direct_writes_refresh_the_mask():
    """Writes to the registered alpha buffer that bypass update_alpha (assignment, as the reference's
    own update_alpha does, and in-place fills) must reach the kernel's mask values."""
    import torch as th
    from nerf_amd import BarfPositionalEncoding
    enc = BarfPositionalEncoding(10, 0.0, 2.0, 6.0, True, 1.0)
    enc.alpha = th.tensor(3.4)
    assert enc.mask_values() == O.barf_mask(3.4, 10).tolist()
    enc.alpha.fill_(7.25)
    assert enc.mask_values() == O.barf_mask(7.25, 10).tolist()
    enc.update_alpha(100.0)
    assert enc.mask_values() == O.barf_mask(10.0, 10).tolist()


def test_barf_alpha_reassigned_twice_without_forward():
    """Two assignments with no mask read between them: the second tensor may reuse the first's
    freed id() at version 0, which an (id, version) check would take for the seen tensor."""
    import gc

    import torch as th
    from nerf_amd import BarfPositionalEncoding
    enc = BarfPositionalEncoding(10, 0.0, 2.0, 6.0, True, 1.0)
    assert enc.mask_values() == O.barf_mask(0.0, 10).tolist()
    for a in (2.5, 6.75, 1.25, 9.5):
        enc.alpha = th.tensor(a)
        enc.alpha = th.tensor(a + 0.125)
        gc.collect()
        assert enc.mask_values() == O.barf_mask(a + 0.125, 10).tolist()


def test_encoder_dims_and_errors():
    from nerf_amd import (FourierFeatures, IdentityPositionalEncoding, IntegratedBarfFourierFeatures,
                          IntegratedFourierFeatures)
    assert FourierFeatures(10).output_dim == 60 and FourierFeatures(4, 1.0).padded_dim == 32
    assert IdentityPositionalEncoding().output_dim == 3
    ipe = IntegratedFourierFeatures(10, 2 * math.pi, True, True)
    assert ipe.output_dim == 63
    with pytest.raises(TypeError):
        ipe._pe_params()          # pixel_width_sigma unset: the reference raises TypeError too
    ib = IntegratedBarfFourierFeatures(10, 0, 0, 1, False, 1.0, True)
    assert ib.output_dim == 60
    with pytest.raises(ValueError):
        FourierFeatures(4).encode_padded(torch.zeros(5, 2))


def test_product_path_refuses_cpu_tensors():
    from nerf_amd import FourierFeatures
    with pytest.raises(ValueError, match="ROCm device"):
        FourierFeatures(4)(torch.zeros(8, 3))


def test_scheduler_le_nice():
    from nerf_amd import SchedulerLeNice
    p = torch.nn.Parameter(torch.zeros(1))
    q = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([{"params": [p], "lr": 1e-3}, {"params": [q], "lr": 5e-4}], eps=1e-5)
    sch = SchedulerLeNice(opt, [1e-3, 5e-4], [1e-5, 5e-5], [100, 0])
    for _ in range(100):
        opt.step()
        sch.step()
    assert abs(opt.param_groups[0]["lr"] - 1e-5) < 1e-9
    assert abs(opt.param_groups[1]["lr"] - 5e-4) < 1e-12
    for _ in range(10):
        opt.step()
        sch.step()
    assert abs(opt.param_groups[0]["lr"] - 1e-5) < 1e-9


def test_renderer_param_groups_and_optimizer():
    from nerf_amd import NerfInterpolation
    m = _models()["barf"]
    ren = NerfInterpolation(2.0, 8.0, m, 128, "equidistant", -1.0, "middle", m, 64)
    assert len(ren.param_groups) == 2 and ren.proposal
    cfg = ren.configure_optimizers()
    assert isinstance(cfg["optimizer"], torch.optim.Adam) and cfg["optimizer"].defaults["eps"] == 1e-5
    assert cfg["lr_scheduler"]["interval"] == "step"
    with pytest.raises(ValueError):
        ren._get_t_query(torch.zeros(1), torch.zeros(1), "bogus")


def test_oracle_resample_fallback_flag():
    w = torch.rand(3, 64)
    w[1] = 0
    tc = torch.sort(torch.rand(3, 64), dim=1).values
    _, _, ok = O.sample_t_pdf_weighted(tc, w, torch.full((3, 64), 0.01), 128, 1.0, 0)
    assert not ok


def test_shard_rays_partition():
    from nerf_amd.ddp import shard_rays
    for n, w in ((4096, 8), (1000, 3), (5, 8)):
        idx = []
        for r in range(w):
            sl = shard_rays(n, r, w)
            idx += list(range(n))[sl]
        assert idx == list(range(n))


def test_camera_extrinsics_oracle_matches_reference(golden):
    """Oracle restatement of CameraExtrinsics.forward (barf/model_camera_extrinsics.py:7-85):
    refined origins / directions, rotations and parameter gradients vs the reference run."""
    from oracle import nerf_oracle as O
    g = golden("pose")
    rot = torch.from_numpy(g["rotation"]).requires_grad_()
    trans = torch.from_numpy(g["translation"]).requires_grad_()
    idx = torch.from_numpy(g["idx"])
    new_o, new_d, R, t = O.camera_extrinsics(rot, trans, idx, torch.from_numpy(g["o"]), torch.from_numpy(g["d"]))
    np.testing.assert_allclose(new_o.detach().numpy(), g["new_o"], atol=1e-6)
    np.testing.assert_allclose(new_d.detach().numpy(), g["new_d"], atol=1e-6)
    np.testing.assert_allclose(R.detach().numpy(), g["R"], atol=1e-6)
    ((new_o * torch.from_numpy(g["go"])).sum() + (new_d * torch.from_numpy(g["gd"])).sum()).backward()
    np.testing.assert_allclose(rot.grad.numpy(), g["drot"], atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(trans.grad.numpy(), g["dtrans"], atol=1e-5, rtol=1e-6)


def test_camera_extrinsics_module_api_and_no_cpu_path():
    """The module keeps the reference's parameters / param_groups; forward refuses host tensors."""
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    m = CameraExtrinsics(10, 1e-3, 1e-5, 100)
    assert [n for n, _ in m.named_parameters()] == ["rotation", "translation"]
    assert len(m.param_groups) == 1
    with pytest.raises(ValueError):
        m(torch.zeros(4, dtype=torch.int64), torch.zeros(4, 3), torch.zeros(4, 3))


def _emulate_fused(plan, fused, image_f64, x_pos, x_dir, dir_rd, relu_floor=True):
    """Lane-level numpy emulation of csrc/mlp_fused.hip over the packed image for ONE 16-sample
    column block: B operands built exactly as the kernel's registers (epilogue order), MFMA
    16x16x32 as D[i][s] += sum_{g,j} A[lane i+16g][j] * B[lane s+16g][j], 16-row output chunks."""
    lane = np.arange(64)
    s_of, g_of = lane & 15, lane >> 4
    j = np.arange(8)
    xreg = None                      # [KBMAX, 64 lanes, 8] register-fed B operand
    outs = []
    for idx, lp in enumerate(plan.layers):
        kbr, kbh, hbm, nb, n16, img_off, hbm_off, bias_off = fused.layers[idx]
        B = []
        for kb in range(kbr):
            B.append(xreg[kb])
        for s in hbm:
            t = x_pos if s.kind == "pos" else x_dir
            rd = 1 if s.kind == "pos" else dir_rd
            for kh in range(s.k_pad // 32):
                c = 32 * kh + 8 * g_of[:, None] + j[None, :]
                rows = (s_of // rd)[:, None]
                B.append(np.where(c < s.k_seg, t[rows, np.minimum(c, t.shape[1] - 1)], 0.0))
        N = lp.module.out_features
        out = np.zeros((16, 16 * n16))
        for c in range(n16):
            bias = image_f64["raw"][bias_off // 4 + 16 * c + np.arange(16)]
            acc = np.tile(bias[:, None], (1, 16))               # [i rows][s]
            for kb in range(kbr + kbh):
                if kb < kbr:
                    h0 = (img_off + (c * kbr + kb) * 2048) // 2
                else:
                    h0 = (hbm_off + (c * kbh + kb - kbr) * 2048) // 2
                frag = image_f64["w"][h0 + lane[:, None] * 8 + j[None, :]]   # hi + lo
                A = np.zeros((16, 32))
                Bm = np.zeros((32, 16))
                for g in range(4):
                    A[:, 8 * g:8 * g + 8] = frag[np.arange(16) + 16 * g]
                    Bm[8 * g:8 * g + 8, :] = B[kb][np.arange(16) + 16 * g].T
                acc += A @ Bm
            out[:, 16 * c:16 * c + 16] = acc.T
        if lp.relu:
            out = np.maximum(out, 0.0)
        outs.append(out[:, :N])
        # epilogue register order: xout[c] lane (s, g) element j <- row 32c + 16(j>>2) + 4g + (j&3)
        xreg = np.zeros((8, 64, 8))
        for c in range(min(nb, 8)):
            rows = 32 * c + 16 * (j[None, :] >> 2) + 4 * g_of[:, None] + (j[None, :] & 3)
            xreg[c] = np.pad(out, ((0, 0), (0, 32 * nb - out.shape[1])))[s_of[:, None], rows]
    return outs


@pytest.mark.parametrize("name", ["barf", "n2v"])
def test_fused_forward_image_emulation(name):
    """The packed image + lane permutations of the fused MLP forward reproduce NerfModel's
    forward (emulated on CPU; the kernel itself is checked by the GPU tests)."""
    from nerf_amd import mlp_fused
    from nerf_amd.mlp import nerf_model_plan
    m = _models()[name]
    pd, dd = m.position_encoder.output_dim, m.direction_encoder.output_dim
    plan, z_last, head = nerf_model_plan(m.n_segments, m.model_segments, m.model_color, m.hidden_dim, pd, dd,
                                         m.delayed_direction, m.delayed_density)
    plan.to_device(torch.device("cpu"))
    assert mlp_fused.eligible(plan, 4096)
    fused = mlp_fused.FusedForward(plan, torch.device("cpu"))
    # pack in numpy exactly as nerf_fused_pack does
    ps = []
    for lp in plan.layers:
        ps += [lp.module.weight.detach().double().numpy().ravel(), lp.module.bias.detach().double().numpy().ravel()]
    src = fused.map_src.numpy().astype(np.int64)
    dst = fused.map_dst.numpy().astype(np.int64)
    vals = np.zeros(src.shape[0])
    for t in range(len(ps)):
        sel = (src >= 0) & ((src >> 24) == t)
        vals[sel] = ps[t][src[sel] & 0xffffff]
    w = np.zeros(fused.image_bytes // 2)
    raw = np.zeros(fused.image_bytes // 4)
    hi = torch.from_numpy(vals).float().bfloat16().double().numpy()
    lo = torch.from_numpy(vals - hi).float().bfloat16().double().numpy()
    fr = dst >= 0
    w[dst[fr]] = hi[fr] + lo[fr]
    raw[~dst[~fr]] = vals[~fr]
    g = torch.Generator().manual_seed(3)
    S = 16
    x_pos = torch.rand(16, pd, generator=g).double().numpy() * 2 - 1
    x_dir = torch.rand(1, dd, generator=g).double().numpy() * 2 - 1
    x_pos = np.pad(x_pos, ((0, 0), (0, (-pd) % 4)))
    x_dir = np.pad(x_dir, ((0, 0), (0, (-dd) % 4)))
    outs = _emulate_fused(plan, fused, {"w": w, "raw": raw}, x_pos, x_dir, S)
    # reference: the Linear stack in fp64
    acts = []
    for idx, lp in enumerate(plan.layers):
        parts = []
        for s in lp.sources:
            if s.kind == "act":
                parts.append(acts[s.layer][:, :s.k_valid])
            elif s.kind == "pos":
                parts.append(x_pos[:, :s.k_valid])
            else:
                parts.append(np.repeat(x_dir[:, :s.k_valid], 16, axis=0))
        x = np.concatenate(parts, axis=1)
        y = x @ lp.module.weight.detach().double().numpy().T + lp.module.bias.detach().double().numpy()
        if lp.relu:
            y = np.maximum(y, 0.0)
        acts.append(y)
    for idx in range(len(plan.layers)):
        err = np.abs(outs[idx] - acts[idx]).max()
        assert err <= 1e-4 * max(1.0, np.abs(acts[idx]).max()), (idx, err)


def test_ray_feed_epoch_order_matches_torch_dataloader():
    """DeviceRayFeed's shuffled index order is the reference DataLoader's (shuffle=True with a
    seeded generator, data_module.py:202-209), epoch after epoch, whatever the batch size."""
    from torch.utils.data import DataLoader, Dataset

    from nerf_amd.ray_feed import dataloader_epoch_order

    class _Idx(Dataset):
        def __len__(self):
            return 77

        def __getitem__(self, i):
            return i

    for kw in (dict(batch_size=8), dict(batch_size=8, drop_last=True), dict(batch_size=77)):
        dl = DataLoader(_Idx(), shuffle=True, generator=torch.Generator().manual_seed(5), **kw)
        g = torch.Generator().manual_seed(5)
        for _ in range(3):
            got = torch.cat(list(dl))
            want = dataloader_epoch_order(77, g)
            assert torch.equal(got, want[:len(got)])


def test_ray_feed_blur_selection():
    """get_blurred_pixel_colors' case split (data_module.py:324-365)."""
    from nerf_amd.ray_feed import blur_selection
    sig = [8.0, 4.0, 2.0, 0.0]
    assert blur_selection(sig, 0.1)[0] == 1
    assert blur_selection(sig, 8.0)[0] == 2
    mode, lo, hi, a, b = blur_selection(sig, 3.0)
    assert (mode, lo, hi) == (3, 1, 2)
    assert abs(a - (3.0 - 2.0) / (4.0 - 2.0 + 1e-8)) < 1e-12 and abs(a + b - 1) < 1e-12


def test_lightning_style_mixin():
    """INTEGRATION.md's Lightning recipe: the renderer mixed with a LightningModule-like base
    (stand-in: pytorch_lightning is not installed) constructs once, keeps the reference's
    attributes and hands the trainer FusedAdam + SchedulerLeNice."""
    import torch.nn as nn
    from nerf_amd import FourierFeatures, NerfModel
    from nerf_amd.model_interpolation import NerfInterpolation as _Renderer, SchedulerLeNice
    from nerf_amd.optim import FusedAdam

    class LightningModule(nn.Module):              # what the recipe relies on of pl.LightningModule
        inits = 0

        def __init__(self):
            super().__init__()
            LightningModule.inits += 1
            self.logged = {}

        def log_dict(self, d, **kw):
            self.logged.update(d)

    class NerfInterpolation(_Renderer, LightningModule):
        def training_step(self, batch, batch_idx):
            return self._step_helper(batch, batch_idx, "train")

    class BarfLike(NerfInterpolation):             # an experiment's subclass, unchanged
        def _step_helper(self, batch, batch_idx, purpose):
            self.log_dict({f"{purpose}_called": 1.0})
            return batch_idx

    torch.manual_seed(0)
    model = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 6.28), FourierFeatures(4, 1.0))
    m = BarfLike(2.0, 8.0, model, 64)
    assert LightningModule.inits == 1
    assert m.training_step(None, 7) == 7 and m.logged == {"train_called": 1.0}
    opt = m.configure_optimizers()
    # torch Adam for host parameters, its FusedAdam subclass once the model is on the GPU
    assert isinstance(opt["optimizer"], torch.optim.Adam) and issubclass(FusedAdam, torch.optim.Adam)
    assert isinstance(opt["lr_scheduler"]["scheduler"], SchedulerLeNice)
    assert [n for n, _ in m.named_parameters()][0].startswith("model_radiance.")
