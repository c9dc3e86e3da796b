"""Generate golden input/output vectors by running the REFERENCE implementation.

Runs only in the build container, where the read-only reference checkout is at
/root/reference (override with NERF_REFERENCE).  The reference source never
leaves that directory: this script imports it (with two import stubs for the
absent pytorch_lightning / data modules), evaluates it on seeded inputs and
writes plain arrays (inputs and expected outputs) to tests/golden/*.npz.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Fixtures:
  pe.npz         FourierFeatures / BarfPositionalEncoding (+ d/dx) / IntegratedFourierFeatures /
                 IntegratedBarfFourierFeatures / mip_NeRF IntegratedFourierFeatures outputs
  composite.npz  NerfInterpolation._render_rays outputs and input gradients
  resample.npz   _sample_t_pdf_weighted (barf) and _sample_t_fine (naive-to-vanilla) outputs
  model.npz      NerfModel (barf config and naive-to-vanilla config): weights, inputs, outputs, gradients
  color.npz      _compute_color end to end with explicit t, and forward coarse+fine with injected t
  cos_kat.npz    barf/cos_test_barf.pt (the reference's own fixture, loaded weights_only)
  ipe_grad.npz   integrated encodings: outputs and gradients w.r.t. position and direction
  garf.npz       GARF RadianceNetwork / ProposalNetwork / GaussAct: checksummed init, outputs, gradients
  pose.npz       CameraExtrinsics (BARF pose refinement): refined rays, rotations, parameter gradients
  pose_render.npz CameraExtrinsics -> NerfInterpolation._compute_color -> backward: rgb and the pose
                 parameters' gradients through the whole rendering path (BarfModel's training input)
  mipnerf.npz    mip_NeRF API: IntegratedFourierFeatures (both variance modes), MipNerfModel forward /
                 gradients, MipNerf coarse+fine forward with injected coarse t
  nerf2d.npz     2d-reconstruction Nerf2d (C1): init, Fourier features, forward, loss, gradients, 3 Adam steps
  hashgrid2d.npz 2d-ingp INGPTable / INGPEncoding (the readable copy of the hash grid): tables, indices, weights, output
  kabsch.npz     CameraCalibrationModel.kabsch_algorithm (outlier removal on / off) and compute_pose_error
  feed.npz       ImagePoseDataset rays + __getitem__ (DataLoader collation) + get_blurred_pixel_colors
                 on a small in-memory image set; the notebook's 4x2 meshgrid known answer

    python tests/golden/make_golden.py [pe composite resample model color cos_kat ipe_grad garf pose]
"""
from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np
import torch as th

REF = os.environ.get("NERF_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    pl = types.ModuleType("pytorch_lightning")

    class LightningModule(th.nn.Module):
        def save_hyperparameters(self, *a, **k):
            pass

        @property
        def device(self):
            return th.device("cpu")

        def log_dict(self, *a, **k):
            pass

    pl.LightningModule = LightningModule
    sys.modules["pytorch_lightning"] = pl
    for name in ("data_module", "dataset"):
        m = types.ModuleType(name)
        m.DatasetOutput = tuple
        m.ImagePoseDataModule = object
        sys.modules[name] = m
    # dataset.py imports torchvision at module level (used only by its image loader, which the
    # feed fixture never calls); pytorch_lightning.callbacks for data_module.py
    sys.modules.setdefault("torchvision", types.ModuleType("torchvision"))
    cb = types.ModuleType("pytorch_lightning.callbacks")
    cb.LambdaCallback = object
    sys.modules["pytorch_lightning.callbacks"] = cb
    pl.callbacks = cb
    pl.LightningDataModule = object
    pl.Trainer = object


def _import_from(subdir: str, names: list[str]):
    """Import reference modules from one experiment directory (bare-name imports)."""
    for n in names + ["model_interpolation_architecture", "positional_encodings", "model_interpolation", "magic"]:
        sys.modules.pop(n, None)
    sys.path.insert(0, os.path.join(REF, subdir))
    try:
        return [importlib.import_module(n) for n in names]
    finally:
        sys.path.pop(0)


def f32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def gen_pe():
    (pe,) = _import_from("barf", ["positional_encodings"])
    g = th.Generator().manual_seed(1)
    N = 257
    x = (th.rand(N, 3, generator=g) * 16 - 8)
    d = th.randn(N, 3, generator=g)
    d = d / th.linalg.vector_norm(d, dim=1, keepdim=True)
    t0 = 2 + th.rand(N, 1, generator=g) * 6
    t1 = t0 + th.rand(N, 1, generator=g) * 0.1 + 1e-3
    out = {"x": f32(x), "dir": f32(d), "t0": f32(t0), "t1": f32(t1)}
    out["fourier_L10_2pi"] = f32(pe.FourierFeatures(10, 2 * th.pi).forward(x))
    out["fourier_L4_1"] = f32(pe.FourierFeatures(4, 1.0).forward(d))
    for alpha in (0.0, 3.4, 10.0):
        for ident in (True, False):
            for scale, sname in ((1.0, "1"), (2 * th.pi, "2pi")):
                enc = pe.BarfPositionalEncoding(10, alpha, 0, 1, ident, scale)
                xx = x.clone().requires_grad_(True)
                y = enc.forward(xx)
                gy = th.randn(y.shape, generator=g)
                (y * gy).sum().backward()
                key = f"barf_L10_a{alpha}_id{int(ident)}_s{sname}"
                out[key] = f32(y)
                out[key + "_gy"] = f32(gy)
                out[key + "_dx"] = f32(xx.grad)
    enc = pe.BarfPositionalEncoding(10, 0.0, 10.0, 20.0, True, 1.0)
    enc.update_alpha(13.7)
    out["barf_update_alpha_13.7"] = np.array([float(enc.alpha)], np.float32)
    out["barf_mask_a3.4"] = f32(pe.BarfPositionalEncoding(10, 3.4, 0, 1, True, 1.0).compute_mask(th.tensor(3.4)))
    for pw, pwname in ((1 / 555.56, "400"), (1 / 1111.1, "800")):
        pwt = th.full((N, 1), pw)
        out[f"pw_{pwname}"] = f32(pwt)
        for dv in (True, False):
            for pws in (0.0, 0.5):
                enc = pe.IntegratedFourierFeatures(10, 2 * th.pi, True, dv)
                enc.pixel_width_sigma = pws
                out[f"ipe_{pwname}_dv{int(dv)}_pws{pws}"] = f32(enc.forward(x, d, pwt, t0, t1))
        enc = pe.IntegratedBarfFourierFeatures(10, 3.4, 0, 1, True, 1.0, True)
        enc.pixel_width_sigma = 0.0
        out[f"ipebarf_{pwname}_a3.4"] = f32(enc.forward(x, d, pwt, t0, t1))
    # older mip_NeRF variant: no identity, scale 2*pi, (pos, dir, t_start, t_end, pixel_width) order
    (mm,) = _import_from("mip_NeRF", ["mip_model"])
    enc = mm.IntegratedFourierFeatures(10, 2 * th.pi, True)
    out["mipnerf_ipe_800"] = f32(enc.forward(x, d, t0, t1, 1 / 1111.1))
    np.savez_compressed(os.path.join(OUT, "pe.npz"), **out)


def gen_composite():
    (mi,) = _import_from("barf", ["model_interpolation"])
    g = th.Generator().manual_seed(2)
    out = {}
    for S in (64, 128, 192):
        B = 48
        sig = th.nn.functional.softplus(th.randn(B, S, generator=g) * 4)
        col = th.rand(B, S, 3, generator=g)
        t = th.sort(2 + th.rand(B, S, generator=g) * 6, dim=1).values
        dist = th.diff(t, dim=1, append=th.full((B, 1), 8.0))
        model = mi.NerfInterpolation.__new__(mi.NerfInterpolation)
        th.nn.Module.__init__(model)
        sig_ = sig.clone().requires_grad_(True)
        col_ = col.clone().requires_grad_(True)
        rgb, w = model._render_rays(sig_, col_, dist)
        grgb = th.randn(B, 3, generator=g)
        gw = th.randn(B, S, generator=g)
        ((rgb * grgb).sum() + (w * gw).sum()).backward()
        k = f"S{S}"
        out.update({f"{k}_sigma": f32(sig), f"{k}_color": f32(col), f"{k}_dist": f32(dist), f"{k}_rgb": f32(rgb),
                    f"{k}_w": f32(w), f"{k}_grgb": f32(grgb), f"{k}_gw": f32(gw), f"{k}_dsigma": f32(sig_.grad),
                    f"{k}_dcolor": f32(col_.grad)})
    np.savez_compressed(os.path.join(OUT, "composite.npz"), **out)


def _weights_suite(g, B, K):
    w = th.nn.functional.softplus(th.randn(B, K, generator=g) * 3) * (th.rand(B, K, generator=g) < 0.7)
    w = w / (w.sum(1, keepdim=True) + 1e-3)
    w[0] = 0
    w[0, 5] = 1.0                      # one-hot
    w[1] = 1.0 / K                     # uniform: every fractional part ties
    w[2] = 0
    w[2, :3] = th.tensor([0.25, 0.25, 0.5])  # exact zeros elsewhere
    w[3] = th.linspace(0, 1, K)        # ramp
    w[4] = 0
    w[4, -1] = 1e-30                   # tiny but valid
    return w


def gen_resample():
    (mi,) = _import_from("barf", ["model_interpolation"])
    g = th.Generator().manual_seed(3)
    out = {}
    model = mi.NerfInterpolation.__new__(mi.NerfInterpolation)
    th.nn.Module.__init__(model)
    model.far_sphere_normalized = 8.0
    B, K = 64, 64
    for N in (128, 256):
        tc = th.sort(2 + th.rand(B, K, generator=g) * 6, dim=1).values
        dist = th.diff(tc, dim=1, append=th.full((B, 1), 8.0))
        w = _weights_suite(g, B, K)
        t0, t1 = model._sample_t_pdf_weighted(tc, w, dist, N)
        out.update({f"barf_N{N}_tc": f32(tc), f"barf_N{N}_w": f32(w), f"barf_N{N}_dist": f32(dist),
                    f"barf_N{N}_t0": f32(t0), f"barf_N{N}_t1": f32(t1)})
    # naive-to-vanilla round/argmax variant (K = 64 coarse + 192 fine)
    (n2v,) = _import_from("naive-to-vanilla", ["model_interpolation"])
    m2 = n2v.NerfInterpolation.__new__(n2v.NerfInterpolation)
    th.nn.Module.__init__(m2)
    m2.samples_per_ray_coarse, m2.samples_per_ray_fine, m2.far_sphere_normalized = 64, 192, 1 / 3
    tc = th.sort(0.1 + th.rand(B, K, generator=g) * (1 / 3 - 0.1), dim=1).values
    dist = th.diff(tc, dim=1, append=th.full((B, 1), 1 / 3))
    w = _weights_suite(g, B, K)
    w = w * 0.9  # the reference variant does not renormalise
    t0, t1 = m2._sample_t_fine(tc, w, dist)
    out.update({"n2v_tc": f32(tc), "n2v_w": f32(w), "n2v_dist": f32(dist), "n2v_t0": f32(t0), "n2v_t1": f32(t1)})
    np.savez_compressed(os.path.join(OUT, "resample.npz"), **out)


def _barf_models(pe, mia):
    th.manual_seed(0)
    barf = mia.NerfModel(4, 256, True, False, 2, pe.BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0),
                         pe.BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0))
    th.manual_seed(0)
    n2v = mia.NerfModel(4, 256, True, True, 2, pe.FourierFeatures(10, 2 * th.pi), pe.FourierFeatures(4, 1.0))
    th.manual_seed(0)
    small = mia.NerfModel(2, 64, False, False, 3, pe.BarfPositionalEncoding(6, 3.4, 0, 1, True, 1.0),
                          pe.BarfPositionalEncoding(2, 1.5, 0, 1, False, 1.0))
    return {"barf": barf, "n2v": n2v, "small": small}


def gen_model():
    pe, mia = _import_from("barf", ["positional_encodings", "model_interpolation_architecture"])
    g = th.Generator().manual_seed(4)
    out = {}
    N = 300
    pos = th.rand(N, 3, generator=g) * 4 - 2
    d = th.randn(N, 3, generator=g)
    d = d / th.linalg.vector_norm(d, dim=1, keepdim=True)
    out["pos"], out["dir"] = f32(pos), f32(d)
    for name, m in _barf_models(pe, mia).items():
        # weights are not stored: the build re-creates them from th.manual_seed(0) (same construction
        # order) and these per-tensor checksums prove the initial weights are identical
        for k, v in m.state_dict().items():
            out[f"{name}.sdsum.{k}"] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
        p = pos.clone().requires_grad_(True)
        dens, rgb = m.forward(p, d, None, None, None)
        gd = th.randn(N, generator=g)
        gc = th.randn(N, 3, generator=g)
        ((dens * gd).sum() + (rgb * gc).sum()).backward()
        out[f"{name}.density"], out[f"{name}.rgb"] = f32(dens), f32(rgb)
        out[f"{name}.gd"], out[f"{name}.gc"] = f32(gd), f32(gc)
        out[f"{name}.dpos"] = f32(p.grad)
        for k, prm in m.named_parameters():
            if k.endswith(".bias") or k in ("model_segments.0.0.weight", "model_color.2.weight",
                                            "model_color.0.weight"):
                out[f"{name}.grad.{k}"] = f32(prm.grad)
            out[f"{name}.gradsum.{k}"] = np.array([prm.grad.double().sum().item(),
                                                   prm.grad.double().abs().sum().item()])
    np.savez_compressed(os.path.join(OUT, "model.npz"), **out)


def gen_color():
    pe, mia, mi = _import_from("barf", ["positional_encodings", "model_interpolation_architecture",
                                        "model_interpolation"])
    g = th.Generator().manual_seed(5)
    out = {}
    B, Kc, Nf = 24, 64, 128
    o = th.randn(B, 3, generator=g)
    o = o / th.linalg.vector_norm(o, dim=1, keepdim=True) * 4.03
    tgt = th.randn(B, 3, generator=g) * 0.3
    d = tgt - o
    d = d / th.linalg.vector_norm(d, dim=1, keepdim=True)
    pw = th.full((B,), 1 / 1111.1)
    th.manual_seed(0)
    model = mia.NerfModel(4, 256, True, False, 2, pe.BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0),
                          pe.BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0))
    ren = mi.NerfInterpolation(2.0, 8.0, model, Nf, "stratified_uniform", 0.0, "middle", model, Kc)
    tc = th.sort(2 + th.rand(B, Kc, generator=g) * 6, dim=1).values
    t0, t1 = ren._get_intervals(tc)
    rgb, w, dist = ren._compute_color(model, t0, t1, o, d, pw, B, Kc)
    out.update({"o": f32(o), "d": f32(d), "pw": f32(pw), "tc": f32(tc), "rgb": f32(rgb), "w": f32(w)})
    # forward coarse+fine with the coarse t injected (RNG-free)
    ren._sample_t_stratified_uniform = lambda *a, **k: ren._get_intervals(tc.clone())
    rgb_f, rgb_c = ren.forward(o, d, pw)
    out["fwd_rgb_fine"], out["fwd_rgb_coarse"] = f32(rgb_f), f32(rgb_c)
    np.savez_compressed(os.path.join(OUT, "color.npz"), **out)


def gen_cos_kat():
    t = th.load(os.path.join(REF, "barf", "cos_test_barf.pt"), weights_only=True)
    np.savez_compressed(os.path.join(OUT, "cos_kat.npz"), cos=f32(t))


def gen_ipe_grad():
    """Autograd of the integrated encodings w.r.t. position AND direction (BARF-style pose
    refinement through mip-NeRF's IPE), positional_encodings.py:170-282."""
    (pe,) = _import_from("barf", ["positional_encodings"])
    g = th.Generator().manual_seed(6)
    N = 193
    x = th.rand(N, 3, generator=g) * 8 - 4
    d = th.randn(N, 3, generator=g)
    d = d / th.linalg.vector_norm(d, dim=1, keepdim=True)
    t0 = 2 + th.rand(N, 1, generator=g) * 6
    t1 = t0 + th.rand(N, 1, generator=g) * 0.2 + 1e-3
    pw = th.full((N, 1), 1 / 1111.1)
    out = {"x": f32(x), "dir": f32(d), "t0": f32(t0), "t1": f32(t1), "pw": f32(pw)}
    cases = {}
    for dv in (True, False):
        for pws in (0.0, 0.5):
            enc = pe.IntegratedFourierFeatures(10, 2 * th.pi, True, dv)
            enc.pixel_width_sigma = pws
            cases[f"ipe_dv{int(dv)}_pws{pws}"] = enc
    for dv in (True, False):
        enc = pe.IntegratedBarfFourierFeatures(10, 6.3, 0, 1, True, 1.0, dv)
        enc.pixel_width_sigma = 0.0
        cases[f"ipebarf_dv{int(dv)}_a6.3"] = enc
    for key, enc in cases.items():
        xx = x.clone().requires_grad_(True)
        dd = d.clone().requires_grad_(True)
        y = enc.forward(xx, dd, pw, t0, t1)
        gy = th.randn(y.shape, generator=g)
        (y * gy).sum().backward()
        out[key] = f32(y)
        out[key + "_gy"] = f32(gy)
        out[key + "_dx"] = f32(xx.grad)
        out[key + "_ddir"] = f32(dd.grad)
    np.savez_compressed(os.path.join(OUT, "ipe_grad.npz"), **out)


def gen_garf():
    """GARF field MLPs (barf/model_garf_radiance.py, barf/model_garf_proposal.py, barf/gaussian.py;
    same layers as garf/model_radiance.py / model_proposal.py): th.manual_seed(0) construction with
    the garf/main.py:29-30 Gaussian init range, forward outputs and all parameter gradients."""
    rad_m, prop_m, gauss_m = _import_from("barf", ["model_garf_radiance", "model_garf_proposal", "gaussian"])
    g = th.Generator().manual_seed(7)
    out = {}
    N = 257
    pos = th.rand(N, 3, generator=g) * 4 - 2
    d = th.randn(N, 3, generator=g)
    d = d / th.linalg.vector_norm(d, dim=1, keepdim=True)
    out["pos"], out["dir"] = f32(pos), f32(d)
    th.manual_seed(0)
    rad = rad_m.RadianceNetwork(0.5, 2.0, 5e-4, 5e-5, 0, 1.0, 0.0)
    th.manual_seed(0)
    prop = prop_m.ProposalNetwork(0.5, 2.0, 5e-4, 5e-5, 0, 1.0, 0.0)
    for name, m in (("radiance", rad), ("proposal", prop)):
        for k, v in m.state_dict().items():
            out[f"{name}.sdsum.{k}"] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
        p = pos.clone().requires_grad_(True)
        dd = d.clone().requires_grad_(True)
        if name == "radiance":
            rgb, dens = m.forward(p, dd)
            gc = th.randn(N, 3, generator=g)
            gd = th.randn(N, generator=g)
            ((rgb * gc).sum() + (dens * gd).sum()).backward()
            out[f"{name}.rgb"], out[f"{name}.density"] = f32(rgb), f32(dens)
            out[f"{name}.gc"], out[f"{name}.gd"] = f32(gc), f32(gd)
            out[f"{name}.ddir"] = f32(dd.grad)
        else:
            dens = m.forward(p)
            gd = th.randn(dens.shape, generator=g)
            (dens * gd).sum().backward()
            out[f"{name}.density"], out[f"{name}.gd"] = f32(dens), f32(gd)
        out[f"{name}.dpos"] = f32(p.grad)
        for k, prm in m.named_parameters():
            if prm.numel() <= 4096:
                out[f"{name}.grad.{k}"] = f32(prm.grad)
            out[f"{name}.gradsum.{k}"] = np.array([prm.grad.double().sum().item(),
                                                   prm.grad.double().abs().sum().item()])
    # GaussActivation alone (forward and both gradients) on extreme inputs
    z = th.randn(64, 48, generator=g) * 3
    z[0, :4] = th.tensor([0.0, -0.0, 30.0, -1e-3])
    s = th.rand(48, generator=g) * 2 - 1
    s[0] = 0.0
    zz = z.clone().requires_grad_(True)
    act = gauss_m.GaussAct(48)
    with th.no_grad():
        act.inv_standard_deviation.copy_(s)
    y = act(zz)
    gy = th.randn(y.shape, generator=g)
    (y * gy).sum().backward()
    out.update({"act.z": f32(z), "act.s": f32(s), "act.y": f32(y), "act.gy": f32(gy), "act.dz": f32(zz.grad),
                "act.ds": f32(act.inv_standard_deviation.grad)})
    np.savez_compressed(os.path.join(OUT, "garf.npz"), **out)


def gen_pose():
    """CameraExtrinsics (barf/model_camera_extrinsics.py:7-85): so3 -> SO3 and the refined rays,
    with gradients w.r.t. rotation / translation."""
    (ce,) = _import_from("barf", ["model_camera_extrinsics"])
    g = th.Generator().manual_seed(8)
    m = ce.CameraExtrinsics(10, 1e-3, 1e-5, 100)
    with th.no_grad():
        m.rotation.copy_(th.randn(10, 3, generator=g) * 0.3)
        m.translation.copy_(th.randn(10, 3, generator=g) * 0.1)
    B = 200
    idx = th.randint(0, 10, (B,), generator=g)
    o = th.randn(B, 3, generator=g)
    d = th.randn(B, 3, generator=g)
    new_o, new_d, R, t = m.forward(idx, o, d)
    go, gd = th.randn(B, 3, generator=g), th.randn(B, 3, generator=g)
    ((new_o * go).sum() + (new_d * gd).sum()).backward()
    np.savez_compressed(os.path.join(OUT, "pose.npz"), rotation=f32(m.rotation), translation=f32(m.translation),
                        idx=idx.numpy().astype(np.int64), o=f32(o), d=f32(d), new_o=f32(new_o), new_d=f32(new_d),
                        R=f32(R), go=f32(go), gd=f32(gd), drot=f32(m.rotation.grad), dtrans=f32(m.translation.grad))


def gen_pose_render():
    """Pose gradients through the whole rendering path, as BarfModel trains them
    (barf/model_barf.py:29-92): CameraExtrinsics.forward (model_camera_extrinsics.py:77-85) ->
    NerfInterpolation._compute_color (model_interpolation.py:356-414) on a BARF NerfModel ->
    backward to the so3 rotation and translation parameters."""
    pe, mia, mi, ce = _import_from("barf", ["positional_encodings", "model_interpolation_architecture",
                                            "model_interpolation", "model_camera_extrinsics"])
    g = th.Generator().manual_seed(10)
    th.manual_seed(0)
    model = mia.NerfModel(4, 256, True, False, 2, pe.BarfPositionalEncoding(10, 6.3, 0, 1, True, 1.0),
                          pe.BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0))
    ren = mi.NerfInterpolation(2.0, 8.0, model, 32, "equidistant", -1.0, "middle")
    extr = ce.CameraExtrinsics(6, 1e-3, 1e-5, 100)
    with th.no_grad():
        extr.rotation.copy_(th.randn(6, 3, generator=g) * 0.05)
        extr.translation.copy_(th.randn(6, 3, generator=g) * 0.05)
    B, S = 40, 32
    o = th.randn(B, 3, generator=g)
    o = o / th.linalg.vector_norm(o, dim=1, keepdim=True) * 4.03
    d = th.randn(B, 3, generator=g) * 0.3 - o
    d = d / th.linalg.vector_norm(d, dim=1, keepdim=True)
    idx = th.randint(0, 6, (B,), generator=g)
    pw = th.full((B,), 1 / 555.56)
    t = 2.0 + th.arange(S, dtype=th.float32).unsqueeze(0).repeat(B, 1) * (6.0 / S) \
        + th.rand(B, 1, generator=g) * (6.0 / S)
    t0, t1 = ren._get_intervals(t)
    o2, d2, _, _ = extr.forward(idx, o, d)
    rgb, w, _ = ren._compute_color(model, t0, t1, o2, d2, pw, B, S)
    grgb = th.randn(B, 3, generator=g)
    (rgb * grgb).sum().backward()
    np.savez_compressed(os.path.join(OUT, "pose_render.npz"), rotation=f32(extr.rotation),
                        translation=f32(extr.translation), idx=idx.numpy().astype(np.int64), o=f32(o), d=f32(d),
                        pw=f32(pw), t0=f32(t0), t1=f32(t1), rgb=f32(rgb), w=f32(w), grgb=f32(grgb),
                        drot=f32(extr.rotation.grad), dtrans=f32(extr.translation.grad))


def gen_mipnerf():
    """The older mip_NeRF directory's API (mip_NeRF/mip_model.py:11-167, model_interpolation.py)."""
    mm, mi = _import_from("mip_NeRF", ["mip_model", "model_interpolation"])
    g = th.Generator().manual_seed(11)
    out = {}
    N = 256
    x = th.rand(N, 3, generator=g) * 4 - 2
    d = th.randn(N, 3, generator=g)
    d = d / th.linalg.vector_norm(d, dim=1, keepdim=True)
    t0 = 1.0 + th.rand(N, 1, generator=g) * 4
    t1 = t0 + th.rand(N, 1, generator=g) * 0.1 + 1e-3
    pw = 1 / 1111.1
    out.update({"x": f32(x), "dir": f32(d), "t0": f32(t0), "t1": f32(t1)})
    for dv in (False, True):
        out[f"ipe_dv{int(dv)}"] = f32(mm.IntegratedFourierFeatures(10, 2 * th.pi, dv).forward(x, d, t0, t1, pw))
    th.manual_seed(0)
    model = mm.MipNerfModel(4, 256, (True, 10, 4), 2, True)
    for k, v in model.state_dict().items():
        out[f"model.sdsum.{k}"] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
    dens, rgb = model.forward(x, d, t0, t1, pw)
    gd, gc = th.randn(N, generator=g), th.randn(N, 3, generator=g)
    ((dens * gd).sum() + (rgb * gc).sum()).backward()
    out.update({"model.density": f32(dens), "model.rgb": f32(rgb), "model.gd": f32(gd), "model.gc": f32(gc)})
    for k, prm in model.named_parameters():
        out[f"model.gradsum.{k}"] = np.array([prm.grad.double().sum().item(), prm.grad.double().abs().sum().item()])
    # coarse (32) + fine (64 more) forward of MipNerf with the coarse t injected (RNG-free)
    th.manual_seed(0)
    ren = mm.MipNerf(1.0, 5.0, 96, 4, (True, 32), (True, 10, 4), 2, distribute_variance=True)
    B = 16
    o = th.randn(B, 3, generator=g) * 0.1
    rd = th.randn(B, 3, generator=g)
    rd = rd / th.linalg.vector_norm(rd, dim=1, keepdim=True)
    pwb = th.full((B,), 1 / 1111.1)
    tc = th.sort(1.0 + th.rand(B, 32, generator=g) * 4, dim=1).values
    ren._sample_t_coarse = lambda batch_size: ren._get_intervals(tc.clone())
    rgb_f, rgb_c = ren.forward(o, rd, pwb)
    out.update({"ren.o": f32(o), "ren.d": f32(rd), "ren.pw": f32(pwb), "ren.tc": f32(tc),
                "ren.rgb_fine": f32(rgb_f), "ren.rgb_coarse": f32(rgb_c)})
    np.savez_compressed(os.path.join(OUT, "mipnerf.npz"), **out)


def gen_feed():
    """Training-batch assembly (barf/dataset.py:407-481, 514-557, 613-637; data_module.py:276-369)
    run by the reference on a small in-memory image set (the Lego data is absent), batches collated
    the way torch's default DataLoader collate stacks __getitem__ tuples."""
    ds_mod, dm_mod, ce = _import_from("barf", ["dataset", "data_module", "model_camera_extrinsics"])
    g = th.Generator().manual_seed(12)
    out = {"kat_meshgrid_4x2": f32(ds_mod.ImagePoseDataset._get_directions_meshgrid(4, 2, 4.0))}
    n, H, W, sigmas = 3, 7, 5, [8.0, 4.0, 0.0]
    images = th.rand(n, H, W, len(sigmas), 3, generator=g)
    R = ce.CameraExtrinsics.so3_to_SO3(th.randn(n, 3, 1, generator=g))
    c2w = th.zeros(n, 4, 4)
    c2w[:, :3, :3] = R
    c2w[:, :3, 3] = th.randn(n, 3, generator=g) * 4
    c2w[:, 3, 3] = 1
    focal = W / 2 / np.tan(0.6911112 / 2)
    ds = ds_mod.ImagePoseDataset.__new__(ds_mod.ImagePoseDataset)
    meshgrid = ds_mod.ImagePoseDataset._get_directions_meshgrid(H, W, focal)
    ray_o, ray_d = ds_mod.ImagePoseDataset._meshgrid_to_world(meshgrid, c2w)
    cam_o, cam_d = ds_mod.ImagePoseDataset._get_cam_origs_and_directions(c2w)
    cam_on, _, ray_on, ray_dn = ds_mod.ImagePoseDataset._apply_noise(cam_o, cam_d, ray_o, ray_d, 0.1, 0.2, 3)
    ds.camera_to_worlds, ds.camera_origins, ds.camera_origins_noisy = c2w, cam_o, cam_on
    ds.ray_directions, ds.ray_directions_noisy = ray_d, ray_dn
    ds.images, ds.image_batch_size, ds.n_images = images, H * W, n
    ds.index_to_index = {i: i for i in range(n)}
    ds.gaussian_blur_sigmas = sigmas
    ds.pixel_width = th.tensor(1 / focal)
    idx = th.randperm(n * H * W, generator=g)[:97]
    items = [ds[int(i)] for i in idx]
    batch = tuple(th.stack([it[k] for it in items]) for k in range(7))
    out.update({"images": f32(images), "c2w": f32(c2w), "focal": np.array([focal], np.float32),
                "sigmas": np.array(sigmas, np.float32), "indices": idx.numpy().astype(np.int64),
                "o_raw": f32(batch[0]), "o_noisy": f32(batch[1]), "d_raw": f32(batch[2]), "d_noisy": f32(batch[3]),
                "colors": f32(batch[4]), "img_idx": batch[5].numpy().astype(np.int64), "pw": f32(batch[6])})
    dm = dm_mod.ImagePoseDataModule.__new__(dm_mod.ImagePoseDataModule)
    dm.gaussian_blur_sigmas = sigmas
    for sigma in (0.1, 2.0, 5.0, 8.0):
        out[f"blur_{sigma}"] = f32(dm.get_blurred_pixel_colors(batch, sigma)[4])
    np.savez_compressed(os.path.join(OUT, "feed.npz"), **out)


def gen_nerf2d():
    """2d-reconstruction (C1): Nerf2d with the reference's default init under th.manual_seed(0),
    fourier_levels 10 (main.py:43-51) — forward on pixel-centre-style points in [0, 1)^2, the MSE
    training-step loss, every parameter gradient, and the parameters after three Adam steps
    (lr 1e-3) on the same batch."""
    (m2d,) = _import_from("2d-reconstruction", ["model"])
    g = th.Generator().manual_seed(21)
    th.manual_seed(0)
    model = m2d.Nerf2d(width=64, height=48, fourier_levels=10)
    out = {f"init_sum.{k}": np.array([v.double().sum().item(), v.double().abs().sum().item()])
           for k, v in model.state_dict().items()}
    x = th.rand(300, 2, generator=g)
    y = th.rand(300, 3, generator=g)
    y_hat = model(x)
    loss = th.nn.functional.mse_loss(y_hat, y)
    loss.backward()
    out.update({"x": f32(x), "y": f32(y), "y_hat": f32(y_hat), "loss": np.array([loss.item()], np.float32),
                "pe": f32(model.model[0](x))})
    out.update({f"grad.{k}": f32(p.grad) for k, p in model.named_parameters()})
    opt = th.optim.Adam(model.parameters(), lr=1e-3)
    for _ in range(3):
        opt.zero_grad()
        th.nn.functional.mse_loss(model(x), y).backward()
        opt.step()
    out.update({f"adam3_sum.{k}": np.array([v.double().sum().item(), v.double().abs().sum().item()])
                for k, v in model.state_dict().items()})
    out.update({f"adam3_head.{k}": f32(v.reshape(-1)[:256]) for k, v in model.state_dict().items()})
    sys.modules.pop("model", None)
    np.savez_compressed(os.path.join(OUT, "nerf2d.npz"), **out)


def gen_kabsch():
    """Kabsch alignment with outlier removal and the pose error of BARF's calibration model
    (barf/model_camera_calibration.py:69-156, 340-345), run by the reference on synthetic camera
    origins: a similarity transform of points on a sphere plus noise, a few gross outliers, a
    reflected cloud, and the no-outlier-removal branch."""
    (cc,) = _import_from("barf", ["model_camera_calibration"])
    M = cc.CameraCalibrationModel
    obj = M.__new__(M)
    g = th.Generator().manual_seed(31)
    out = {}

    def rot(v):
        return th.matrix_exp(th.cross(-th.eye(3).view(1, 3, 3), v.view(-1, 3, 1), dim=1))[0]

    cases = {"noisy": (100, 0.01, 0, False), "outliers": (100, 0.005, 6, False), "reflect": (60, 0.01, 0, True),
             "small": (12, 0.02, 1, False)}
    for name, (n, noise, n_out, reflect) in cases.items():
        raw = th.nn.functional.normalize(th.randn(n, 3, generator=g), dim=1) * 4.03
        R0 = rot(th.randn(3, generator=g))
        c0 = 0.5 + th.rand(1, generator=g).item()
        t0 = th.randn(1, 3, generator=g)
        src = raw * th.tensor([1.0, 1.0, -1.0]) if reflect else raw
        pred = (R0 @ src.T).T * c0 + t0 + noise * th.randn(n, 3, generator=g)
        if n_out:
            pred[:n_out] += 3.0 * th.randn(n_out, 3, generator=g)
        out[f"{name}.raw"], out[f"{name}.pred"] = f32(raw), f32(pred)
        for ro in (True, False):
            R, t, c = obj.kabsch_algorithm(raw, pred, remove_outliers=ro)
            out[f"{name}.ro{int(ro)}.R"], out[f"{name}.ro{int(ro)}.t"] = f32(R), f32(t)
            out[f"{name}.ro{int(ro)}.c"] = np.array([float(c)], np.float32)
        # compute_pose_error: kabsch(pred -> raw) with outlier removal, mean distance over all cameras
        obj.compute_post_transform_params = (
            lambda from_raw_to_pred=True, return_origs=False, remove_outliers=True, raw=raw, pred=pred:
            (obj.kabsch_algorithm(pred, raw, remove_outliers=remove_outliers), raw, pred))
        out[f"{name}.pose_error"] = np.array([float(M.compute_pose_error(obj))], np.float32)
    np.savez_compressed(os.path.join(OUT, "kabsch.npz"), **out)


def gen_hashgrid2d():
    """2d-ingp/model.py:13-115 INGPTable / INGPEncoding: the reference's readable copy of the
    multiresolution hash grid (the 3d-ingp file itself was not read).  8 levels between 16 and
    4096, T = 2^14, 2 features, the reference's own table init under th.manual_seed(0); inputs on a
    1/1024 grid (so that u = x/8 + 0.5 exactly for the 3-D kernel's x = 8u - 4).  Stored: the
    resolutions, bijective flags, per-level tables, corner indices (compute_idx on the corners
    (x_i, y_j) in the forward's order), bilinear weights and the encoding output."""
    (m,) = _import_from("2d-ingp", ["model"])
    th.manual_seed(0)
    enc = m.INGPEncoding(4096, 16, 2 ** 14, 2, 8)
    g = th.Generator().manual_seed(3)
    k = th.randint(0, 1024, (509, 2), generator=g)
    k = th.cat((k, th.tensor([[0, 0], [1023, 1023], [0, 1023]])), dim=0)
    u = k.float() / 1024
    out = {"u": f32(u), "res": np.array([t.resolution for t in enc.encodings], np.int64),
           "bijective": np.array([int(t.bijective) for t in enc.encodings], np.int64),
           "features": f32(enc(u))}
    for l, t in enumerate(enc.encodings):
        xs = u * t.resolution
        fl = th.floor(xs)
        lim = th.stack((fl, fl + 1), dim=1)
        corners = th.stack([lim[:, [i, j], th.arange(2)] for i, j in [(0, 0), (0, 1), (1, 0), (1, 1)]],
                           dim=1).to(th.int64)
        out[f"table{l}"] = f32(t.table)
        out[f"idx{l}"] = t.compute_idx(corners).numpy().astype(np.int64)
        out[f"w{l}"] = f32(th.prod(1 - th.abs(xs.unsqueeze(1) - corners), dim=-1))
    np.savez_compressed(os.path.join(OUT, "hashgrid2d.npz"), **out)


GENERATORS = {"hashgrid2d": gen_hashgrid2d, "kabsch": gen_kabsch, "nerf2d": gen_nerf2d, "pe": gen_pe, "composite": gen_composite, "resample": gen_resample, "model": gen_model,
              "color": gen_color, "cos_kat": gen_cos_kat, "ipe_grad": gen_ipe_grad, "garf": gen_garf,
              "pose": gen_pose, "pose_render": gen_pose_render, "mipnerf": gen_mipnerf, "feed": gen_feed}


if __name__ == "__main__":
    _install_stubs()
    th.set_num_threads(8)
    for name in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[name]()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
