#!/usr/bin/env python3
"""Headline benchmark: NeRF training-step throughput in ray-samples/s (coarse + fine).

Default workload (BASELINE.json's metric: "ray-samples/sec (coarse+fine) ... Lego 800²" =
configs[2]): mip-NeRF masked integrated PE, per GPU 4096 rays x (64 coarse + 128 fine) samples per
step — stratified coarse t (offset -1) -> IPE -> shared NerfModel (n_hidden 4, width 256, 2 segments,
delayed direction) -> compositing -> pdf resample (largest remainder) -> fine IPE -> NerfModel ->
compositing -> MSE(fine) + MSE(coarse) -> backward -> (N>1: RCCL all-reduce) -> Adam
(barf/model_builders.py:106-195, barf/model_mip.py:85-304, barf/model_interpolation.py:417-526).
Lego 800x800 pixel width; synthetic Lego-scale rays (no dataset is available offline).

Other BASELINE.json configs as extra workloads (same JSON line, their own `config`):
  --workload n2v   configs[1]: naive-to-vanilla NeRF, Lego 400x400, 4096 rays x 64 stratified samples,
                   Fourier PE L10/L4, delayed density, density factor 3*7 (naive-to-vanilla/main.py:89-102)
  --workload barf  configs[3]: BARF pose refinement — masked Fourier PE L10/L4 + identity, 128
                   equidistant samples (run_barf.py:150-196), rays refined by per-image so3
                   CameraExtrinsics (100 views) whose gradients come back through the fused
                   ray-mode encoding backward, 4096 rays per GPU

  --workload garf  garf GarfModel (SURVEY §8 a8 + f3): proposal estimator on 64 samples (interlevel loss) ->
                   inverse-cdf 192 samples -> radiance network, 4096 rays per GPU
  --workload ingp  configs[4]: 3d-ingp NaiveINGP (3d-ingp/model.py:195-519): INGPEncoding(1600, 16, 2^16, 2, 16)
                   + FourierFeatures(4) shared by separate coarse / fine NerfModelINGP (8 x 256) fields,
                   64 coarse samples, fine pass of 64 + 192 (round/argmax), positions at the sample t,
                   Adam(0.9, 0.99, 1e-15); 5120 rays per GPU -> 64 + 256 ray-samples per ray

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload mip|n2v|barf|garf|ingp]
    N>1: `python bench.py --gpus N` starts N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE,
    MASTER_ADDR 127.0.0.1, a free MASTER_PORT; launch_ranks), or run it under
    `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N` (WORLD_SIZE must equal N).

Prints ONE JSON line on rank 0 (schema: see DESIGN.md §Measurement).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nerf-experiments_amd"))

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_MFMA_PEAK_TFLOPS = 2516.6  # MI355X_MICROARCH.md: ~2.5 PF dense (32x32x16 bf16, 32 cycles, 2.4 GHz)
X3_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 3.0   # 3 bf16 MFMAs per fp32-accurate product
HBM_PEAK_GBS = 8000.0

RAYS = 4096
SAMPLES = 64
NEAR, FAR = 0.1, 1.0 / 3.0

WORKLOADS = {
    "n2v": {"config": "naive-to-vanilla NeRF training step, Lego 400x400, 4096 rays x 64 samples per GPU "
                      "(BASELINE.json configs[1])", "rays": RAYS, "coarse": 0, "fine": SAMPLES},
    "mip": {"config": "mip-NeRF masked integrated PE, coarse 64 + fine 128 samples (pdf resample), shared "
                      "NerfModel, Lego 800x800, 4096 rays per GPU (BASELINE.json configs[2])",
            "rays": 4096, "coarse": 64, "fine": 128},
    "garf": {"config": "garf GarfModel step: nerfacc-equivalent PropNetEstimator (lindisp, stratified) with "
                       "ProposalNetwork (3-512-256-128-1) on 64 samples -> inverse-cdf 192 samples -> RadianceNetwork "
                       "(601,604 params) -> rendering; MSE + interlevel loss, both networks fwd+bwd, Adam; near/far "
                       "2/7 (garf/main.py:168-171, model_garf.py:194-260), 4096 rays per GPU (the reference trains "
                       "at 1024)",
             "rays": 4096, "coarse": 64, "fine": 192},
    "ingp": {"config": "3d-ingp NaiveINGP step: INGPEncoding(1600, 16, 2^16, 2, 16) + FourierFeatures(4) shared by "
                       "separate coarse and fine NerfModelINGP fields (8 x 256, softplus(z - 1)); 64 coarse samples, "
                       "fine pass of 64 + 192 (round/argmax resample) at the sample t; MSE(coarse) + MSE(fine), "
                       "Adam(0.9, 0.99, 1e-15); near/far 2/7 (3d-ingp/main.py:40-118), 5120 rays per GPU "
                       "(BASELINE.json configs[4])", "rays": 5120, "coarse": 64, "fine": 256},
    "barf": {"config": "BARF camera-pose refinement: masked Fourier PE L10/L4 + identity, 128 equidistant "
                       "samples, per-image so3 CameraExtrinsics (100 views), 4096 rays per GPU "
                       "(BASELINE.json configs[3])", "rays": 4096, "coarse": 0, "fine": 128},
}


def synthetic_batch(n_rays: int, seed: int, device):
    """Lego-shaped rays in naive-to-vanilla's normalised space: camera centres on the upper
    hemisphere (radius 0.168) looking at the scene centre, 400x400 pixel cone width."""
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(n_rays, 2, generator=g)
    theta = u[:, 0] * 2 * math.pi
    z = u[:, 1] * 0.9 + 0.1
    r = torch.sqrt(1 - z * z)
    o = torch.stack((r * torch.cos(theta), r * torch.sin(theta), z), dim=1) * 0.168
    jitter = (torch.rand(n_rays, 3, generator=g) - 0.5) * 0.08
    d = torch.nn.functional.normalize(-o + jitter, dim=1)
    pw = torch.full((n_rays,), 1.0 / 555.56)
    target = 0.5 + 0.5 * torch.sin(torch.stack((3 * d[:, 0], 5 * d[:, 1] + 1, 7 * d[:, 2] + 2), dim=1))
    return o.to(device), d.to(device), pw.to(device), target.to(device)


def synthetic_batch_lego(n_rays: int, seed: int, device, image_size: int):
    """Blender-Lego-scale rays in barf space: camera centres at radius 4.03 on the upper hemisphere
    looking at the origin, pixel width 1/focal for the given image size."""
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(n_rays, 2, generator=g)
    theta = u[:, 0] * 2 * math.pi
    z = u[:, 1] * 0.9 + 0.1
    r = torch.sqrt(1 - z * z)
    o = torch.stack((r * torch.cos(theta), r * torch.sin(theta), z), dim=1) * 4.03
    jitter = (torch.rand(n_rays, 3, generator=g) - 0.5) * 0.5
    d = torch.nn.functional.normalize(-o + jitter, dim=1)
    focal = image_size / 2 / math.tan(0.6911112 / 2)
    pw = torch.full((n_rays,), 1.0 / focal)
    target = 0.5 + 0.5 * torch.sin(torch.stack((3 * d[:, 0], 5 * d[:, 1] + 1, 7 * d[:, 2] + 2), dim=1))
    img = torch.randint(0, 100, (n_rays,), generator=g)
    return o.to(device), d.to(device), pw.to(device), target.to(device), img.to(device)


def lookat_c2w(n_views: int, radius: float, seed: int) -> torch.Tensor:
    """[n, 4, 4] camera-to-world matrices of cameras on the upper hemisphere at `radius` looking at
    the origin (camera looks down -z, y up: the Blender convention of barf/dataset.py:417-451)."""
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(n_views, 2, generator=g)
    theta = u[:, 0] * 2 * math.pi
    z = u[:, 1] * 0.9 + 0.1
    r = torch.sqrt(1 - z * z)
    back = torch.stack((r * torch.cos(theta), r * torch.sin(theta), z), dim=1)
    right = torch.nn.functional.normalize(torch.linalg.cross(torch.tensor([0.0, 0.0, 1.0]).expand_as(back), back),
                                          dim=1)
    up = torch.linalg.cross(back, right)
    c2w = torch.zeros(n_views, 4, 4)
    c2w[:, :3, 0], c2w[:, :3, 1], c2w[:, :3, 2] = right, up, back
    c2w[:, :3, 3] = back * radius
    c2w[:, 3, 3] = 1
    return c2w


def device_feed(name: str, device, rank: int, batch_size: int):
    """DeviceRayFeed over 100 synthetic views (procedural colours of each pixel's ray direction)
    at the workload's scene scale; the feed assembles every step's batch on the GPU."""
    from nerf_amd.ray_feed import DeviceRayFeed
    size, radius = (400, 0.168) if name == "n2v" else ((800, 4.03) if name == "mip" else (400, 4.03))
    focal = size / 2 / math.tan(0.6911112 / 2)
    c2w = lookat_c2w(100, radius, 77)
    images = torch.zeros(100, size, size, 1, 3, device=device)
    feed = DeviceRayFeed(images, c2w, focal, batch_size, rotation_noise_sigma=0.15 if name == "barf" else 0.0,
                         translation_noise_sigma=0.15 if name == "barf" else 0.0, noise_seed=0,
                         dataloader_seed=rank, device=device)
    n = 100 * size * size
    flat = images.view(n, 3)
    for s in range(0, n, 1 << 22):
        idx = torch.arange(s, min(n, s + (1 << 22)), device=device)
        d = feed.batch(idx)[2]
        flat[s:s + idx.shape[0]] = 0.5 + 0.5 * torch.sin(torch.stack((3 * d[:, 0], 5 * d[:, 1] + 1, 7 * d[:, 2] + 2),
                                                                     dim=1))
    return feed


def build_model(device):
    from nerf_amd import FourierFeatures, NerfInterpolation, NerfModel
    torch.manual_seed(0)
    model = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0),
                      learning_rate_start=5e-4, learning_rate_stop=5e-5)
    ren = NerfInterpolation(NEAR, FAR, model, SAMPLES, "stratified_uniform", 0.0, "middle",
                            density_factor=(3.0, 7.0)).to(device)
    return ren


def _feed_stream(feed):
    """Endless batches: epoch after epoch of the feed's shuffled order."""
    while True:
        yield from feed.epoch()


def build_workload(name: str, device, rank: int, feed: bool = False):
    """(renderer, extra modules, optimizer, loss closure, render closure) for one workload; with
    feed=True every step draws a fresh batch from the on-device ray feed."""
    from nerf_amd import (BarfPositionalEncoding, FusedAdam, IntegratedBarfFourierFeatures, NerfInterpolation,
                          NerfModel)
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    w = WORKLOADS[name]
    if name == "n2v":
        ren = build_model(device)
        o, d, pw, target = synthetic_batch(w["rays"], 1000 + rank, device)
        opt = ren.configure_optimizers()["optimizer"]
        if feed:
            nxt = _feed_stream(device_feed(name, device, rank, w["rays"]))

            def loss_fn():
                o_, _, d_, _, c_, _, pw_ = next(nxt)
                return ren.training_loss(o_, d_, pw_, c_[:, -1])[0]

            def render_fn():
                o_, _, d_, _, _, _, pw_ = next(nxt)
                return ren(o_, d_, pw_)
            return ren, [ren], opt, loss_fn, render_fn

        def loss_fn():
            return ren.training_loss(o, d, pw, target)[0]
        return ren, [ren], opt, loss_fn, lambda: ren(o, d, pw)
    if name == "mip":
        torch.manual_seed(0)
        pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
        pos.pixel_width_sigma = 0.0
        dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
        model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-4, 200000)
        ren = NerfInterpolation(2.0, 8.0, model, w["fine"], "stratified_uniform", -1.0, "middle", model,
                                w["coarse"]).to(device)
        o, d, pw, target, _ = synthetic_batch_lego(w["rays"], 1000 + rank, device, 800)
        opt = ren.configure_optimizers()["optimizer"]
        if feed:
            nxt = _feed_stream(device_feed(name, device, rank, w["rays"]))

            def loss_fn():
                o_, _, d_, _, c_, _, pw_ = next(nxt)
                return ren.training_loss(o_, d_, pw_, c_[:, -1])[0]

            def render_fn():
                o_, _, d_, _, _, _, pw_ = next(nxt)
                return ren(o_, d_, pw_)
            return ren, [ren], opt, loss_fn, render_fn

        def loss_fn():
            return ren.training_loss(o, d, pw, target)[0]
        return ren, [ren], opt, loss_fn, lambda: ren(o, d, pw)
    if name == "barf":
        torch.manual_seed(0)
        pos = BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0)
        dirs = BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0)
        model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-5, 200000)
        ren = NerfInterpolation(2.0, 8.0, model, w["fine"], "equidistant", -1.0, "middle").to(device)
        extr = CameraExtrinsics(100, 1e-3, 1e-5, 200000).to(device)
        with torch.no_grad():
            extr.rotation.normal_(0, 0.02)
            extr.translation.normal_(0, 0.02)
        o, d, pw, target, img = synthetic_batch_lego(w["rays"], 1000 + rank, device, 400)
        groups = [{"params": list(g["parameters"]), "lr": g["learning_rate_start"], "weight_decay": g["weight_decay"]}
                  for g in ren.param_groups + extr.param_groups]
        opt = FusedAdam(groups, eps=1e-5)

        if feed:
            nxt = _feed_stream(device_feed(name, device, rank, w["rays"]))

            def loss_fn():
                # noisy poses refined by the per-image extrinsics (model_barf.py's training input)
                _, o_, _, d_, c_, i_, pw_ = next(nxt)
                o2, d2, _, _ = extr(i_, o_, d_)
                return ren.training_loss(o2, d2, pw_, c_[:, -1])[0]

            def render_fn():
                _, o_, _, d_, _, i_, pw_ = next(nxt)
                o2, d2, _, _ = extr(i_, o_, d_)
                return ren(o2, d2, pw_)
            return ren, [ren, extr], opt, loss_fn, render_fn

        def loss_fn():
            o2, d2, _, _ = extr(img, o, d)
            return ren.training_loss(o2, d2, pw, target)[0]

        def render_fn():
            o2, d2, _, _ = extr(img, o, d)
            return ren(o2, d2, pw)
        return ren, [ren, extr], opt, loss_fn, render_fn
    if name == "ingp":
        from nerf_amd.model_ingp import FourierFeatures as IngpFourier
        from nerf_amd.model_ingp import INGPEncoding, NaiveINGP
        torch.manual_seed(0)
        # 3d-ingp/main.py:94-118 with the hash-grid position encoder of its commented config (:98-104)
        ren = NaiveINGP(near_sphere_normalized=2, far_sphere_normalized=7, samples_per_ray_fine=192,
                        samples_per_ray_coarse=64, position_encoder=INGPEncoding(1600, 16, 2 ** 16, 2, 16),
                        direction_encoder=IngpFourier(4), n_hidden=8, hidden_dim=256,
                        learning_rate=1e-5, learning_rate_decay=1, weight_decay=0).to(device)
        o, d, pw, target, _ = synthetic_batch_lego(w["rays"], 1000 + rank, device, 400)
        opt = ren.configure_optimizers()["optimizer"]
        if feed:
            nxt = _feed_stream(device_feed(name, device, rank, w["rays"]))

            def loss_fn():
                o_, _, d_, _, c_, _, _ = next(nxt)
                return ren.training_loss(o_, d_, c_[:, -1])[0]

            def render_fn():
                o_, _, d_, _, _, _, _ = next(nxt)
                return ren(o_, d_)
            return ren, [ren], opt, loss_fn, render_fn

        def loss_fn():
            return ren.training_loss(o, d, target)[0]
        return ren, [ren], opt, loss_fn, lambda: ren(o, d)
    if name == "garf":
        import types
        from nerf_amd import ProposalNetwork, RadianceNetwork
        from nerf_amd.prop_sampler import PropNetEstimator, rendering
        torch.manual_seed(0)
        # garf/main.py:24-39,168-175: gaussian init [0.5, 2], gaussian lr factor 16
        radiance = RadianceNetwork(0.5, 2.0, 2e-4, 2e-5, 0, 16.0).to(device)
        proposal = ProposalNetwork(0.5, 2.0, 5e-4, 5e-5, 0, 16.0).to(device)
        estimator = PropNetEstimator()
        groups = [{"params": list(g["parameters"]), "lr": g["learning_rate_start"], "weight_decay": g["weight_decay"]}
                  for g in proposal.param_groups + radiance.param_groups]
        opt = FusedAdam(groups, eps=1e-5)
        o, d, pw, target, _ = synthetic_batch_lego(w["rays"], 1000 + rank, device, 400)
        B, P, S = w["rays"], w["coarse"], w["fine"]

        def points(o_, d_, t0, t1):
            # garf/model_garf.py:87-111: o + d (t0 + t1) / 2
            pos = o_[:, None] + d_[:, None] * (t0 + t1)[..., None] / 2
            return pos.reshape(-1, 3), d_[:, None].expand(pos.shape).reshape(-1, 3)

        def render(o_, d_):
            # GarfModel.forward (garf/model_garf.py:194-236) on nerf_amd's nerfacc-equivalent estimator
            def prop_fn(t0, t1):
                return proposal(points(o_, d_, t0, t1)[0]).view(t0.shape)

            def rad_fn(t0, t1, _):
                pos, dirs = points(o_, d_, t0, t1)
                rgb, dens = radiance(pos, dirs)
                return rgb.view(*t0.shape, 3), dens.view(t0.shape)

            t0, t1 = estimator.sampling([prop_fn], [P], S, B, 2.0, 7.0, "lindisp", stratified=True,
                                        requires_grad=torch.is_grad_enabled())
            rgb, _, _, extras = rendering(t0, t1, rgb_sigma_fn=rad_fn)
            return rgb, extras

        def loss_of(o_, d_, c_):
            rgb, extras = render(o_, d_)
            # GarfModel._forward_loss (:239-260): interlevel loss for the proposal + MSE for the radiance
            return torch.nn.functional.mse_loss(rgb, c_) + estimator.compute_loss(extras["trans"])

        ren = types.SimpleNamespace(model_radiance=radiance)
        if feed:
            nxt = _feed_stream(device_feed(name, device, rank, w["rays"]))

            def loss_fn():
                o_, _, d_, _, c_, _, _ = next(nxt)
                return loss_of(o_, d_, c_[:, -1])

            def render_fn():
                o_, _, d_, _, _, _, _ = next(nxt)
                return render(o_, d_)
            return ren, [radiance, proposal], opt, loss_fn, render_fn

        def loss_fn():
            return loss_of(o, d, target)
        return ren, [radiance, proposal], opt, loss_fn, lambda: render(o, d)
    raise ValueError(name)


def flops_per_sample(ren) -> float:
    """Algorithmic MLP FLOPs per sample for fwd + bwd (dX and dW): 2*MACs * 3."""
    model = ren.model_fine if hasattr(ren, "model_fine") else ren.model_radiance
    macs = sum(m.in_features * m.out_features for m in model.modules() if isinstance(m, torch.nn.Linear))
    return 2.0 * macs * 3.0


def _cpu_model_name() -> str:
    cpu_model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu_model


def _cpu_mip_state():
    """The mip workload's NerfModel (same constructor, same torch.manual_seed(0) init) on the CPU."""
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfModel
    torch.manual_seed(0)
    pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
    dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
    model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-4, 200000)
    return model.state_dict()


def cpu_baseline(workload: str, seconds: float = 15.0):
    """The CPU oracle (oracle/nerf_oracle.py, PyTorch CPU fp32 — a restatement of the reference's
    CPU path, pinned to the reference's own outputs by tests/golden) running the workload's training
    step on a bounded sample: the same model, encodings, sample counts and loss, B rays per step."""
    from oracle import nerf_oracle as O
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    torch.manual_seed(4321)
    if workload == "mip":
        sd = {k: v.clone().requires_grad_(True) for k, v in _cpu_mip_state().items() if not k.endswith("alpha")}
        B, K, S = 1024, WORKLOADS["mip"]["coarse"], WORKLOADS["mip"]["fine"]
        near, far = 2.0, 8.0
        o, d, pw, target, _ = synthetic_batch_lego(B, 123, "cpu", 800)
        pw_rows = pw.view(B, 1)
        ones10 = torch.ones(10)

        def color(t0, t1, n):
            pos, dirs = O.compute_positions(o, d, t0, t1, "middle")
            N = B * n
            pw_s = pw_rows.repeat(1, n).view(N, 1)
            pos_pe = O.integrated_pe(pos.reshape(N, 3), dirs.reshape(N, 3), pw_s, t0.reshape(N, 1),
                                     t1.reshape(N, 1), 10, 1.0, True, True, 0.0, mask=ones10)
            dir_pe = O.barf_pe(dirs.reshape(N, 3), 4, 4.0, True, 1.0)
            dens, rgb = O.nerf_model_forward(sd, pos_pe, dir_pe, 2, 4, True, False)
            return O.render_rays(dens.view(B, n), rgb.view(B, n, 3), t1 - t0, 3.0, 1 / 3)

        def step():
            interval = (far - near) / K
            t = O.linspace_t(near, far, K).unsqueeze(0).repeat(B, 1) + torch.rand(B, K) * interval
            t = t + torch.rand(B, 1) * interval * -1.0          # uniform_sampling_offset_size = -1
            t0, t1 = O.intervals(t, far)
            rgb_c, w = color(t0, t1, K)
            f0, f1, _ = O.sample_t_pdf_weighted_batched(t0, w.detach(), (t1 - t0), S, far)
            rgb_f, _ = color(f0, f1, S)
            loss = torch.nn.functional.mse_loss(rgb_f, target) + torch.nn.functional.mse_loss(rgb_c, target)
            opt.zero_grad()
            loss.backward()
            opt.step()
        per_step = B * (K + S)
        desc = (f"training steps of {B} rays x (64 coarse + 128 fine) samples: masked IPE, shared NerfModel "
                f"fwd+bwd on both passes, pdf resample, Adam")
    else:
        ren = build_model("cpu") if workload == "n2v" else None
        if ren is None:
            return None
        sd = {k: v.clone().requires_grad_(True) for k, v in ren.model_radiance.state_dict().items()}
        B = 1024
        o, d, pw, target = synthetic_batch(B, 123, "cpu")

        def step():
            interval = (FAR - NEAR) / SAMPLES
            t = O.linspace_t(NEAR, FAR, SAMPLES).unsqueeze(0).repeat(B, 1) + torch.rand(B, SAMPLES) * interval
            t0, t1 = O.intervals(t, FAR)
            pos, dirs = O.compute_positions(o, d, t0, t1, "middle")
            pos_pe = O.fourier_features(pos.view(-1, 3), 10, 2 * math.pi)
            dir_pe = O.fourier_features(dirs.reshape(-1, 3), 4, 1.0)
            dens, rgb = O.nerf_model_forward(sd, pos_pe, dir_pe, 2, 4, True, True)
            out, _ = O.render_rays(dens.view(B, SAMPLES), rgb.view(B, SAMPLES, 3), t1 - t0, 3.0, 7.0)
            loss = torch.nn.functional.mse_loss(out, target)
            opt.zero_grad()
            loss.backward()
            opt.step()
        per_step = B * SAMPLES
        desc = f"training steps of {B} rays x {SAMPLES} samples (Fourier PE, NerfModel fwd+bwd, compositing, Adam)"
    opt = torch.optim.Adam(list(sd.values()), lr=5e-4, eps=1e-5)
    step()  # warm-up
    n, t_start = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t_start
        if el >= seconds or n >= 50:
            break
    return {"value": n * per_step / el, "unit": "ray-samples/s", "cores": threads, "kind": "port",
            "sample": f"{n} {desc}; oracle/nerf_oracle.py on torch CPU fp32, {el:.1f} s on {_cpu_model_name()}"}


def evidence_tag(workload: str, fn: str) -> str:
    """File tag of a kernel function's committed PMC evidence (tools/roofline_evidence.py):
    profiles/traffic_<tag>.json and profiles/pmc_<tag>.json."""
    return f"{workload}_" + "".join(c if c.isalnum() or c == "_" else "_" for c in fn).strip("_")


def _roofline(ks_fn: dict, prec: str, steps: int, workload: str):
    """Roofline object for the MFMA kernel FUNCTION with the most device time in the timed region
    (launches grouped by HIP kernel function, as rocprofv3 reports them: the fused kernel's forward
    and input-gradient-chain launches are one entry).  prec: "x3" (peak = bf16 dense / 3 MFMAs per
    product), "x1" (one bf16 pass: bf16 dense) or "fp32" (fp32 MFMA)."""
    peak = {"x3": X3_PEAK_TFLOPS, "x1": BF16_MFMA_PEAK_TFLOPS}.get(prec, FP32_MFMA_PEAK_TFLOPS)
    # HIP kernel functions as rocprofv3 names them (template instantiations separately: the fused
    # kernel's forward is mlp_fused_kernel<0>, its input-gradient chain mlp_fused_kernel<1>; <2> / <3>
    # in one bf16 pass)
    mfma_fns = ("mlp_fused_kernel<0>", "mlp_fused_kernel<1>", "mlp_fused_kernel<2>", "mlp_fused_kernel<3>",
                "linear_nt_x3_glds_kernel", "linear_nt_x3_kernel",
                "linear_wgrad_x3_tr_kernel", "linear_wgrad_x3_stream_kernel", "linear_wgrad_x3_kernel", "linear_nt_kernel",
                "linear_wgrad_kernel")
    cands = [k for k in mfma_fns if k in ks_fn]
    if not cands:
        return None
    dom = max(cands, key=lambda k: ks_fn[k]["ms"])
    r = ks_fn[dom]
    n = max(r["launches"], 1)
    avg_ms, avg_flops, avg_bytes = r["ms"] / n, r["flops"] / n, r["bytes"] / n
    achieved = avg_flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    intensity = avg_flops / avg_bytes if avg_bytes > 0 else float("inf")
    ridge = peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    hbm_bound = intensity < ridge
    achieved_gbs = avg_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = None
    tag = evidence_tag(workload, dom)
    tfile = os.path.join(ROOT, "profiles", f"traffic_{tag}.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            traffic = json.load(f).get("bytes_per_launch")
    pmc = None
    pfile = os.path.join(ROOT, "profiles", f"pmc_{tag}.json")
    if os.path.exists(pfile):
        with open(pfile) as f:
            pmc = json.load(f)
    total_ms = sum(v["ms"] for v in ks_fn.values())
    return {"kernel": dom, "roles": r["tags"],
            "precision": {"x3": "3 x bf16 MFMA; peak = bf16 dense / 3",
                          "x1": "1 x bf16 MFMA (matmul precision medium); peak = bf16 dense"}.get(prec, "fp32 MFMA 32x32x2"),
            "bound": "hbm" if hbm_bound else "mfma",
            "achieved": achieved_gbs if hbm_bound else achieved,
            "peak": HBM_PEAK_GBS if hbm_bound else peak,
            "unit": "GB/s" if hbm_bound else "TFLOP/s",
            "frac": achieved_gbs / HBM_PEAK_GBS if hbm_bound else achieved / peak,
            "traffic": traffic,
            "traffic_unit": "bytes per launch (PMC 2*FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
            "arithmetic_intensity": intensity, "ridge": ridge,
            "achieved_tflops": achieved, "peak_tflops": peak,
            "attainable_tflops": min(peak, intensity * HBM_PEAK_GBS * 1e9 / 1e12),
            "avg_launch_us": avg_ms * 1e3, "avg_flops_per_launch": avg_flops,
            "avg_bytes_per_launch": avg_bytes, "launches_per_step": r["launches"] / steps,
            "share_of_timed_kernel_time": r["ms"] / total_ms if total_ms > 0 else None,
            "pmc": pmc}


def _hbm_roofline(ks, hbm_bytes, hbm_ms, hbm_gbs, steps):
    """roofline_hbm of a step that launches the encoding / compositing kernels (NERF_FUSE_ENC=0,
    NERF_FUSE_COMPOSITE=0, or rays that do not fill the fused kernel's tiles)."""
    names = [k for k in ("encode_fwd", "composite_fwd", "composite_bwd") if k in ks]
    return {"kernel": " + ".join(names) + " (algorithmic bytes per launch)",
            "encode_launches_per_step": ks.get("encode_fwd", {}).get("launches", 0) / steps,
            "composite_launches_per_step": (ks.get("composite_fwd", {}).get("launches", 0)
                                            + ks.get("composite_bwd", {}).get("launches", 0)) / steps,
            "bound": "hbm", "achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": hbm_gbs / HBM_PEAK_GBS, "us_per_step": hbm_ms * 1e3 / steps,
            "bytes_per_step": hbm_bytes / steps}


MALL_GATHER_GBS = 8600.0   # MI355X_MICROARCH.md "Indexed rows": random rows of a 38 MB table (Infinity Cache)


def _gather_roofline(ks_fn: dict, steps: int, workload: str):
    """The hash-grid kernels (C5) against the rate of the cache level their 7.2 MB table lives in:
    larger than one XCD's 4 MB L2, far smaller than the 256 MB Infinity Cache (MALL), whose random-row
    gather rate the guide measures at 8.6 TB/s chip-wide.  achieved = algorithmic bytes per launch
    (8 corners x F fp32 gathered + F fp32 written per (sample, level); the backward:
    F fp32 read + 8 corners x F 8-byte fixed-point adds) / the launch's event-timed duration
    (nerf_hashgrid_bwd: the whole bucketed backward call, its kernels together)."""
    out = {}
    for fn in ("hashgrid_fwd_tile_kernel", "hashgrid_fwd_level_kernel", "hashgrid_fwd_kernel", "hashgrid_bwd_walk_kernel",
               "hashgrid_bwd_kernel", "nerf_hashgrid_bwd"):
        r = ks_fn.get(fn)
        if not r or r["ms"] <= 0:
            continue
        gbs = r["bytes"] / (r["ms"] * 1e-3) / 1e9
        entry = {"bound": "mall", "achieved": gbs, "peak": MALL_GATHER_GBS, "unit": "GB/s",
                 "frac": gbs / MALL_GATHER_GBS, "avg_launch_us": r["ms"] * 1e3 / max(r["launches"], 1),
                 "avg_bytes_per_launch": r["bytes"] / max(r["launches"], 1),
                 "launches_per_step": r["launches"] / steps, "ms_per_step": r["ms"] / steps}
        for kind in ("traffic", "pmc"):
            f = os.path.join(ROOT, "profiles", f"{kind}_{evidence_tag(workload, fn)}.json")
            if os.path.exists(f):
                with open(f) as fh:
                    d = json.load(fh)
                entry[kind] = d.get("bytes_per_launch") if kind == "traffic" else d
        out[fn] = entry
    return out or None


def frame_roofline(ren, wl: dict, device, H: int = 800, W: int = 800, reps: int = 3):
    """HBM roofline of the same positional-encoding and compositing kernels at ONE full-frame
    launch: H*W rays (800 x 800: the C3 view size) x the workload's coarse and fine sample counts,
    the size a full-view render hands them on a 288 GB GPU (the training batch is 4096 rays: a
    latency-bound 6-20 MB per compositing launch).  Same kernel parameters as the step (the
    model's own encoders; density factors and fused activations of its renderer); synthetic
    rays and raw heads; untimed warm-up, then `reps` event-timed launches each."""
    from nerf_amd import kernels as K
    from nerf_amd.positional_encodings import PositionalEncoding
    model = getattr(ren, "model_radiance", None)
    enc = getattr(model, "position_encoder", None)
    if not isinstance(enc, PositionalEncoding):
        return None                                   # hash grid (ingp) / garf: no PE kernel
    B = H * W
    g = torch.Generator(device=device).manual_seed(7)
    o = torch.randn(B, 3, device=device, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0], device=device)
    d = torch.nn.functional.normalize(torch.randn(B, 3, device=device, generator=g) * 0.2
                                      - torch.tensor([0.0, 0.0, 1.0], device=device), dim=1)
    pw = torch.full((B,), 1 / 1111.1, device=device)
    sa, sb = ren.density_factor
    counts = sorted({wl["coarse"], wl["fine"]} - {0})
    timer, prev = K.KernelTimer(), K.TIMER
    with torch.no_grad():
        for S in counts:
            t = torch.linspace(ren.near_sphere_normalized, ren.far_sphere_normalized, S + 1, device=device)
            t0, t1 = t[:-1].expand(B, S).contiguous(), t[1:].expand(B, S).contiguous()
            dist = t1 - t0
            dens = torch.randn(B * S, device=device, generator=g)
            col = torch.randn(B * S, 4, device=device, generator=g)
            g_rgb = torch.randn(B, 3, device=device, generator=g)
            gd, gc = torch.empty_like(dens), torch.empty_like(col)
            for rep in range(reps + 1):
                K.TIMER = timer if rep > 0 else None
                enc.encode_rays(o, d, t0, t1, pw, S, 1, 1)
                K.composite_fwd(dens, 1, col, 4, dist, B, S, sa, sb, True, 0.0)
                K.composite_bwd(dens, 1, col, 4, dist, B, S, sa, sb, True, 0.0, g_rgb, None, gd, 1, gc, 4)
            K.TIMER = prev
            del t0, t1, dist, dens, col, gd, gc
    torch.cuda.synchronize()
    ks = timer.summary()
    per = {k: {"gbs": v["bytes"] / (v["ms"] * 1e-3) / 1e9, "us_per_launch": v["ms"] * 1e3 / v["launches"],
               "bytes_per_launch": v["bytes"] / v["launches"]} for k, v in ks.items()}
    nb, ms = sum(v["bytes"] for v in ks.values()), sum(v["ms"] for v in ks.values())
    gbs = nb / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    return {"kernel": "encode_fwd + composite_fwd + composite_bwd, one launch per full %dx%d frame "
                      "(%d rays x %s samples; algorithmic bytes per launch)" % (H, W, B, "/".join(map(str, counts))),
            "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "per_kernel": per}


def frame_render(ren, wl: dict, device, name: str, H: int = 800, W: int = 800):
    """One full H x W view rendered the way the reference's image logger does it
    (barf/image_logger.py:155-214 through NerfInterpolation.render_image: batches of 65 536 rays
    through forward, clip to [0, 1]) — the C3 frame render.  Reports its rate and which kernels it
    launched: with the fused compositing no positional-encoding or compositing kernel runs (the
    encodings are generated and the rays composited inside nerf_mlp_fused_render)."""
    from nerf_amd import kernels as K
    if not hasattr(ren, "render_image"):
        return None
    B = H * W
    o, d, pw, _, _ = synthetic_batch_lego(B, 4242, device, W)
    pw = pw.view(B, 1)
    ren.render_image(o[:65536], d[:65536], pw[:65536])      # warm-up
    torch.cuda.synchronize()
    timer, prev = K.KernelTimer(), K.TIMER
    K.TIMER = timer
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    rgb = ren.render_image(o, d, pw)
    e.record()
    K.TIMER = prev
    torch.cuda.synchronize()
    ms = s.elapsed_time(e)
    ks = timer.summary()
    spr = wl["coarse"] + wl["fine"]
    return {"view": f"{H}x{W} ({B} rays x {spr} samples), batches of up to 65536 rays through forward (render_image: at most 2 GB of fused-pass rows per batch), clip to [0, 1]",
            "ms": ms, "ray_samples_per_s": B * spr / (ms * 1e-3),
            "launches": {k: v["launches"] for k, v in ks.items()},
            "encode_launches": ks.get("encode_fwd", {}).get("launches", 0),
            "composite_launches": ks.get("composite_fwd", {}).get("launches", 0),
            "mean_rgb": float(rgb.mean().item())}


def init_distributed(backend: str = "nccl"):
    """(world, rank, local_rank, torch.distributed or None) from the torchrun environment; one
    process per GPU ("nccl" = RCCL on ROCm), "gloo" for the CPU rehearsal in tests/."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world <= 1:
        return world, rank, local_rank, None
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)
    return world, rank, local_rank, dist


def run_timed(step, steps: int, warmup: int, dist, sync, device, on_timed_start=None):
    """W untimed warmup steps, then EXACTLY K steps bracketed by barrier + device sync on both sides;
    returns (max over ranks of the timed wall time, the last step's return value)."""
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    if on_timed_start is not None:
        on_timed_start()
    out = None
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def teardown(dist) -> None:
    if dist is not None:
        dist.destroy_process_group()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, cmd: list[str], env: dict | None = None, poll_s: float = 0.2) -> int:
    """Start ``cmd`` as N rank processes of one node (RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set as torch.distributed.run sets them)
    and wait for them.  The caller has touched no GPU (the ranks initialise their own devices) and
    is not replaced (no exec): rank 0's stdout — the JSON line — passes straight through, the other
    ranks' stdout goes to stderr.  If a rank fails, the others (this launcher's own children, by
    PID) are terminated, so a rank blocked in a collective cannot hang the job; returns the first
    non-zero exit status, else 0."""
    import signal
    import subprocess
    base = dict(os.environ if env is None else env)
    base.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": base.get("MASTER_PORT") or str(_free_port()),
                 "GROUP_RANK": "0", "ROLE_RANK": "0"})
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), ROLE_WORLD_SIZE=str(n))
        procs.append(subprocess.Popen(cmd, env=e, stdout=None if r == 0 else sys.stderr))
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]          # every rank polled (no short-circuit)
            if all(c is not None for c in codes):
                break
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                status = bad[0]
                break
            time.sleep(poll_s)
    finally:
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.send_signal(signal.SIGTERM)
        for p in live:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if status == 0:
        status = next((p.returncode for p in procs if p.returncode != 0), 0)
    return status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="mip", choices=tuple(WORKLOADS))
    ap.add_argument("--mode", default="train", choices=("train", "render"),
                    help="train: forward + backward + all-reduce + Adam per step (the headline metric); "
                         "render: the forward pass only, without autograd (BASELINE.json's render metric)")
    ap.add_argument("--feed", default="device", choices=("device", "fixed"),
                    help="device: every step draws a fresh shuffled batch from 100 synthetic views through "
                         "the on-device ray feed (nerf_ray_batch); fixed: one resident batch reused")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-frame-roofline", action="store_true",
                    help="skip the full-frame launch measurement of the PE / compositing kernels")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--matmul-precision", default="high", choices=("highest", "high", "medium"),
                    help="torch.set_float32_matmul_precision for the MLP GEMMs: highest = fp32 MFMA, "
                         "high = 3 x bf16 split MFMA (fp32-accurate to ~2^-16), medium = one bf16 pass "
                         "(the reference's naive-to-vanilla run: medium + 16-mixed, main.py:53,58)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start N rank processes of this same
        # command (one per GPU) and relay rank 0's line.  Nothing above has touched the GPU, and
        # this process is not replaced (no exec): it only waits for its children.
        sys.exit(launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    torch.set_float32_matmul_precision(args.matmul_precision)

    # NERF_DIST_BACKEND=gloo rehearses the multi-process step on fewer GPUs than ranks (ranks share
    # devices round-robin); the driver's runs use RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("NERF_DIST_BACKEND", "nccl")
    world, rank, local_rank, dist = init_distributed(backend)
    if world != args.gpus:
        # under torch.distributed.run the world is the launcher's; a different --gpus would make
        # the line's n_gpus disagree with the ranks that ran
        teardown(dist)
        ap.error(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    device = torch.device("cuda", local_rank if backend == "nccl" else local_rank % torch.cuda.device_count())
    torch.cuda.set_device(device)

    import nerf_amd
    from nerf_amd import kernels as K
    from nerf_amd.ddp import BucketedGradAllReduce
    nerf_amd._lib.load()

    wl = WORKLOADS[args.workload]
    ren, modules, opt, loss_fn, render_fn = build_workload(args.workload, device, rank, args.feed == "device")
    # gradient buckets all-reduced asynchronously while backward runs; direct=True: the field MLPs'
    # weight gradients land in their buckets (N=1: in .grad) from the slab reduce itself, layer by
    # layer, and a field used twice per step accumulates there without an extra add per parameter
    allreduce = BucketedGradAllReduce([p for m in modules for p in m.parameters()], direct=True)
    torch.manual_seed(1234 + rank)
    render = args.mode == "render"

    def step():
        if render:
            with torch.no_grad():
                rgb, _ = render_fn()
            return rgb.mean()
        opt.zero_grad(set_to_none=True)
        loss = loss_fn()
        loss.backward()
        allreduce.finish()       # waits for the bucket all-reduces launched during backward
        opt.step()
        return loss

    def start_timer():
        K.TIMER = K.KernelTimer()

    elapsed, loss = run_timed(step, args.steps, args.warmup, dist, torch.cuda.synchronize, device, start_timer)
    timer, K.TIMER = K.TIMER, None
    final_loss = float(loss.item())

    samples_per_gpu = wl["rays"] * (wl["coarse"] + wl["fine"])
    samples_total = samples_per_gpu * world * args.steps
    value = samples_total / elapsed
    ks = timer.summary()
    ks_fn = timer.summary(by="fn")
    from nerf_amd.mlp import matmul_precision
    prec = matmul_precision()
    roofline = _roofline(ks_fn, prec, args.steps, args.workload)

    # HBM roofline of the bandwidth-bound kernels BASELINE.json's north_star names (positional
    # encoding + alpha compositing): algorithmic bytes (kernels.py, per launch) / event-timed duration
    hbm_tags = ("encode_fwd", "composite_fwd", "composite_bwd")
    hbm_bytes = sum(ks.get(k, {}).get("bytes", 0.0) for k in hbm_tags)
    hbm_ms = sum(ks.get(k, {}).get("ms", 0.0) for k in hbm_tags)
    hbm_gbs = hbm_bytes / (hbm_ms * 1e-3) / 1e9 if hbm_ms > 0 else 0.0

    if rank == 0:
        out = {
            "metric": ("ray-samples/sec (coarse+fine), render (forward only)" if render
                       else "ray-samples/sec (coarse+fine), training step"),
            "value": value,
            "unit": "ray-samples/s",
            "n_gpus": dist.get_world_size() if dist is not None else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if prec != "x1" else "bf16 products, fp32 accumulate",
            "matmul": {"x3": "3xbf16 split MFMA (hi*hi+hi*lo+lo*hi, fp32 accumulate)",
                       "x1": "1xbf16 MFMA (bf16(w)*bf16(x), fp32 accumulate; matmul precision medium)"}.get(
                prec, "fp32 MFMA"),
            "matmul_precision": args.matmul_precision,
            "data": ("synthetic: 100 procedural views at Lego scale, a fresh shuffled batch per step from the "
                     "on-device ray feed; random-init weights (torch.manual_seed(0))" if args.feed == "device" else
                     "synthetic Lego-shaped rays/targets (one resident batch), random-init weights "
                     "(torch.manual_seed(0))"),
            "config": {"workload": wl["config"], "workload_key": args.workload,
                       "rays_per_gpu": wl["rays"], "samples_per_ray": wl["coarse"] + wl["fine"],
                       "coarse_samples": wl["coarse"], "fine_samples": wl["fine"], "global_rays": wl["rays"] * world,
                       "parallelism": f"ray-batch dp{world}" + ((" (RCCL bucketed all-reduce from post-accumulate-grad hooks)"
                                                          if backend == "nccl" else
                                                          f" ({backend} bucketed all-reduce: a multi-process rehearsal)")
                                                         if world > 1 else "")},
            "roofline": roofline,
            "roofline_hbm": (_hbm_roofline(ks, hbm_bytes, hbm_ms, hbm_gbs, args.steps) if hbm_ms > 0 else
                             {"kernel": "none: the positional encodings and the alpha compositing have no launch "
                                        "of their own in this step; they run inside mlp_fused_kernel<0> (encoding "
                                        "rows generated per tile, rays composited at the tile end) and "
                                        "mlp_fused_kernel<1> (the compositing's gradient from per-sample "
                                        "coefficients), whose algorithmic bytes include theirs (DESIGN.md §3)",
                              "encode_launches_per_step": 0.0, "composite_launches_per_step": 0.0,
                              "bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": None, "us_per_step": 0.0, "bytes_per_step": 0.0}),
            "roofline_gather": _gather_roofline(ks_fn, args.steps, args.workload),
            "kernels": {k: {"launches_per_step": v["launches"] / args.steps, "ms_per_step": v["ms"] / args.steps,
                            "tflops": (v["flops"] / (v["ms"] * 1e-3) / 1e12) if v["ms"] > 0 else 0.0,
                            "gbs": (v["bytes"] / (v["ms"] * 1e-3) / 1e9) if v["ms"] > 0 else 0.0}
                        for k, v in ks.items()},
            "kernel_functions": {k: {"launches_per_step": v["launches"] / args.steps,
                                     "ms_per_step": v["ms"] / args.steps, "roles": v["tags"]}
                                 for k, v in ks_fn.items()},
            "mlp_tflops_per_step": (flops_per_sample(ren) / (3.0 if render else 1.0)) * samples_per_gpu
                                   / (elapsed / args.steps) / 1e12,
            ("mean_rgb" if render else "final_loss"): final_loss,
        }
        if world == 1 and not args.no_frame_roofline:
            try:          # auxiliary measurements: their failure must not cost the bench line
                out["frame_render"] = frame_render(ren, wl, device, args.workload)
            except Exception as e:      # noqa: BLE001
                out["frame_render"] = {"error": f"{type(e).__name__}: {e}"}
            try:
                fr = frame_roofline(ren, wl, device)
                if fr is not None:
                    fr["scope"] = ("the stand-alone encoding / compositing kernels, which neither the C3 training "
                                   "step nor its frame render (frame_render) launches: they serve samples-per-ray "
                                   "counts the fused compositing does not take (S not dividing the 128-sample tile, "
                                   "other than 256), matmul precision 'highest' and GARF's nerfacc-style rendering")
                out["roofline_hbm_frame"] = fr
            except Exception as e:      # noqa: BLE001
                out["roofline_hbm_frame"] = {"error": f"{type(e).__name__}: {e}"}
        if world == 1 and not args.no_cpu_baseline and not render:
            cb = cpu_baseline(args.workload, args.cpu_seconds)
            if cb is not None:
                out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    teardown(dist)


if __name__ == "__main__":
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # a rank that fails must exit at once: left to the interpreter's shutdown it can block in
        # the process group's teardown while its peers wait in a collective, and the job hangs
        try:
            main()
        except SystemExit:
            raise
        except BaseException:       # noqa: BLE001
            import traceback
            traceback.print_exc()
            sys.stderr.flush()
            sys.stdout.flush()
            os._exit(1)
    else:
        main()
