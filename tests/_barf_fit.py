"""A fixed-seed BARF pose-refinement fit on the GPU path (test helper, not collected by pytest).

Scene: three overlapping soft spheres with a sinusoidal colour texture (analytic density and colour;
the target of every pixel ray of N_VIEWS views at radius 4.03 looking at the origin is the
volume-rendering integral over 1024 midpoint samples, barf space, near / far 2 / 8).  The student
(NerfModel seed 0 with BARF's coarse-to-fine masked encoding, alpha 0 -> 10 over the first half of
the fit, + per-image CameraExtrinsics, barf/model_barf.py:29-92) sees the rays of PERTURBED poses
(rotation noise about the world axes, translation noise) and learns the scene and the per-image
corrections with FusedAdam, one fixed random ray batch order for every run.  Metrics
at the end: PSNR of the training rays (-10 log10 MSE, model_interpolation.py:588-597) and the
pose error of the refined camera origins against the true ones (compute_pose_error: Kabsch
similarity alignment with outlier removal, model_camera_calibration.py:340-345).

run_fit(precision) is what tests/test_gpu_barf_fit_precision.py and tools/barf_precision_fit.py
call with "high" (3 x bf16 split MFMA) and "highest" (exact fp32 MFMA)."""
from __future__ import annotations

import math

import torch

N_VIEWS, H, W = 24, 32, 32
RADIUS = 4.03


def _lookat(n: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(n, 2, generator=g)
    theta = u[:, 0] * 2 * math.pi
    z = u[:, 1] * 0.8 + 0.15
    r = torch.sqrt(1 - z * z)
    back = torch.stack((r * torch.cos(theta), r * torch.sin(theta), z), dim=1)
    right = torch.nn.functional.normalize(torch.linalg.cross(torch.tensor([0.0, 0.0, 1.0]).expand_as(back), back),
                                          dim=1)
    up = torch.linalg.cross(back, right)
    R = torch.stack((right, up, back), dim=2)          # columns: camera x, y, z in the world
    return R, back * RADIUS


def _rays(R: torch.Tensor, t: torch.Tensor):
    focal = W / 2 / math.tan(0.6911112 / 2)
    j, i = torch.meshgrid(torch.arange(W, dtype=torch.float32), torch.arange(H, dtype=torch.float32), indexing="xy")
    dc = torch.stack(((j - W / 2 + 0.5) / focal, -(i - H / 2 + 0.5) / focal, -torch.ones_like(j)), dim=-1)
    dc = torch.nn.functional.normalize(dc.reshape(-1, 3), dim=1)
    d = torch.einsum("vab,nb->vna", R, dc)                        # [V, HW, 3]
    o = t[:, None, :].expand_as(d)
    img = torch.arange(R.shape[0])[:, None].expand(R.shape[0], H * W)
    return o.reshape(-1, 3).contiguous(), d.reshape(-1, 3).contiguous(), img.reshape(-1).contiguous(), 1.0 / focal


def _so3(w: torch.Tensor) -> torch.Tensor:
    K = torch.zeros(w.shape[0], 3, 3)
    K[:, 0, 1], K[:, 0, 2], K[:, 1, 2] = -w[:, 2], w[:, 1], -w[:, 0]
    K = K - K.transpose(1, 2)
    return torch.matrix_exp(K)


def _field(seed: int):
    from nerf_amd import BarfPositionalEncoding, NerfModel
    torch.manual_seed(seed)
    pos = BarfPositionalEncoding(10, 0.0, 0.0, 0.5, True, 1.0)       # alpha 0 -> 10 over [0, 0.5]
    dirs = BarfPositionalEncoding(4, 0.0, 0.0, 0.5, True, 1.0)
    return NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-5, 200000)


_CENTERS = torch.tensor([[0.45, 0.0, 0.0], [-0.4, 0.35, 0.2], [0.0, -0.45, -0.3]])
_RADII = torch.tensor([0.6, 0.45, 0.5])


def _scene(x: torch.Tensor):
    """(density, colour) of the analytic scene at points x [..., 3] (float64)."""
    c, r = _CENTERS.to(x), _RADII.to(x)
    dist = (torch.linalg.norm(x[..., None, :] - c, dim=-1) - r).min(dim=-1).values
    sigma = 40.0 * torch.sigmoid(-dist / 0.02)
    col = 0.5 + 0.45 * torch.sin(torch.stack((7 * x[..., 0] + 3 * x[..., 1], 9 * x[..., 1] - 2 * x[..., 2] + 1,
                                              8 * x[..., 2] + 4 * x[..., 0] + 2), dim=-1))
    return sigma, col


def _render_scene(o: torch.Tensor, d: torch.Tensor, near: float = 2.0, far: float = 8.0, n: int = 1024):
    """Volume-rendered colour of the analytic scene along rays (midpoint rule, float64)."""
    out = []
    for s in range(0, o.shape[0], 2048):
        oo, dd = o[s:s + 2048].double(), d[s:s + 2048].double()
        t = torch.linspace(near, far, n + 1, dtype=torch.float64, device=o.device)
        tm, dt = (t[1:] + t[:-1]) / 2, t[1:] - t[:-1]
        x = oo[:, None, :] + tm[None, :, None] * dd[:, None, :]
        sigma, col = _scene(x)
        b = -sigma * dt
        T = torch.exp(torch.cumsum(torch.cat([torch.zeros_like(b[:, :1]), b[:, :-1]], 1), 1))
        w = T * (1 - torch.exp(b))
        out.append((w[..., None] * col).sum(1).float())
    return torch.cat(out)


def run_fit(precision: str, steps: int = 2000, batch: int = 2048, rot_noise: float = 0.03,
            trans_noise: float = 0.08, seed: int = 0) -> dict:
    from nerf_amd import FusedAdam, NerfInterpolation
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    from nerf_amd.pose import compute_pose_error
    dev = torch.device("cuda", 0)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(precision)
    try:
        R, t = _lookat(N_VIEWS, 77)
        o, d, img, pw = _rays(R, t)
        target = _render_scene(o.to(dev), d.to(dev))
        g = torch.Generator().manual_seed(1234 + seed)
        Rn = _so3(torch.randn(N_VIEWS, 3, generator=g) * rot_noise)
        tn = torch.randn(N_VIEWS, 3, generator=g) * trans_noise
        o_noisy = (o + tn[img]).to(dev)
        d_noisy = torch.einsum("nab,nb->na", Rn[img], d).contiguous().to(dev)
        img_d = img.to(dev)
        model = _field(0)
        ren = NerfInterpolation(2.0, 8.0, model, 128, "equidistant", 0.0, "middle").to(dev)
        extr = CameraExtrinsics(N_VIEWS, 1e-3, 1e-5, 200000).to(dev)
        groups = [{"params": list(gr["parameters"]), "lr": gr["learning_rate_start"], "weight_decay": 0.0}
                  for gr in ren.param_groups + extr.param_groups]
        opt = FusedAdam(groups, eps=1e-5)
        order = torch.randint(0, o.shape[0], (steps, batch), generator=g).to(dev)
        pwb = torch.full((batch,), pw, device=dev)
        losses = []
        encs = (model.position_encoder, model.direction_encoder)
        for s in range(steps):
            idx = order[s]
            for e in encs:
                e.update_alpha(s / steps)
            opt.zero_grad(set_to_none=True)
            o2, d2, _, _ = extr(img_d[idx], o_noisy[idx], d_noisy[idx])
            rgb, _ = ren(o2, d2, pwb)
            loss = torch.nn.functional.mse_loss(rgb, target[idx])
            loss.backward()
            opt.step()
            if s % (steps // 10) == 0 or s == steps - 1:
                losses.append(float(loss.detach()))
        with torch.no_grad():
            mse = 0.0
            for s in range(0, o.shape[0], 4096):
                sl = slice(s, s + 4096)
                o2, d2, _, _ = extr(img_d[sl], o_noisy[sl], d_noisy[sl])
                rgb, _ = ren(o2, d2, torch.full((o2.shape[0],), pw, device=dev))
                mse += float(((rgb - target[sl]) ** 2).sum())
            mse /= o.shape[0] * 3
            origs_true = t.to(dev)
            origs_pred, _ = extr.forward_origins(torch.arange(N_VIEWS, device=dev), (t + tn).to(dev))
            err = float(compute_pose_error(origs_true, origs_pred.contiguous()))
            err0 = float(compute_pose_error(origs_true, (t + tn).to(dev)))
        return {"precision": precision, "steps": steps, "psnr": -10 * math.log10(mse), "pose_error": err,
                "pose_error_initial": err0, "loss_curve": losses}
    finally:
        torch.set_float32_matmul_precision(prev)
