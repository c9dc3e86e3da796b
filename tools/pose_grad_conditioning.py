"""How well-conditioned are BARF's pose gradients?  The reference fixture pose_render.npz is
recomputed by the CPU oracle in fp32 and in fp64 (same weights, rays and t), and the GPU path in
"highest" (fp32 MFMA) and "high" (3 x bf16 split) is compared with the fp64 value.  Prints the
max error of each relative to the largest fp64 gradient magnitude."""
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-experiments_amd")]
from oracle import nerf_oracle as O  # noqa: E402


def oracle_grads(g, sd, dtype):
    rot = torch.tensor(g["rotation"], dtype=dtype, requires_grad=True)
    trans = torch.tensor(g["translation"], dtype=dtype, requires_grad=True)
    idx = torch.from_numpy(g["idx"])
    o, d = torch.tensor(g["o"], dtype=dtype), torch.tensor(g["d"], dtype=dtype)
    # so3 -> SO3 as barf/model_camera_extrinsics.py:39-43 (matrix_exp of the skew matrix)
    R = torch.matrix_exp(torch.cross(-torch.eye(3, dtype=dtype).view(1, 3, 3), rot.view(-1, 3, 1), dim=1))
    o2 = o + trans[idx]
    d2 = torch.matmul(R[idx], d.unsqueeze(-1)).squeeze(-1)
    t0, t1 = torch.tensor(g["t0"], dtype=dtype), torch.tensor(g["t1"], dtype=dtype)
    B, S = t0.shape
    pos, dirs = O.compute_positions(o2, d2, t0, t1, "middle")
    sdd = {k: v.to(dtype) for k, v in sd.items()}

    def pe(x, L, alpha):
        args = x.repeat_interleave(L, dim=1) * (2.0 ** torch.arange(L, dtype=dtype)).repeat(3)
        m = O.barf_mask(alpha, L).to(dtype).repeat(3).view(1, -1)
        return torch.cat((x, m * torch.cos(args), m * torch.sin(args)), dim=1)
    dens, rgb = O.nerf_model_forward(sdd, pe(pos.reshape(-1, 3), 10, 6.3), pe(dirs.reshape(-1, 3), 4, 4.0), 2, 4,
                                     True, False)
    b = (-dens.view(B, S) * (t1 - t0)) * 3.0 * (1 / 3)
    alpha = 1 - torch.exp(b)
    T = torch.cat((torch.ones(B, 1, dtype=dtype), torch.exp(torch.cumsum(b[:, :-1], dim=1))), dim=1)
    out = torch.sum((T * alpha).unsqueeze(-1) * rgb.view(B, S, 3), dim=1)
    (out * torch.tensor(g["grgb"], dtype=dtype)).sum().backward()
    return rot.grad.double().numpy(), trans.grad.double().numpy()


def gpu_grads(g, precision):
    from nerf_amd import BarfPositionalEncoding, NerfInterpolation, NerfModel
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    torch.set_float32_matmul_precision(precision)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 6.3, 0, 1, True, 1.0),
                      BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0))
    ren = NerfInterpolation(2.0, 8.0, model, 32, "equidistant", -1.0, "middle").to(dev)
    extr = CameraExtrinsics(6, 1e-3, 1e-5, 100).to(dev)
    with torch.no_grad():
        extr.rotation.copy_(torch.from_numpy(g["rotation"]))
        extr.translation.copy_(torch.from_numpy(g["translation"]))
    T = lambda a: torch.from_numpy(np.asarray(a)).to(dev)  # noqa: E731
    B, S = g["t0"].shape
    o2, d2, _, _ = extr(T(g["idx"]), T(g["o"]), T(g["d"]))
    rgb, _, _ = ren._compute_color(model, T(g["t0"]), T(g["t1"]), o2, d2, T(g["pw"]), B, S)
    (rgb * T(g["grgb"])).sum().backward()
    return extr.rotation.grad.double().cpu().numpy(), extr.translation.grad.double().cpu().numpy()


def main():
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "pose_render.npz")))
    from nerf_amd import BarfPositionalEncoding, NerfModel
    torch.manual_seed(0)
    sd = NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 6.3, 0, 1, True, 1.0),
                   BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0)).state_dict()
    sd = {k: v for k, v in sd.items() if not k.endswith("alpha")}
    ref64 = oracle_grads(g, sd, torch.float64)
    rows = {"reference_fixture_fp32": (g["drot"].astype(np.float64), g["dtrans"].astype(np.float64)),
            "oracle_fp32": oracle_grads(g, sd, torch.float32)}
    if torch.cuda.is_available():
        import nerf_amd
        nerf_amd._lib.load()
        rows["gpu_highest"] = gpu_grads(g, "highest")
        rows["gpu_high"] = gpu_grads(g, "high")
    res = {}
    for name, (dr, dt) in rows.items():
        res[name] = {"drot": float(np.abs(dr - ref64[0]).max() / np.abs(ref64[0]).max()),
                     "dtrans": float(np.abs(dt - ref64[1]).max() / np.abs(ref64[1]).max())}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
