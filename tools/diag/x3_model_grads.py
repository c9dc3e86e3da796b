"""Diagnostic: per-parameter gradient differences of NerfModel under fp32 vs 3xbf16 GEMMs."""
import math, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nerf-experiments_amd"))
from nerf_amd import BarfPositionalEncoding, NerfModel  # noqa: E402

g = np.load(os.path.join(ROOT, "tests/golden/model.npz"))
res = {}
for prec in ("highest", "high"):
    torch.set_float32_matmul_precision(prec)
    torch.manual_seed(0)
    m = NerfModel(4, 256, True, False, 2, BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0),
                  BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0)).cuda()
    pos = torch.tensor(g["pos"]).cuda().requires_grad_(True)
    d = torch.tensor(g["dir"]).cuda()
    dens, rgb = m(pos, d, None, None, None)
    ((dens * torch.tensor(g["barf.gd"]).cuda()).sum() + (rgb * torch.tensor(g["barf.gc"]).cuda()).sum()).backward()
    res[prec] = {k: p.grad.double().cpu() for k, p in m.named_parameters()}
    res[prec]["pos"] = pos.grad.double().cpu()
    res[prec]["dens"] = dens.detach().double().cpu()
for k in res["highest"]:
    a, b = res["highest"][k], res["high"][k]
    s = g.get(f"barf.gradsum.{k}")
    print(f"{k:32s} max|g|={a.abs().max():.3e} maxdiff={((a-b).abs().max()):.3e} "
          f"abssum fp32={a.abs().sum():.6e} x3={b.abs().sum():.6e} golden={s[1] if s is not None else float('nan'):.6e}")
