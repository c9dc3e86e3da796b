"""Determinism of the fused forward on NaiveINGP's fine field: render_raw / render_composite run
three times on the same rays, with the hash features in-kernel or from the stand-alone launch."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nerf-experiments_amd"))
from nerf_amd import model_interpolation_architecture as A  # noqa: E402
from nerf_amd.model_ingp import FourierFeatures, INGPEncoding, NaiveINGP  # noqa: E402

dev = torch.device("cuda", 0)
torch.set_float32_matmul_precision("high")
torch.manual_seed(0)
ren = NaiveINGP(2, 7, 192, 64, INGPEncoding(1600, 16, 2 ** 16, 2, 16), FourierFeatures(4), 8, 256).to(dev)
g = torch.Generator().manual_seed(5)
for S, B in ((256, 1024), (64, 4096), (256, 4096)):
    model = ren.model_fine
    o = (torch.randn(B, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 - torch.tensor([0.0, 0.0, 1.0]), dim=1).to(dev)
    t = (torch.linspace(2.0, 7.0 - 5.0 / S, S).repeat(B, 1) + torch.rand(B, S, generator=g) * (5.0 / S)).to(dev).contiguous()
    t_end = ren._intervals(t)
    dist = (t_end - t).contiguous()
    for fe in (True, False):
        A.FUSE_ENCODINGS = fe
        raws, comps = [], []
        with torch.no_grad():
            for _ in range(3):
                h = model.render_raw(o, d, None, t, t_end, S, 0, 1)
                raws.append((h.color_base[:, :3].clone(), h.dens_base[:, h.dens_col].clone()))
                rgb, w = model.render_composite(o, d, None, t, t_end, S, 0, 1, dist, 1.0, 1.0)
                comps.append((rgb.clone(), w.clone()))
        rr = [torch.equal(comps[0][0], c[0]) and torch.equal(comps[0][1], c[1]) for c in comps[1:]]
        ra = [torch.equal(raws[0][0], c[0]) and torch.equal(raws[0][1], c[1]) for c in raws[1:]]
        print(f"S={S} B={B} fuse_enc={fe}: render_composite repeatable {rr}, render_raw repeatable {ra}")
