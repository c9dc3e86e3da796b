"""Probe: the 32-sample-wave forward (NERF_FUSED_W32=1) against the 16-sample kernel, per layer,
at several M: counts of rows / columns off by more than the parity bar, and their patterns."""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-experiments_amd"), os.path.join(ROOT, "tests")]
import test_gpu_fused as F  # noqa: E402

torch.set_float32_matmul_precision("high")
DEV = "cuda"
model = F._model("n2v").to(DEV)
plan = model._get_plan()
plan.to_device(torch.device(DEV))
for M in [int(a) for a in (sys.argv[1:] or ["128", "256", "4096", "32768", "262144"])]:
    g = torch.Generator(device=DEV).manual_seed(21)
    pos_pe = torch.zeros(M, 64, device=DEV)
    pos_pe[:, :63] = torch.rand(M, 63, device=DEV, generator=g) * 2 - 1
    dir_pe = torch.zeros(M, 32, device=DEV)
    dir_pe[:, :27] = torch.rand(M, 27, device=DEV, generator=g) * 2 - 1
    os.environ["NERF_FUSED_W32"] = "0"
    _, a16, m16, _ = F._run(model, pos_pe, dir_pe, 1, True)
    os.environ["NERF_FUSED_W32"] = "1"
    _, a32, m32, _ = F._run(model, pos_pe, dir_pe, 1, True)
    print(f"M={M}")
    for li, (x, y) in enumerate(zip(a16, a32)):
        n = plan.layers[li].N
        d = (x[:, :n] - y[:, :n]).abs()
        scale = max(1.0, x[:, :n].abs().max().item())
        bad = d > 1e-4 * scale
        nb = int(bad.sum())
        line = f"  layer {li} N={n} maxerr={d.max().item():.3e} bad={nb}"
        if nb:
            rows = bad.any(1).nonzero()[:, 0].cpu().numpy()
            cols = bad.any(0).nonzero()[:, 0].cpu().numpy()
            line += f" rows={len(rows)} first={rows[:6].tolist()} tiles={np.unique(rows // 128)[:10].tolist()}"
            line += f" rowmod128={np.unique(rows % 128)[:12].tolist()} cols={len(cols)} firstcols={cols[:12].tolist()}"
            line += f" y_nan={int(torch.isnan(y[:, :n]).sum())}"
        print(line, flush=True)
