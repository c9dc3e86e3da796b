"""Probe: fused forward time of the 16- and 32-sample-wave kernels on the MLP alone (encoding rows
given, no compositing), n2v NerfModel, M samples (training path: every layer output stored)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-experiments_amd"), os.path.join(ROOT, "tests")]
import test_gpu_fused as F  # noqa: E402
from nerf_amd import mlp, mlp_fused  # noqa: E402
from nerf_amd.mlp import MLPFunction  # noqa: E402

torch.set_float32_matmul_precision("high")
DEV = "cuda"
M = int(sys.argv[1]) if len(sys.argv) > 1 else 524288
model = F._model("n2v").to(DEV)
plan = model._get_plan()
plan.to_device(torch.device(DEV))
g = torch.Generator(device=DEV).manual_seed(21)
pos_pe = torch.zeros(M, 64, device=DEV)
pos_pe[:, :63] = torch.rand(M, 63, device=DEV, generator=g) * 2 - 1
dir_pe = torch.zeros(M // 64, 32, device=DEV)
dir_pe[:, :27] = torch.rand(M // 64, 27, device=DEV, generator=g) * 2 - 1
params = [p.detach().requires_grad_(True) for p in plan.params()]
for w in os.environ.get("W32_LIST", "0,1,0,1").split(","):
    os.environ["NERF_FUSED_W32"] = w
    for _ in range(3):
        MLPFunction.apply(plan, M, pos_pe, dir_pe, 64, *params)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        MLPFunction.apply(plan, M, pos_pe, dir_pe, 64, *params)
    e1.record()
    torch.cuda.synchronize()
    print(f"W32={w} M={M}: {e0.elapsed_time(e1) / n:.3f} ms per forward (incl. image pack)", flush=True)
