"""Per-parameter gradient error of the fused input-gradient chain vs the layer-by-layer backward
(n2v NerfModel), printed for every parameter (debug aid for csrc/mlp_fused.hip).
Usage: python tools/chain_check.py [M] [rd]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-experiments_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.set_float32_matmul_precision("high")
from test_gpu_fused import _model  # noqa: E402
from nerf_amd import mlp_fused  # noqa: E402
from nerf_amd.mlp import MLPFunction  # noqa: E402

DEV = torch.device("cuda", 0)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
rd = int(sys.argv[2]) if len(sys.argv) > 2 else 1
g = torch.Generator(device=DEV).manual_seed(7)
pos_pe = torch.zeros(M, 64, device=DEV)
pos_pe[:, :60] = torch.rand(M, 60, device=DEV, generator=g) * 2 - 1
nd = (M + rd - 1) // rd
dir_pe = torch.zeros(nd, 32, device=DEV)
dir_pe[:, :24] = torch.rand(nd, 24, device=DEV, generator=g) * 2 - 1
w_out = torch.randn(M, 4, device=DEV, generator=g)
grads, dys = {}, {}
for fused in (False, True):
    model = _model("n2v").to(DEV)
    plan = model._get_plan()
    mlp_fused.ENABLED = fused
    outs = MLPFunction.apply(plan, M, pos_pe, dir_pe, rd, *plan.params())
    (outs[1][:, :4] * w_out).sum().backward()
    torch.cuda.synchronize()
    grads[fused] = {n: p.grad.detach().double() for n, p in model.named_parameters()}
for n in grads[False]:
    a, b = grads[False][n], grads[True][n]
    scale = max(a.abs().max().item(), 1e-12)
    err = (a - b).abs() / scale
    idx = (err == err.max()).nonzero()[0].tolist()
    print(f"{n:40s} rel err {err.max().item():.3e} at {idx}  nbad {(err > 1e-2).sum().item()}")
