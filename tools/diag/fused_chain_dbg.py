"""Debug helper: parameter gradients of the fused input-gradient chain and of the layer-by-layer
backward against an fp64 torch reference (n2v NerfModel)."""
import sys
import torch
sys.path[:0] = ["/root/repo", "/root/repo/nerf-experiments_amd", "/root/repo/tests"]
import test_gpu_fused as T  # noqa: E402
import nerf_amd  # noqa: E402
from nerf_amd import mlp_fused  # noqa: E402
from nerf_amd.mlp import MLPFunction  # noqa: E402
nerf_amd._lib.load()
torch.set_float32_matmul_precision("high")
DEV = "cuda"
M, rd = 4096 * 64, 64
g = torch.Generator(device=DEV).manual_seed(7)
pos_pe = torch.zeros(M, 64, device=DEV)
pos_pe[:, :60] = torch.rand(M, 60, device=DEV, generator=g) * 2 - 1
dir_pe = torch.zeros(M // rd, 32, device=DEV)
dir_pe[:, :24] = torch.rand(M // rd, 24, device=DEV, generator=g) * 2 - 1
w_out = torch.randn(M, 4, device=DEV, generator=g)
res = {}
for fused in (False, True):
    model = T._model("n2v").to(DEV)
    plan = model._get_plan()
    mlp_fused.ENABLED = fused
    outs = MLPFunction.apply(plan, M, pos_pe, dir_pe, rd, *plan.params())
    (outs[1][:, :4] * w_out).sum().backward()
    torch.cuda.synchronize()
    res[fused] = {n: p.grad.detach().double() for n, p in model.named_parameters()}
# fp64 reference on the same plan
model = T._model("n2v").to(DEV).double()
plan = model._get_plan()
acts = []
pe64, de64 = pos_pe.double(), dir_pe.double()
for idx, lp in enumerate(plan.layers):
    parts = []
    for s in lp.sources:
        if s.kind == "act":
            parts.append(acts[s.layer][:, :s.k_valid])
        elif s.kind == "pos":
            parts.append(pe64[:, :s.k_valid])
        else:
            parts.append(de64.repeat_interleave(rd, dim=0)[:, :s.k_valid])
    y = torch.nn.functional.linear(torch.cat(parts, 1), lp.module.weight, lp.module.bias)
    acts.append(torch.relu(y) if lp.relu else y)
(acts[-1][:, :4] * w_out.double()).sum().backward()
ref = {n: p.grad.detach() for n, p in model.named_parameters()}
for n, r in ref.items():
    s = r.abs().max().item()
    print(f"{n:32s} scale {s:.3e} layerwise {(res[False][n] - r).abs().max().item() / s:.2e} "
          f"fused {(res[True][n] - r).abs().max().item() / s:.2e}")
