"""Step-by-step check of the fused input-gradient chain (n2v NerfModel): every dY[l] the chain
writes against torch (fp64) from the same head gradient, weights and ReLU masks (debug aid for
csrc/mlp_fused.hip).  Usage: python tools/chain_steps.py [M]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-experiments_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.set_float32_matmul_precision("high")
from test_gpu_fused import _model  # noqa: E402
from nerf_amd import mlp, mlp_fused  # noqa: E402
from nerf_amd.mlp import MLPFunction  # noqa: E402

DEV = torch.device("cuda", 0)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
g = torch.Generator(device=DEV).manual_seed(7)
pos_pe = torch.zeros(M, 64, device=DEV)
pos_pe[:, :60] = torch.rand(M, 60, device=DEV, generator=g) * 2 - 1
dir_pe = torch.zeros(M, 32, device=DEV)
dir_pe[:, :24] = torch.rand(M, 24, device=DEV, generator=g) * 2 - 1
model = _model("n2v").to(DEV)
plan = model._get_plan()
mlp.CAPTURE = []
with torch.enable_grad():
    MLPFunction.apply(plan, M, pos_pe, dir_pe, 1, *plan.params())
acts, masks = mlp.CAPTURE[0]
mlp.CAPTURE = None
L = len(plan.layers)
fd = mlp_fused.FusedInputGrad(plan, DEV, False, False)
NH = plan.layers[L - 1].N
g_head = torch.zeros(M, (NH + 3) // 4 * 4, device=DEV)
g_head[:, :NH] = torch.randn(M, NH, device=DEV, generator=g)
dY = [torch.full((M, plan.layers[l].out_ld), float("nan"), device=DEV) for l in range(L - 1)]
fd.run(M, g_head, dY, masks, {}, {})
torch.cuda.synchronize()
gcur = g_head[:, :NH].double()
for l in range(L - 1, 0, -1):
    W = plan.layers[l].module.weight.detach().double()
    k = plan.layers[l].sources[0].k_valid
    ref = gcur @ W[:, :k]
    if plan.layers[l - 1].relu:
        ref = ref * (acts[l - 1][:, :k].double() > 0)
    got = dY[l - 1][:, :k].double()
    scale = max(ref.abs().max().item(), 1e-12)
    err = (got - ref).abs() / scale
    bad = (err > 1e-3).nonzero()
    if l == L - 1:
        unm = (gcur @ W[:, :k])
        torch.set_printoptions(precision=4, linewidth=200)
        print("unmasked row0", unm[0, :16].float().cpu())
        print("ref      row0", ref[0, :16].float().cpu())
        print("got      row0", got[0, :16].float().cpu())
        print("act>0    row0", (acts[l - 1][0, :16] > 0).int().cpu())
        print("mask words row0", [hex(x) for x in masks[l - 1][0].view(torch.int32).cpu().tolist()])
    print(f"dY[{l - 1}] rel err {err.max().item():.3e} nbad {bad.shape[0]} first {bad[:6].tolist()}")
    gcur = ref
