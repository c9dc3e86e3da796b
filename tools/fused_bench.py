"""Microbenchmark of the fused field-MLP forward alone (n2v NerfModel, 4096 x 64 samples):
average launch time by HIP events, for A/B runs and rocprofv3 counter passes.
Usage: python tools/fused_bench.py [--iters N] [--layerwise]"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-experiments_amd")]

import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--M", type=int, default=4096 * 64)
ap.add_argument("--layerwise", action="store_true")
ap.add_argument("--train", action="store_true", help="record autograd: every layer output and mask is stored")
args = ap.parse_args()

import nerf_amd  # noqa: E402
from nerf_amd import FourierFeatures, NerfModel, mlp_fused  # noqa: E402
from nerf_amd.mlp import MLPFunction  # noqa: E402

torch.set_float32_matmul_precision("high")
mlp_fused.ENABLED = not args.layerwise
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0)).to(dev)
M = args.M
pos = torch.zeros(M, 64, device=dev)
pos[:, :60] = torch.rand(M, 60, device=dev) * 2 - 1
dirs = torch.zeros(M // 64, 32, device=dev)
dirs[:, :24] = torch.rand(M // 64, 24, device=dev) * 2 - 1
plan = model._get_plan()
with torch.set_grad_enabled(args.train):
    for _ in range(3):
        MLPFunction.apply(plan, M, pos, dirs, 64, *plan.params())
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.iters):
        MLPFunction.apply(plan, M, pos, dirs, 64, *plan.params())
    e.record()
    torch.cuda.synchronize()
ms = s.elapsed_time(e) / args.iters
flops = sum(2.0 * M * lp.module.in_features * lp.module.out_features for lp in plan.layers)
print(f"{'layerwise' if args.layerwise else 'fused'} {'training' if args.train else 'inference'} forward: {ms * 1e3:.1f} us/iter, "
      f"{flops / ms / 1e9:.1f} TFLOP/s (fp32-equivalent)")
