"""Times one 256 x 256 weight-gradient launch (M = 262144, the default bench's batch) from cold
inputs with HIP events.  Usage: python tools/wgrad_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nerf-experiments_amd"))
from nerf_amd import kernels as K  # noqa: E402

M, N, Kd = 262144, 256, 256
dev = torch.device("cuda:0")
dY = torch.randn(M, N, device=dev)
X = torch.randn(M, Kd, device=dev)
ws = torch.empty((K.linear_wgrad_workspace_bytes(M, N, Kd) + 3) // 4, device=dev)
for _ in range(3):
    K.linear_wgrad_x3(dY, N, [(X, Kd, 1)], M, ws)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
n = 20
for _ in range(n):
    K.linear_wgrad_x3(dY, N, [(X, Kd, 1)], M, ws)
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) * 1e3 / n
print(f"linear_wgrad_x3 256 x 256, M {M}: {us:.1f} us, "
      f"{2 * M * 1024 / us / 1e3:.0f} GB/s of dY+X  (NERF_WGRAD_SPLITS={os.environ.get('NERF_WGRAD_SPLITS', 'auto')})")
# with the fixed-order slab reduction into the nn.Linear layout, as the backward runs it
col_map = torch.arange(Kd, dtype=torch.int32, device=dev)
gW = torch.empty(N, Kd, device=dev)
gb = torch.empty(N, device=dev)
s.record()
for _ in range(n):
    K.linear_wgrad_x3(dY, N, [(X, Kd, 1)], M, ws)
    K.linear_wgrad_reduce(M, N, Kd, N, ws, col_map, gW, gb)
e.record()
torch.cuda.synchronize()
print(f"  + reduce: {s.elapsed_time(e) * 1e3 / n:.1f} us per layer")
