"""Transposed-read weight gradient vs fp64 over M (steps per split / ragged tails); bias error too."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nerf-experiments_amd"))
from nerf_amd import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
lib = K._lib.load()
for M in [8192, 8192 + 5, 12288, 16384, 32768, 65536, 100000, 100003]:
    N = Kc = 256
    dY = torch.randn(M, N, device=dev, generator=g)
    X = torch.ones(M, Kc, device=dev)
    ref = dY.double().T @ X.double()
    bound = dY.double().abs().T @ X.double().abs()
    ws = torch.empty((K.linear_wgrad_workspace_bytes(M, N, Kc) + 3) // 4, device=dev)
    col_map = torch.arange(Kc, dtype=torch.int32, device=dev)
    dW = torch.empty(N, Kc, device=dev)
    db = torch.empty(N, device=dev)
    K.linear_wgrad_x3_rows([(dY, [(X, Kc, 1)], M), (dY, [(X, Kc, 1)], 0)], N, ws)
    K.linear_wgrad_reduce(M, N, Kc, N, ws, col_map, dW, db)
    torch.cuda.synchronize()
    rel = ((dW.double() - ref).abs() / bound)
    splits = lib.nerf_wgrad_choose_splits(M, lib.nerf_wgrad_split_tiles(N, Kc)) if hasattr(lib, "nerf_wgrad_choose_splits") else -1
    print(f"M={M:6d} splits={splits}: max rel {rel.max().item():.3e}; db max err {(db.double() - dY.double().sum(0)).abs().max().item():.3e}")
