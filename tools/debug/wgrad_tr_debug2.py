"""Which operand loses precision in the transposed-read weight gradient: X = ones with random dY,
then dY = ones with random X (M rows, one split or many); error relative to sum |dY| |X|."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nerf-experiments_amd"))
from nerf_amd import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
for M in [16, 64, 4096, 100003]:
    for mode in ("x_ones", "y_ones", "both"):
        N = Kc = 256
        dY = torch.randn(M, N, device=dev, generator=g) if mode != "y_ones" else torch.ones(M, N, device=dev)
        X = torch.randn(M, Kc, device=dev, generator=g) if mode != "x_ones" else torch.ones(M, Kc, device=dev)
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
        print(f"M={M:6d} {mode:6s}: max rel {rel.max().item():.3e} (2^{torch.log2(rel.max()).item():.1f}); "
              f"db max err {(db.double() - dY.double().sum(0)).abs().max().item():.3e}")
