"""Structured-input check of the transposed-read weight gradient (NERF_WGRAD_TR=1): dY one-hot
rows, X[m][k] = 1000 m + k (exact in hi + lo bf16), so dW[n][k] = X[n][k] for n < M; prints where
the kernel's slab differs.  python tools/wgrad_tr_debug.py [M]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nerf-experiments_amd"))
from nerf_amd import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
for M in [int(a) for a in sys.argv[1:]] or [16, 32, 48, 256, 4096]:
    N, Kc = 256, 256
    dY = torch.zeros(M, N, device=dev)
    idx = torch.arange(M, device=dev)
    dY[idx, idx % N] = 1.0
    X = (1000.0 * (idx % 16).float().unsqueeze(1) + torch.arange(Kc, device=dev).float().unsqueeze(0)).contiguous()
    ref = dY.double().T @ X.double()
    ws = torch.empty((K.linear_wgrad_workspace_bytes(M, N, Kc) + 3) // 4, device=dev)
    col_map = torch.arange(Kc, dtype=torch.int32, device=dev)
    dW = torch.empty(N, Kc, device=dev)
    db = torch.empty(N, device=dev)
    K.linear_wgrad_x3_rows([(dY, [(X, Kc, 1)], M), (dY, [(X, Kc, 1)], 0)], N, ws)
    K.linear_wgrad_reduce(M, N, Kc, N, ws, col_map, dW, db)
    torch.cuda.synchronize()
    err = (dW.double() - ref).abs()
    bad = (err > 1e-3).nonzero()
    print(f"M={M}: max err {err.max().item():.4g}, bad entries {bad.shape[0]} of {N * Kc}")
    for n, k in bad[:12].tolist():
        print(f"   dW[{n}][{k}] = {dW[n, k].item():.3f}  want {ref[n, k].item():.3f}")
