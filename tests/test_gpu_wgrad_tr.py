"""The register-staged, transposed-read weight gradient (linear_wgrad_x3_tr_kernel)
against the LDS-DMA stream kernel it replaces (NERF_WGRAD_TR=0, run in a child process: the switch
is read once per process).  Same 16-sample MFMA steps in sample order, same split: the weight
gradients are bitwise equal; the bias gradients, the 257th row and the per-ray dY sums come from
per-wave partials added in a fixed order, equal to fp32 summation order (1e-6 of scale).  Shapes
cover one and two row blocks, ragged splits (M not a multiple of 16), padded columns (N, K < 256,
a 60-wide segment padded to 64), inputs of <= 128 columns (JN = 1), the 257-row layer and the per-ray
route."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nerf-experiments_amd")

CASES = [  # (name, M0, M1, N, [(k, row_div)], rays S0/S1 or None)
    ("single_256", 100003, 0, 256, [(256, 1)], None),
    ("enc_64", 50000, 0, 256, [(60, 1)], None),
    ("narrow_n", 40000, 0, 128, [(256, 1)], None),
    ("two_blocks", 30000, 70001, 256, [(256, 1)], None),
    ("row257", 65536, 0, 257, [(256, 1)], None),
    ("row257_two_blocks", 32768, 65536, 257, [(256, 1)], None),
    ("rays", 64 * 300, 128 * 200, 256, [(256, 1)], (64, 128)),
    # inputs of <= 128 columns: the column blocks spread over the four SIMDs (JN = 1)
    ("narrow_k_row257", 65536, 0, 257, [(96, 1)], None),
    ("narrow_k_two_segs", 30000, 20001, 256, [(64, 1), (24, 1)], None),
]

SCRIPT = r"""
import json, sys, torch
sys.path.insert(0, {pkg!r})
from nerf_amd import kernels as K
torch.set_float32_matmul_precision("high")
dev = torch.device("cuda", 0)
out = {{}}
for name, M0, M1, N, ks, rays in {cases!r}:
    g = torch.Generator(device=dev).manual_seed(M0 + 7 * M1 + N)
    N4 = (N + 3) // 4 * 4
    def block(M):
        dY = torch.randn(M, N4, device=dev, generator=g)
        dY[:, N:] = 0
        segs = [(torch.randn((M + r - 1) // r, k, device=dev, generator=g), k, r) for k, r in ks]
        return dY, segs, M
    b0, b1 = block(M0), block(max(M1, 1))
    if M1 == 0:
        b1 = (b1[0], b1[1], 0)
    Kp = sum(K.pad32(k) for k, _ in ks)
    ws = torch.empty((K.linear_wgrad_workspace_bytes(M0 + M1, N4, Kp) + 3) // 4, device=dev)
    col_map = torch.arange(Kp, dtype=torch.int32, device=dev)
    dW = torch.empty(N, Kp, device=dev)
    db = torch.empty(N, device=dev)
    rs = None
    if rays is not None:
        S0, S1 = rays
        rs = torch.zeros(M0 // S0 + M1 // S1, N4, device=dev)
        K.linear_wgrad_x3_rays([b0, b1], N4 if N <= 256 else N, ws, rs, S0, S1)
    else:
        K.linear_wgrad_x3_rows([b0, b1], N4 if N <= 256 else N, ws)
    K.linear_wgrad_reduce(M0 + M1, N4, Kp, N, ws, col_map, dW, db)
    torch.cuda.synchronize()
    out[name] = (dW.cpu(), db.cpu(), rs.cpu() if rs is not None else None)
torch.save(out, sys.argv[1])
"""


def _run(tmp_path, tr: bool):
    f = tmp_path / ("tr.pt" if tr else "dma.pt")
    code = SCRIPT.format(pkg=PKG, cases=CASES)
    env = dict(os.environ, NERF_WGRAD_TR="1" if tr else "0")
    r = subprocess.run([sys.executable, "-c", code, str(f)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(f, weights_only=True)


def test_tr_kernel_equals_the_stream_kernel(tmp_path):
    new, ref = _run(tmp_path, True), _run(tmp_path, False)
    for name, *_ in CASES:
        (w, b, rs), (w0, b0, rs0) = new[name], ref[name]
        rows = min(256, w.shape[0])
        assert torch.equal(w[:rows], w0[:rows]), (name, (w[:rows] - w0[:rows]).abs().max().item())
        if w.shape[0] > 256:        # row 256: fp32 FMAs, per-wave partials
            assert (w[256:] - w0[256:]).abs().max() <= 1e-6 * w0[256:].abs().max(), name
        assert (b - b0).abs().max() <= 1e-6 * b0.abs().max(), name
        if rs0 is not None:
            assert (rs - rs0).abs().max() <= 1e-6 * rs0.abs().max(), name
