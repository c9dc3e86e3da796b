"""Times the register-staged weight-gradient kernel (linear_wgrad_x3_tr_kernel) alone at the mip
bench's merged row count (M = 786432: coarse + fine rows of 4096 rays) for the trunk's shapes, with
HIP events on the stream the kernel runs on.  Pick the library with NERF_AMD_LIB (diagnostic
NERF_WT_DIAG_* builds need NERF_ALLOW_DIAG_BUILD=1).  Prints one JSON line.
Usage: python tools/wgrad_tr_diag.py [M]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nerf-experiments_amd"))
from nerf_amd import kernels as K  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 786432
dev = torch.device("cuda:0")
out = {"lib": os.path.basename(os.environ.get("NERF_AMD_LIB", "libnerf_amd.so")), "M": M}
dY = torch.randn(M, 256, device=dev)
for kd in (256, 96, 32):
    X = torch.randn(M, kd, device=dev)
    ws = torch.empty((K.linear_wgrad_workspace_bytes(M, 256, kd) + 3) // 4, device=dev)
    for _ in range(3):
        K.linear_wgrad_x3(dY, 256, [(X, kd, 1)], M, ws)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    s.record()
    for _ in range(n):
        K.linear_wgrad_x3(dY, 256, [(X, kd, 1)], M, ws)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / n
    out[f"K{kd}_us"] = round(us, 1)
    out[f"K{kd}_TBps"] = round(M * 4 * (256 + kd) / us / 1e6, 3)
    del X, ws
print(json.dumps(out))
