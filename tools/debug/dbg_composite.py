"""Debug: fused compositing vs the stand-alone kernel on the same heads (which inputs differ)."""
import sys
import torch
sys.path.insert(0, "nerf-experiments_amd"); sys.path.insert(0, "tests")
torch.set_float32_matmul_precision("high")
import nerf_amd
from nerf_amd import kernels as K
from test_gpu_fused_composite import _model, _rays
DEV = "cuda"
model = _model(False)
S, B = 64, 256
o, d, t0, t1, pw = _rays(B, S)
dist = (t1 - t0).contiguous()
with torch.no_grad():
    heads = model.render_raw(o, d, pw, t0, t1, S, 1, 1)
    rgb0, w0 = K.composite_fwd(heads.dens_base.view(-1), 1, heads.color_base, 4, dist, B, S, 3.0, 7.0, True, 0.0)
    rgb1, w1 = model.render_composite(o, d, pw, t0, t1, S, 1, 1, dist, 3.0, 7.0)
torch.cuda.synchronize()
dw = (w0 - w1).abs()
print("rgb max diff", (rgb0 - rgb1).abs().max().item(), "w max diff", dw.max().item())
bad = (dw > 0).nonzero()
print("n differing weights", bad.shape[0], "first", bad[:10].tolist())
rows = (dw.max(1).values > 0).nonzero().flatten()
print("rays differing", rows.numel(), rows[:20].tolist())
# per-sample check: does w1 correspond to a composite of shifted / permuted inputs?
sig = torch.nn.functional.softplus(heads.dens_base.view(B, S).double(), threshold=8)
b = -sig * dist.double() * 21
T = torch.exp(torch.cumsum(b, 1) - b)
wd = T * (1 - torch.exp(b))
print("w0 vs fp64", (w0.double() - wd).abs().max().item(), " w1 vs fp64", (w1.double() - wd).abs().max().item())
r = rows[0].item() if rows.numel() else 0
print("ray", r, "w0", w0[r, :8].tolist()); print("ray", r, "w1", w1[r, :8].tolist())
print("sigma raw", heads.dens_base.view(B, S)[r, :8].tolist())
print("dist", dist[r, :8].tolist())
