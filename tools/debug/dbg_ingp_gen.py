"""The hash-grid rows the fused forward generates (and stores) vs nerf_hashgrid_fwd on the same
samples, over repeated runs: which rows / levels differ."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nerf-experiments_amd"))
from nerf_amd import kernels as K  # noqa: E402
from nerf_amd import model_interpolation_architecture as A  # noqa: E402
from nerf_amd.model_ingp import FourierFeatures, INGPEncoding, NaiveINGP  # noqa: E402
from nerf_amd import model_ingp as M  # noqa: E402

M.FUSE_HASH = True          # the in-kernel hash generation is opt-in (NERF_FUSE_HASH=1)

dev = torch.device("cuda", 0)
torch.set_float32_matmul_precision("high")
torch.manual_seed(0)
enc = INGPEncoding(1600, 16, 2 ** 16, 2, 16)
ren = NaiveINGP(2, 7, 192, 64, enc, FourierFeatures(4), 8, 256).to(dev)
g = torch.Generator().manual_seed(5)
S, B = 64, 4096
model = ren.model_coarse
o = (torch.randn(B, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 - torch.tensor([0.0, 0.0, 1.0]), dim=1).to(dev)
t = (torch.linspace(2.0, 7.0 - 5.0 / S, S).repeat(B, 1) + torch.rand(B, S, generator=g) * (5.0 / S)).to(dev).contiguous()
t_end = ren._intervals(t)
stash = []
orig = INGPEncoding.encode_rays


def spy(self, *a, **k):
    out = orig(self, *a, **k)
    stash.append(out)
    return out


INGPEncoding.encode_rays = spy
ref = None
with torch.no_grad():
    A.FUSE_ENCODINGS = False
    model.render_raw(o, d, None, t, t_end, S, 0, 1)
    torch.cuda.synchronize()
    ref = stash[-1].clone()
    A.FUSE_ENCODINGS = True
    for rep in range(3):
        model.render_raw(o, d, None, t, t_end, S, 0, 1)
        torch.cuda.synchronize()
        rows = stash[-1]
        diff = (rows[:, :32] != ref[:, :32])
        bad = diff.nonzero()
        print(f"run {rep}: rows differing {diff.any(1).sum().item()} of {rows.shape[0]}, entries {bad.shape[0]}, "
              f"max {(rows[:, :32] - ref[:, :32]).abs().max().item():.3e}, pad nonzero {(rows[:, 32:] != 0).sum().item()}")
        if bad.shape[0]:
            r = bad[:, 0]
            wv = rows[bad[:, 0], bad[:, 1]]
            print("   wrong entries NaN (never stored):", int(torch.isnan(wv).sum()), "of", bad.shape[0],
                  "| columns", sorted(set(bad[:, 1].tolist())), "| wave", sorted(set(((r % 128) // 16).tolist())),
                  "| sample in wave", sorted(set((r % 16).tolist())))
            print("   samples", r[:8].tolist(), "cols", bad[:8, 1].tolist(), "sample mod 128:",
                  sorted(set((r % 128).tolist()))[:20], "tile-wave:", sorted(set(((r % 128) // 16).tolist())))

# where do the wrong values come from?  search the reference features for each wrong value
rows = stash[-1]
bad = (rows[:, :32] != ref[:, :32]).nonzero()
flat = ref[:, :32].reshape(-1)
for n, col in bad[:6].tolist():
    v = rows[n, col]
    hits = (flat == v).nonzero().view(-1)
    print(f"sample {n} col {col}: wrong {v.item():.6e} right {ref[n, col].item():.6e}; equals ref at",
          [(int(h) // 32, int(h) % 32) for h in hits[:5]])
