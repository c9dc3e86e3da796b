"""A/B the 30-step training-loss test under variations (diagnostic, GPU)."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nerf-experiments_amd"))


def run(tag):
    from nerf_amd import FourierFeatures, NerfInterpolation, NerfModel
    torch.manual_seed(0)
    model = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0)).to("cuda")
    ren = NerfInterpolation(0.1, 1 / 3, model, 64, "stratified_uniform", density_factor=(3.0, 7.0)).to("cuda")
    opt = ren.configure_optimizers()["optimizer"]
    B = 1024
    o = (torch.nn.functional.normalize(torch.randn(B, 3), dim=1) * 0.168).to("cuda")
    d = torch.nn.functional.normalize(-o.cpu() + torch.randn(B, 3) * 0.1, dim=1).to("cuda")
    pw = torch.full((B,), 1 / 555.56, device="cuda")
    target = torch.full((B, 3), 0.3, device="cuda")
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss, _ = ren.training_loss(o, d, pw, target)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    print(tag, losses[0], losses[-1], flush=True)


if __name__ == "__main__":
    run("as-is")
    orig = torch.optim.Adam

    def unfused(*a, **k):
        k.pop("fused", None)
        return orig(*a, **k)

    torch.optim.Adam = unfused
    run("unfused-adam")
    torch.optim.Adam = orig
    torch.autograd.function.FunctionCtx.set_materialize_grads = lambda self, v: None
    run("materialize")
    torch.optim.Adam = unfused
    run("unfused+materialize")
