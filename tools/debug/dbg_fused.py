"""Debug helper: per-layer fused-forward outputs against the layer-by-layer path on a small
batch (prints the error pattern of the first rows / columns)."""
import math
import sys

import torch

sys.path.insert(0, "nerf-experiments_amd")


def main():
    import nerf_amd
    from nerf_amd import FourierFeatures, NerfModel, mlp, mlp_fused
    from nerf_amd.mlp import MLPFunction
    nerf_amd._lib.load()
    torch.set_float32_matmul_precision("high")
    torch.manual_seed(0)
    model = NerfModel(4, 256, True, True, 2, FourierFeatures(10, 2 * math.pi), FourierFeatures(4, 1.0)).cuda()
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    g = torch.Generator(device="cuda").manual_seed(11)
    pos = torch.zeros(M, 64, device="cuda")
    pos[:, :60] = torch.rand(M, 60, device="cuda", generator=g) * 2 - 1
    dirs = torch.zeros(M, 32, device="cuda")
    dirs[:, :24] = torch.rand(M, 24, device="cuda", generator=g) * 2 - 1
    plan = model._get_plan()
    res = {}
    for fused in (False, True):
        mlp_fused.ENABLED = fused
        mlp.CAPTURE = []
        MLPFunction.apply(plan, M, pos, dirs, 1, *plan.params())
        torch.cuda.synchronize()
        res[fused] = mlp.CAPTURE[0][0]
    for li, (x, y) in enumerate(zip(res[False], res[True])):
        n = plan.layers[li].N
        d = (x[:, :n] - y[:, :n]).abs()
        print(f"layer {li}: N={n} max err {d.max().item():.3e} scale {x[:, :n].abs().max().item():.3e}")
        if d.max().item() > 1e-3:
            bad = (d > 1e-3)
            print("  bad rows:", bad.any(1).nonzero().flatten()[:20].tolist(), "of", int(bad.any(1).sum()))
            print("  bad cols:", bad.any(0).nonzero().flatten()[:40].tolist(), "of", int(bad.any(0).sum()))
            print("  chunk max err:", [round(d[:, 16 * c:16 * c + 16].max().item(), 4) for c in range((n + 15) // 16)])
            print("  ref row0 c2:", x[0, 32:40].tolist())
            print("  fus row0 c2:", y[0, 32:40].tolist())
            print("  ref row0:", x[0, :8].tolist())
            print("  fus row0:", y[0, :8].tolist())
            b = plan.layers[li].module.bias
            print("  bias   :", b[:8].tolist())


if __name__ == "__main__":
    main()
