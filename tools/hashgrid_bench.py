"""Per-level timing of the hash-grid encoding kernels on ray samples shaped like bench.py's ingp
workload (rays from a sphere of radius 4 towards the origin, t in [2, 7], sorted per ray).

    python tools/hashgrid_bench.py [--rays 5120] [--spr 256] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nerf-experiments_amd"))
from nerf_amd import kernels  # noqa: E402
from nerf_amd.model_ingp import ingp_resolutions  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=5120)
    ap.add_argument("--spr", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--table", type=int, default=2 ** 16)
    ap.add_argument("--only", type=int, default=None, help="time just this level (for PMC passes)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    R, S, F, T = args.rays, args.spr, 2, args.table
    o = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1) * 4.0
    d = torch.nn.functional.normalize(-o + 0.5 * torch.randn(R, 3, generator=g), dim=-1)
    t0 = torch.sort(2.0 + 5.0 * torch.rand(R, S, generator=g), dim=-1).values
    t1 = t0 + 5.0 / S
    o, d, t0, t1 = (v.contiguous().to(dev) for v in (o, d, t0, t1))
    n = R * S
    res_all = ingp_resolutions(16, 16, 1600)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / args.iters

    def run(res):
        L = len(res)
        p = kernels.make_hashgrid_params(L, T, F, res, query=1)
        table = (torch.rand(kernels.hashgrid_table_rows(p), F, generator=g) * 2e-4 - 1e-4).to(dev)
        out = torch.empty(n, L * F, device=dev)
        gout = torch.randn(n, L * F, generator=g).to(dev)
        gt = torch.empty_like(table)
        ws = torch.empty(kernels.hashgrid_workspace_bytes(p, n) // 8 + 1, dtype=torch.int64, device=dev)
        kw = dict(ray_o=o, ray_d=d, t_start=t0, t_end=t1, n_samples=n, samples_per_ray=S)
        f = timed(lambda: kernels.hashgrid_fwd(p, table, out, **kw))
        b = timed(lambda: kernels.hashgrid_bwd(p, gout, gt, ws, **kw))
        return f, b

    if args.only is not None:
        f, b = run([res_all[args.only]])
        print(f"level {args.only}: fwd {f * 1e3:8.1f} us  bwd {b * 1e3:8.1f} us")
        return
    f, b = run(res_all)
    print(f"all {len(res_all)} levels: fwd {f * 1e3:8.1f} us  bwd {b * 1e3:8.1f} us  ({n} samples)")
    for l, r in enumerate(res_all):
        f, b = run([r])
        kind = "bij" if (r + 1) ** 3 <= T else "hash"
        print(f"level {l:2d} r={r:5d} {kind:4s}: fwd {f * 1e3:8.1f} us  bwd {b * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
