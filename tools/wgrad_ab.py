"""Times the split-precision weight gradient (nerf_linear_wgrad_x3 + reduce) per layer shape
(HIP events, cold-ish inputs: a 512 MB buffer is written between launches) and saves dW / db;
with --compare it checks two builds' results bitwise (dW) and to fp32 summation order (db) —
how the LDS-DMA streamed single-tile kernel was A/B'd against the register-staged one it
replaced.

    python tools/wgrad_ab.py --out /tmp/a.pt          # build A
    python tools/wgrad_ab.py --out /tmp/b.pt --compare /tmp/a.pt   # build B
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nerf-experiments_amd"))
from nerf_amd import kernels as K  # noqa: E402

SHAPES = [  # (M, N, [(k, row_div)])
    (262144, 256, [(256, 1)]),
    (524288, 256, [(256, 1)]),
    (524288, 256, [(64, 1)]),
    (524288, 128, [(256, 1)]),
    (524288, 4, [(128, 1)]),
    (524288, 128, [(128, 1), (32, 128)]),
    (100003, 256, [(256, 1)]),
    (1000, 256, [(256, 1)]),
    # layers wider than one 256 x 256 tile (mip's 319 -> 256, 283 -> 128, 256 -> 257; GARF-like 512)
    (524288, 256, [(256, 1), (64, 1)]),
    (524288, 128, [(256, 1), (28, 128)]),
    (524288, 260, [(256, 1)]),
    (524288, 257, [(256, 1)]),         # the true row count: one 256 x 256 tile + row 256 (fp32 FMAs)
    (262144, 257, [(256, 1)]),
    (262144, 512, [(256, 1)]),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--compare")
    ap.add_argument("--rtol", type=float, default=0.0,
                    help="compare dW to this relative tolerance of its scale instead of bitwise "
                         "(builds that split M differently sum in another order)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    flush = torch.empty(128 * 1024 * 1024, device=dev)
    res = {}
    for M, N, ks in SHAPES:
        g = torch.Generator(device=dev).manual_seed(M + N)
        N4 = (N + 3) // 4 * 4                 # dY rows padded to 4 (zero columns), reduce over N4
        dY = torch.randn(M, N4, device=dev, generator=g)
        dY[:, N:] = 0
        segs = [((torch.randn((M + r - 1) // r, k, device=dev, generator=g)), k, r) for k, r in ks]
        Kp = sum(K.pad32(k) for k, _ in ks)
        ws = torch.empty((K.linear_wgrad_workspace_bytes(M, N4, Kp) + 3) // 4, device=dev)
        col_map = torch.arange(Kp, dtype=torch.int32, device=dev)
        dW = torch.empty(N, Kp, device=dev)
        db = torch.empty(N, device=dev)
        ts = []
        try:
            for it in range(12):
                flush.fill_(float(it))
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                K.linear_wgrad_x3(dY, N, segs, M, ws)
                e.record()
                K.linear_wgrad_reduce(M, N4, Kp, N, ws, col_map, dW, db)
                torch.cuda.synchronize()
                if it >= 2:
                    ts.append(s.elapsed_time(e) * 1e3)
        except RuntimeError as err:      # a build without this shape's path
            print(f"M{M}_N{N}: {err}", flush=True)
            continue
        ts.sort()
        us = ts[len(ts) // 2]
        nbytes = 4.0 * M * N + sum(4.0 * ((M + r - 1) // r) * k for k, r in ks)
        key = f"M{M}_N{N}_" + "_".join(f"{k}r{r}" for k, r in ks)
        print(f"{key}: {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s", flush=True)
        res[key] = (dW.cpu(), db.cpu())
    torch.save(res, args.out)
    if args.compare:
        ref = torch.load(args.compare, weights_only=True)
        for k, (w, b) in res.items():
            if k not in ref:
                continue
            w0, b0 = ref[k]
            if args.rtol == 0 and w.shape[0] == 257:
                # the 257th row is fp32 FMAs summed in a kernel-specific order
                same = torch.equal(w[:256], w0[:256]) and \
                    bool((w[256:] - w0[256:]).abs().max() <= 1e-6 * w0[256:].abs().max())
            else:
                same = torch.equal(w, w0) if args.rtol == 0 else \
                    bool((w - w0).abs().max() <= args.rtol * w0.abs().max())
            db_err = ((b - b0).abs().max() / b0.abs().max().clamp_min(1e-30)).item()
            what = "bitwise" if args.rtol == 0 else f"to {args.rtol:g} of scale"
            print(f"{k}: dW {what} {'equal' if same else 'DIFFERENT max ' + str((w - w0).abs().max().item())}, "
                  f"db rel {db_err:.2e}")
            assert same and db_err < 1e-5, k


if __name__ == "__main__":
    main()
