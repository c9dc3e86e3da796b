#!/usr/bin/env python3
"""Per-kernel, per-shape timing of the nerf_amd C-ABI kernels (HIP events on the
launch stream, median of repeated launches).  Shapes are the layers of the
bench workload (naive-to-vanilla NerfModel at 4096 rays x 64 samples).

    python tools/microbench.py [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-experiments_amd"))

from nerf_amd import kernels as K  # noqa: E402
from nerf_amd._lib import NERF_EPI_BIAS, NERF_EPI_MASK, NERF_EPI_MASKBITS, NERF_EPI_MASKOUT, NERF_EPI_RELU  # noqa: E402

NERF_EPI_NO_PERSIST = 256
NERF_EPI_NARROW_TILE = 512

DEV = torch.device("cuda", 0)


def time_it(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def bench_linear(M, N, ks, rd, epi=NERF_EPI_BIAS | NERF_EPI_RELU, x3=False):
    segs = [(torch.randn((M + r - 1) // r, k, device=DEV), k, r) for k, r in zip(ks, rd)]
    Kt = sum(K.pad32(k) for k in ks)
    W = torch.randn(K.pad128(N), Kt, device=DEV) * 0.05
    b = torch.randn(N, device=DEV)
    ldo = (N + 3) // 4 * 4
    out = torch.empty(M, ldo, device=DEV)
    aux = torch.randn(M, ldo, device=DEV) if epi & NERF_EPI_MASK else None
    if epi & NERF_EPI_MASKBITS:
        aux = torch.randint(0, 256, (M, 32), dtype=torch.uint8, device=DEV)
    fl = 2.0 * M * N * sum(ks)
    if x3:
        Wh = W.bfloat16()
        Wx = K.interleave_x3(Wh, (W - Wh.float()).bfloat16())
        ms = time_it(lambda: K.linear_fwd_x3(segs, M, Wx, Kt, N, b, out, epi, aux=aux))
        r = {"kernel": "linear_nt_x3", "M": M, "N": N, "K": ks, "ms": ms, "tflops": fl / ms / 1e9}
        ms_np = time_it(lambda: K.linear_fwd_x3(segs, M, Wx, Kt, N, b, out, epi | NERF_EPI_NO_PERSIST, aux=aux))
        r["tflops_no_persist"] = fl / ms_np / 1e9
        if 128 < N <= 256:
            ms_n = time_it(lambda: K.linear_fwd_x3(segs, M, Wx, Kt, N, b, out, epi | NERF_EPI_NARROW_TILE, aux=aux))
            r["tflops_narrow_tile"] = fl / ms_n / 1e9
        return r
    ms = time_it(lambda: K.linear_fwd(segs, M, W, Kt, N, b, out, epi, aux=aux))
    r = {"kernel": "linear_nt", "M": M, "N": N, "K": ks, "ms": ms, "tflops": fl / ms / 1e9}
    # A/B in the same process: one tile per workgroup (no persistence)
    ms_np = time_it(lambda: K.linear_fwd(segs, M, W, Kt, N, b, out, epi | NERF_EPI_NO_PERSIST, aux=aux))
    r["tflops_no_persist"] = fl / ms_np / 1e9
    return r


def bench_wgrad(M, N, ks, rd, x3=False):
    segs = [(torch.randn((M + r - 1) // r, k, device=DEV), k, r) for k, r in zip(ks, rd)]
    Kt = sum(K.pad32(k) for k in ks)
    N4 = (N + 3) // 4 * 4
    dY = torch.randn(M, N4, device=DEV)
    ws = torch.empty((K.linear_wgrad_workspace_bytes(M, N4, Kt) + 3) // 4, device=DEV)
    dW = torch.empty(N, Kt, device=DEV)
    db = torch.empty(N, device=DEV)
    cm = torch.arange(Kt, dtype=torch.int32, device=DEV)
    wg = K.linear_wgrad_x3 if x3 else K.linear_wgrad
    ms1 = time_it(lambda: wg(dY, N4, segs, M, ws))
    ms2 = time_it(lambda: K.linear_wgrad_reduce(M, N4, Kt, N, ws, cm, dW, db))
    fl = 2.0 * M * N * sum(ks)
    return {"kernel": "linear_wgrad_x3" if x3 else "linear_wgrad", "M": M, "N": N, "K": ks, "ms": ms1, "reduce_ms": ms2,
            "tflops": fl / ms1 / 1e9}


def bench_composite(B, S):
    head = torch.randn(B * S, 4, device=DEV)
    dist = torch.rand(B, S, device=DEV) * 0.01
    ms = time_it(lambda: K.composite_fwd(head[:, 3:], 4, head, 4, dist, B, S, 3.0, 7.0, True))
    algo = B * S * (16 + 4 + 4) + B * 12
    g = torch.randn(B, 3, device=DEV)
    gh = torch.zeros_like(head)
    ms_b = time_it(lambda: K.composite_bwd(head[:, 3:], 4, head, 4, dist, B, S, 3.0, 7.0, True, 0.0, g, None,
                                           gh[:, 3:], 4, gh, 4))
    algo_b = B * S * (16 + 4 + 16) + B * 12
    return {"kernel": "composite", "B": B, "S": S, "fwd_ms": ms, "fwd_GBs_algo": algo / ms / 1e6,
            "bwd_ms": ms_b, "bwd_GBs_algo": algo_b / ms_b / 1e6}


def bench_encode(B, S):
    o = torch.randn(B, 3, device=DEV)
    d = torch.nn.functional.normalize(torch.randn(B, 3, device=DEV), dim=1)
    t0 = torch.rand(B, S, device=DEV)
    t1 = t0 + 0.01
    p = K.make_pe_params(0, 10, False, 2 * math.pi, query=1)
    ms = time_it(lambda: K.encode_fwd(p, 60, ray_o=o, ray_d=d, t_start=t0, t_end=t1, n_samples=B * S,
                                      samples_per_ray=S, n_rays=B, out_ld=64, device=DEV))
    algo = B * S * (8 + 64 * 4)
    return {"kernel": "encode", "B": B, "S": S, "ms": ms, "GBs_algo": algo / ms / 1e6}


def bench_resample(B, Kb, N):
    tc = torch.sort(torch.rand(B, Kb, device=DEV), dim=1).values
    w = torch.rand(B, Kb, device=DEV)
    dist = torch.rand(B, Kb, device=DEV) * 0.01
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    ms = time_it(lambda: K.resample_pdf(tc, w, dist, N, 0, 0.0, 1.0, 1, 0, st))
    algo = B * (12 * Kb + 8 * N)
    return {"kernel": "resample", "B": B, "K": Kb, "N": N, "ms": ms, "GBs_algo": algo / ms / 1e6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--hbm", action="store_true", help="only the compositing / encoding kernels")
    ap.add_argument("--only", help="run one shape repeatedly for counter collection: nt256 | nt256mask | wgrad256")
    args = ap.parse_args()
    M = 4096 * 64
    res = []
    if args.only:
        fn = {"nt256": lambda: bench_linear(M, 256, (256,), (1,)),
              "nt256mask": lambda: bench_linear(M, 256, (256,), (1,), NERF_EPI_MASK),
              "wgrad256": lambda: bench_wgrad(M, 256, (256,), (1,)),
              "nt256x3": lambda: bench_linear(M, 256, (256,), (1,), x3=True),
              "nt256maskx3": lambda: bench_linear(M, 256, (256,), (1,), NERF_EPI_MASK, x3=True),
              "nt256bitsx3": lambda: bench_linear(M, 256, (256,), (1,), NERF_EPI_MASK | NERF_EPI_MASKBITS, x3=True),
              "wgrad256x3": lambda: bench_wgrad(M, 256, (256,), (1,), x3=True),
              "encode": lambda: bench_encode(4096, 64),
              "encode_big": lambda: bench_encode(65536, 128)}[args.only]
        print(json.dumps(fn()))
        return
    if args.hbm:  # the HBM-bound kernels at bench size and at sizes where launch latency is amortised
        res = [bench_composite(4096, 64), bench_composite(65536, 64), bench_composite(65536, 128),
               bench_composite(262144, 128), bench_encode(4096, 64), bench_encode(65536, 128)]
        for r in res:
            print(json.dumps(r))
        if args.json:
            with open(args.json, "w") as f:
                json.dump(res, f, indent=1)
        return
    for x3 in (False, True):
        # forward layers of the bench model
        res.append(bench_linear(M, 256, (64,), (1,), x3=x3))
        res.append(bench_linear(M, 256, (256,), (1,), x3=x3))
        res.append(bench_linear(M, 256, (256, 64), (1, 1), x3=x3))
        res.append(bench_linear(M, 128, (256, 32), (1, 64), x3=x3))
        if not x3:
            res.append(bench_linear(M, 4, (128,), (1,), NERF_EPI_BIAS))
        # input-gradient layers
        res.append(bench_linear(M, 256, (256,), (1,), NERF_EPI_MASK, x3=x3))
        res.append(bench_linear(M, 256, (256,), (1,), NERF_EPI_MASK | NERF_EPI_MASKBITS, x3=x3))
        res.append(bench_linear(M, 128, (4,), (1,), NERF_EPI_MASK | NERF_EPI_MASKBITS, x3=x3))
        res.append(bench_linear(M, 256, (128,), (1,), 0, x3=x3))
        # weight gradients
        res.append(bench_wgrad(M, 256, (256,), (1,), x3=x3))
        res.append(bench_wgrad(M, 256, (256, 64), (1, 1), x3=x3))
        res.append(bench_wgrad(M, 128, (256, 32), (1, 64), x3=x3))
        res.append(bench_wgrad(M, 4, (128,), (1,), x3=x3))
    res.append(bench_composite(4096, 64))
    res.append(bench_composite(65536, 128))
    res.append(bench_encode(4096, 64))
    res.append(bench_encode(65536, 128))
    res.append(bench_resample(65536, 64, 192))
    for r in res:
        print(json.dumps(r))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
