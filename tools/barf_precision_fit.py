"""BARF pose-refinement fit in split ("high") vs exact fp32 ("highest") precision on the GPU
(tests/_barf_fit.py): prints one JSON line per run and the differences.
    python tools/barf_precision_fit.py [steps] [seeds]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-experiments_amd"), os.path.join(ROOT, "tests")]

import nerf_amd  # noqa: E402
from _barf_fit import run_fit  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
nerf_amd._lib.load()
for seed in range(seeds):
    r = {p: run_fit(p, steps, seed=seed) for p in ("high", "highest")}
    for p in r:
        print(json.dumps({"seed": seed, **r[p]}), flush=True)
    print(json.dumps({"seed": seed, "d_psnr_db": r["high"]["psnr"] - r["highest"]["psnr"],
                      "pose_error_ratio": r["high"]["pose_error"] / r["highest"]["pose_error"]}), flush=True)
