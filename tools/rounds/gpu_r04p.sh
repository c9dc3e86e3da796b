#!/bin/bash
# Bucketed hash-grid backward: tests, A/B against the walk, and per-kernel times of the hash-grid
# bench (rocprofv3 kernel stats).  Usage (on the box): bash tools/gpu_r04p.sh <tag>
set -u
TAG=${1:-r04p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_r04i.sh $TAG ${VARIANTS:-bucket=NERF_HG_BUCKET=1@nerf_amd/libnerf_amd.so walk=NERF_HG_BUCKET=0@nerf_amd/libnerf_amd.so} || exit 1
NERF_HG_BUCKET=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 tools/hashgrid_bench.py --iters 5 > "$OUT/prof.log" 2>&1 || { echo "prof failed"; tail "$OUT/prof.log"; exit 1; }
python3 - "$OUT/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "hashgrid" in r["Name"]:
        print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY
