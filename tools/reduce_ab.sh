#!/bin/bash
# rocprofv3 kernel stats of a short mip bench under two library builds: the slab reduce's time
set -u
OUT=gpurun_out/${1:-red}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so "$@"; do
  n=$(basename $lib .so)
  NERF_AMD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-frame-roofline --steps 30 --warmup 5 > $OUT/$n.log 2>&1 || { echo "stats $n failed"; exit 1; }
  python3 - $OUT/$n $n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "reduce" in r["Name"] or "smalln" in r["Name"]:
        print(sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
