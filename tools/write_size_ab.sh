#!/bin/bash
# WRITE_SIZE per launch of the fused kernels under library variants (rocprofv3 --pmc, kernel trace only)
set -u
OUT=gpurun_out/${1:-ws}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so "$@"; do
  n=$(basename $lib .so)
  NERF_AMD_LIB=$lib timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/$n -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-frame-roofline --steps 3 --warmup 1 > $OUT/$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
  python3 - $OUT/$n $n <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "mlp_fused_kernel" in r["Kernel_Name"]:
        k = "fwd" if "<0>" in r["Kernel_Name"] else "chain"
        d[k].append(float(r["Counter_Value"]) * 1024 / 1e9)
print(sys.argv[2], {k: [round(x, 2) for x in v] for k, v in d.items()})
PY
done
