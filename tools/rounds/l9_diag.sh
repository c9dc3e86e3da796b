#!/bin/bash
# per-launch weight-gradient times of one mip step under two library builds (rocprofv3 kernel trace)
set -u
OUT=gpurun_out/${1:-l9}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so "$@"; do
  n=$(basename $lib .so)
  NERF_AMD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/$n -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-frame-roofline --steps 10 --warmup 3 > $OUT/$n.log 2>&1 || { echo "trace $n failed"; exit 1; }
  python3 - $OUT/$n $n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
idx = [i for i, (k, _) in enumerate(seq) if "mlp_fused_kernel<1>" in k]
print(sys.argv[2], [round(d, 1) for k, d in seq[idx[-1]:idx[-1] + 30] if "wgrad" in k and "reduce" not in k])
PY
done
