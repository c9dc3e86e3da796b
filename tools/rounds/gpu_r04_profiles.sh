#!/bin/bash
# Round-4 evidence, part 2: rocprofv3 kernel stats + PMC passes (tools/profile_bench.sh) for mip and
# ingp, and an L2 hit pass for ingp.  Usage (on the box): bash tools/gpu_r04_profiles.sh <tag>
set -u
TAG=${1:-r04x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/profile_bench.sh "$OUT/prof_mip" || { echo "mip profile failed"; exit 1; }
bash tools/profile_bench.sh "$OUT/prof_ingp" --workload ingp || { echo "ingp profile failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/prof_ingp/bench_l2" -o run --output-format csv \
  -- python3 bench.py --workload ingp --no-cpu-baseline --no-frame-roofline --steps 5 --warmup 2 > "$OUT/prof_ingp/bench_l2.log" 2>&1 \
  || { echo "ingp l2 pass failed"; exit 1; }
echo done
