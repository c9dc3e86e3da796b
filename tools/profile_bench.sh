#!/bin/bash
# Kernel-trace stats + HBM traffic (FETCH_SIZE, WRITE_SIZE) + SQ instruction / cycle counters (each group
# in its own --pmc pass) of a bench
# command.  Usage: tools/profile_bench.sh <outdir> [bench args...]
set -u
OUT=${1:?outdir}; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-frame-roofline --steps 50 --warmup 10 "$@" > "$OUT/stats.log" 2>&1 \
  || { echo "stats pass failed"; exit 1; }
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $group -d "$OUT/bench_p$i" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-frame-roofline --steps 5 --warmup 2 "$@" > "$OUT/bench_p$i.log" 2>&1 \
    || { echo "pmc pass $i failed"; exit 1; }
done
echo done
