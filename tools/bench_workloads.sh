#!/bin/bash
# One GPU call: the bench line of every workload (BASELINE.json configs[1..3]).
# Usage (on the box): bash tools/bench_workloads.sh <tag> [extra bench args]
set -u
TAG=${1:-workloads}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for w in n2v mip barf; do
  timeout -k 10 300 python -u bench.py --workload "$w" --no-cpu-baseline "$@" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { echo "bench $w failed: $?"; tail -30 "$OUT/bench_$w.err"; exit 1; }
  cat "$OUT/bench_$w.json"
done
