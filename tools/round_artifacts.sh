#!/bin/bash
# One GPU call producing a round's evidence: GPU tests, smoke, the default bench (mip, with CPU
# baseline), the other workload lines, rocprofv3 kernel stats of the default bench and the
# FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel trace only).  Usage: bash tools/round_artifacts.sh <tag>
set -u
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/gpu_tests.txt" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 \
  || { echo "smoke failed"; tail -20 "$OUT/smoke.txt"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
  || { echo "bench failed"; tail -20 "$OUT/bench_default.err"; exit 1; }
cat "$OUT/bench_default.json"
for w in n2v barf garf ingp; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { echo "bench $w failed"; tail -20 "$OUT/bench_$w.err"; exit 1; }
done
bash tools/profile_bench.sh "$OUT/prof_mip" --workload mip || exit 1
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
echo done
