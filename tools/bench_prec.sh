#!/bin/bash
# One GPU call: the new / changed GPU tests first, the whole GPU suite, then the mip bench and the
# n2v bench at matmul precision high and medium.  Usage (on the box): bash tools/bench_prec.sh <tag> [first tests]
set -u
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > "$OUT/first_tests.txt" 2>&1 \
    || { echo "first tests failed: $?"; tail -40 "$OUT/first_tests.txt"; exit 1; }
  tail -2 "$OUT/first_tests.txt"
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 \
  || { echo "gpu tests failed: $?"; tail -40 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', d['final_loss'], {k: round(v['ms_per_step'],3) for k, v in d['kernel_functions'].items()})"; }
timeout -k 10 300 python -u bench.py --no-frame-roofline > "$OUT/bench_mip.json" 2> "$OUT/bench_mip.err" || { echo "bench mip failed"; tail -20 "$OUT/bench_mip.err"; exit 1; }
summ "$OUT/bench_mip.json" mip
for p in high medium; do
  timeout -k 10 300 python -u bench.py --workload n2v --matmul-precision $p --no-cpu-baseline --no-frame-roofline > "$OUT/bench_n2v_$p.json" 2> "$OUT/bench_n2v_$p.err" \
    || { echo "bench n2v $p failed"; tail -20 "$OUT/bench_n2v_$p.err"; exit 1; }
  summ "$OUT/bench_n2v_$p.json" n2v_$p
done
