#!/bin/bash
# One GPU call: parity tests, smoke, default bench.  Every GPU step has its own time limit
# and the chain stops at the first failure.  Usage (on the box): bash tools/gpu_check.sh [tag] [test args]
set -u
TAG=${1:-check}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" \
  > "$OUT/gpu_tests.txt" 2>&1 || { echo "gpu tests failed: $?"; tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -3 "$OUT/gpu_tests.txt"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 \
  || { echo "smoke failed: $?"; tail -30 "$OUT/smoke.txt"; exit 1; }
cat "$OUT/smoke.txt"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed: $?"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['final_loss'], {k: round(v['ms_per_step'],3) for k, v in d['kernel_functions'].items()})"
