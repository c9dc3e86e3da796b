#!/bin/bash
# One GPU call producing a round's evidence: GPU tests, smoke, the default bench (mip, with CPU
# baseline and the frame roofline), the other workload lines (n2v also at matmul precision medium),
# the HBM rate probe, rocprofv3 kernel stats of the default bench and its PMC passes (separate runs,
# kernel trace only: tools/profile_bench.sh).  Usage: bash tools/round_artifacts.sh <tag>
set -u
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/gpu_tests.txt" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 \
  || { echo "smoke failed"; tail -20 "$OUT/smoke.txt"; exit 1; }
cat "$OUT/smoke.txt"
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
  || { echo "bench failed"; tail -20 "$OUT/bench_default.err"; exit 1; }
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', {k: round(v['ms_per_step'],3) for k, v in d['kernel_functions'].items()})"; }
summ "$OUT/bench_default.json" mip
for w in n2v barf garf ingp; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { echo "bench $w failed"; tail -20 "$OUT/bench_$w.err"; exit 1; }
  summ "$OUT/bench_$w.json" $w
done
timeout -k 10 300 python -u bench.py --workload n2v --matmul-precision medium --no-cpu-baseline \
  > "$OUT/bench_n2v_medium.json" 2> "$OUT/bench_n2v_medium.err" || { echo "bench n2v medium failed"; exit 1; }
summ "$OUT/bench_n2v_medium.json" n2v_medium
timeout -k 10 120 python -u tools/hbm_probe.py > "$OUT/hbm_probe.json" 2> "$OUT/hbm_probe.err" || { echo "probe failed"; exit 1; }
cat "$OUT/hbm_probe.json"
bash tools/profile_bench.sh "$OUT/prof_mip" --workload mip || exit 1
bash tools/profile_bench.sh "$OUT/prof_n2v_medium" --workload n2v --matmul-precision medium || exit 1
echo done
