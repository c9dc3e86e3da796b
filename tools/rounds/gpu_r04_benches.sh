#!/bin/bash
# Round-4 evidence, part 1: GPU suite, smoke, the default bench line (CPU baseline and frame
# measurements) and the other workloads' lines.  Usage (on the box): bash tools/gpu_r04_benches.sh <tag>
set -u
TAG=${1:-r04x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 \
  || { echo "gpu tests failed: $?"; tail -40 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail "$OUT/bench_default.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('default', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'cpu', d['cpu_baseline']['value'], 'frame', d.get('frame_render',{}).get('ray_samples_per_s'), d.get('frame_render',{}).get('launches'))" "$OUT/bench_default.json"
for w in ingp n2v barf garf; do
  timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { echo "bench $w failed"; tail "$OUT/bench_$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in d['kernels'].items() if v['ms_per_step']>0.2})" "$OUT/bench_$w.json" $w
done
echo done
