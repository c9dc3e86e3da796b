#!/bin/bash
set -u
OUT=gpurun_out/fused1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?
tail -30 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_fused.json 2> $OUT/bench_fused.err || { tail -20 $OUT/bench_fused.err; exit 1; }
cat $OUT/bench_fused.json
NERF_FUSED=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_layer.json 2> $OUT/bench_layer.err || { tail -20 $OUT/bench_layer.err; exit 1; }
cat $OUT/bench_layer.json
