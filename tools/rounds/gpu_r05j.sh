#!/bin/bash
# 32-sample-wave forward (NERF_FUSED_W32): parity tests, then interleaved bench A/B against the
# 16-sample kernel
set -u
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_w32.py -x -v --timeout 120 --timeout-method thread \
  > $O/w32_tests.txt 2>&1 || { tail -40 $O/w32_tests.txt; exit 1; }
tail -3 $O/w32_tests.txt
for rep in 1 2; do
for w in 0 1; do
  NERF_FUSED_W32=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 100 --warmup 10 \
    > $O/bench_w${w}_$rep.json 2> $O/bench_w${w}_$rep.err || { tail -20 $O/bench_w${w}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_w${w}_$rep.json'));k=d['kernels'];print('w32=$w', round(d['ms_per_step'],3), {n:round(v['ms_per_step'],3) for n,v in k.items()})"
done
done
