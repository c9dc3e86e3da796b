#!/bin/bash
# the tile-start encodings' tasks per sample (NERF_FUSED_GEN_TASKS 1) vs the flat task loop (0) and production; encoding tests on the new lib first
set -u
O=gpurun_out/r05ar; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
run() {
  t=$1_$2
  NERF_AMD_LIB=$L/var/lib_$1.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), round(d['final_loss'],9), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n})"
}
NERF_AMD_LIB=$L/var/lib_gt1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_encoding.py tests/test_gpu_fused.py tests/test_gpu_fused_composite.py -x -q --timeout 120 --timeout-method thread > $O/tests_gt1.txt 2>&1 || { tail -30 $O/tests_gt1.txt; exit 1; }
tail -2 $O/tests_gt1.txt
for v in prod gt1 gt0; do run $v 1 || exit 1; done
for v in gt1 gt0 prod; do run $v 2 || exit 1; done
for v in gt0 prod gt1; do run $v 3 || exit 1; done
for v in gt1 prod gt0; do run $v 4 || exit 1; done
