#!/bin/bash
# the next chunk's LDS-DMA issued after k-step 0 / 1 (NERF_FUSED_DMA_STAGE 1 / 2) vs before k-step 0
set -u
O=gpurun_out/r05aa; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
NERF_AMD_LIB=$L/var/lib_dma2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fused_composite.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
run() {
  t=$1_$2
  NERF_AMD_LIB=$L/var/lib_$1.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), round(d['final_loss'],9), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n})"
}
for v in prod dma1 dma2; do run $v 1 || exit 1; done
for v in dma2 prod dma1; do run $v 2 || exit 1; done
for v in dma1 dma2 prod; do run $v 3 || exit 1; done
