#!/bin/bash
# forward epilogue at stage 3 (product now) vs 4 (before): GPU fused tests, four rotating repetitions
set -u
O=gpurun_out/r05y; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fused_composite.py tests/test_gpu_fused_encoding.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
run() {
  t=$(basename $1 .so)_$2
  NERF_AMD_LIB=$L/$1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), round(d['final_loss'],9), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n})"
}
run nerf_amd/libnerf_amd.so 1 && run var/lib_epi44.so 1 && run var/lib_epi44.so 2 && run nerf_amd/libnerf_amd.so 2 && \
run nerf_amd/libnerf_amd.so 3 && run var/lib_epi44.so 3 && run var/lib_epi44.so 4 && run nerf_amd/libnerf_amd.so 4
