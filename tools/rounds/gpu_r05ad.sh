#!/bin/bash
# the chain without its forward biases loaded a chunk ahead (product now) vs at the next chunk start (NERF_FUSED_BIAS_AHEAD=0)
set -u
O=gpurun_out/r05ad; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fused_composite.py tests/test_gpu_barf_fit_precision.py tests/test_gpu_mip_pose_feed.py tests/test_gpu_fullsize.py tests/test_gpu_fused_encoding.py tests/test_gpu_fused_w32.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
run() {
  t=$1_$2
  NERF_AMD_LIB=$L/var/lib_$1.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), round(d['final_loss'],9), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n})"
}
for r in 1 2; do run new $r && run old $r && run old $((r+2)) && run new $((r+2)) || exit 1; done
