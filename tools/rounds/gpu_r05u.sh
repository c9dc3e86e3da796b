#!/bin/bash
# chain pairs back to back (PAIR=4, chunk -1 guard fixed) vs the default (PAIR=3): the tests that
# caught the unguarded form, then interleaved A/B
set -u
O=gpurun_out/r05u; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
NERF_AMD_LIB=$L/var/lib_PAIR4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_barf_fit_precision.py tests/test_gpu_fused.py tests/test_gpu_fused_composite.py tests/test_gpu_mip_pose_feed.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $O/p4_tests.txt 2>&1 || { tail -30 $O/p4_tests.txt; exit 1; }
tail -2 $O/p4_tests.txt
for rep in 1 2; do
for lib in nerf_amd/libnerf_amd.so var/lib_PAIR4.so; do
  t=$(basename $lib .so)_$rep
  NERF_AMD_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), round(d['final_loss'],9), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n or 'tr_' in n})"
done
done
