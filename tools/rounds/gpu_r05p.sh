#!/bin/bash
# weight gradient: three register stages (var/lib_wg3.so) vs two (product), bitwise tests then A/B
set -u
O=gpurun_out/r05p; mkdir -p $O
export TMPDIR=/tmp
V=nerf-experiments_amd/var/lib_wg3.so
NERF_AMD_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad_tr.py tests/test_gpu_wgrad_rays.py -x -q --timeout 120 --timeout-method thread > $O/wg3_tests.txt 2>&1 || { tail -30 $O/wg3_tests.txt; exit 1; }
tail -2 $O/wg3_tests.txt
for rep in 1 2; do
for lib in nerf_amd/libnerf_amd.so var/lib_wg3.so; do
  t=$(basename $lib .so)_$rep
  NERF_AMD_LIB=nerf-experiments_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), {n:round(v['ms_per_step'],3) for n,v in k.items()})"
done
done
