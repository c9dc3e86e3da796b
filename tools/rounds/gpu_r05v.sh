#!/bin/bash
# the ring's chunk barrier without the LDS drain (NERF_FUSED_RING_LGKM0=0) vs the product
set -u
O=gpurun_out/r05v; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
NERF_AMD_LIB=$L/var/lib_nolgkm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fused_composite.py tests/test_gpu_fused_encoding.py tests/test_gpu_barf_fit_precision.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
for lib in nerf_amd/libnerf_amd.so var/lib_nolgkm.so; do
  t=$(basename $lib .so)_$rep
  NERF_AMD_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), round(d['final_loss'],9), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n})"
done
done
