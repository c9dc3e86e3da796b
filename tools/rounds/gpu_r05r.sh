#!/bin/bash
# 16-sample forward: diagnostic builds (no weight stream / no per-chunk barrier / no stores)
set -u
O=gpurun_out/r05r; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
for rep in 1 2; do
for lib in nerf_amd/libnerf_amd.so var/lib_w16_NODMA.so var/lib_w16_NOBARRIER.so var/lib_w16_NOSTORE.so; do
  t=$(basename $lib .so)_$rep
  NERF_ALLOW_DIAG_BUILD=1 NERF_AMD_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 40 --warmup 5 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n})"
done
done
