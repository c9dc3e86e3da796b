#!/bin/bash
# the previous chunk's epilogue at k-steps 2-4 / 5-7 (NERF_FUSED_EPI0) vs 4-6 (product)
set -u
O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
for rep in 1 2; do
for lib in nerf_amd/libnerf_amd.so var/lib_epi2.so var/lib_epi5.so; do
  t=$(basename $lib .so)_$rep
  NERF_AMD_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), round(d['final_loss'],9), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n})"
done
done
