#!/bin/bash
# input-gradient chain store variants: pairs back to back (PAIR=4), single stores (PAIR=0), default
# cache policy for the chain's stores (AUX_DG=0) vs the product (PAIR=3, nt)
set -u
O=gpurun_out/r05s; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
for rep in 1 2; do
for lib in nerf_amd/libnerf_amd.so var/lib_PAIR4.so var/lib_PAIR0.so var/lib_AUXDG0.so; do
  t=$(basename $lib .so)_$rep
  NERF_AMD_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 40 --warmup 5 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n or 'tr_' in n})"
done
done
