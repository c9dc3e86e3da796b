#!/bin/bash
# chain stores as back-to-back half-line pairs (NERF_FUSED_PAIR=4, now the default): GPU suite, then
# interleaved A/B against the round's earlier default (PAIR=3) and two cache-policy variants
set -u
O=gpurun_out/r05t; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for rep in 1 2; do
for lib in nerf_amd/libnerf_amd.so var/lib_PAIR3.so var/lib_P4AUXDG0.so var/lib_P4AUX0.so; do
  t=$(basename $lib .so)_$rep
  NERF_AMD_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n or 'tr_' in n or 'x3_kernel' in n})"
done
done
