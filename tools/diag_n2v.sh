#!/bin/bash
set -u
O=gpurun_out/r06h; mkdir -p $O
for rep in 1 2; do
for v in prod nodma nobar; do
  lib=nerf-experiments_amd/nerf_amd/libnerf_amd.so; [ $v != prod ] && lib=nerf-experiments_amd/var/lib_$v.so
  for p in high medium; do
    NERF_ALLOW_DIAG_BUILD=1 NERF_AMD_LIB=$lib timeout -k 10 150 python3 bench.py --workload n2v --matmul-precision $p --steps 60 --warmup 10 --no-cpu-baseline --no-frame-roofline > $O/${v}_${p}_$rep.json 2> $O/${v}_${p}_$rep.err || { echo fail $v $p; tail -5 $O/${v}_${p}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_${p}_$rep.json'));print('$v $p', round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in d['kernel_functions'].items() if 'fused' in k})"
  done
done
done
