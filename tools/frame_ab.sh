#!/bin/bash
# The frame roofline of the stand-alone encoding / compositing kernels (bench.py roofline_hbm_frame)
# across library variants: bash tools/frame_ab.sh <tag> <reps> <lib>...  (the in-tree library first)
set -u
TAG=$1; REPS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 $REPS); do
  for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so "$@"; do
    n=$(basename $lib .so)
    NERF_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/${n}_$rep.json 2> $O/${n}_$rep.err \
      || { echo "failed $lib"; tail -5 $O/${n}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${n}_$rep.json'))['roofline_hbm_frame'];print('$n', round(d['frac'],3), {k: round(v['gbs']) for k,v in d['per_kernel'].items()})"
  done
done
