#!/bin/bash
# composite pair-interleaved variants at one full frame
set -u
O=gpurun_out/r05h; mkdir -p $O
for rep in 1 2; do
for lib in nerf_amd/libnerf_amd.so var/lib_comppair.so var/lib_comppairfast.so; do
  NERF_AMD_LIB=nerf-experiments_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/frame_$(basename $lib .so)_$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/frame_$(basename $lib .so)_$rep.json'));f=d['roofline_hbm_frame'];print('$lib', round(f['frac'],3), {k:round(v['gbs']) for k,v in f['per_kernel'].items()})"
done
done
