#!/bin/bash
# round 5: per-wave encode kernel (parity + frame HBM A/B vs the block kernel, NT stores), composite
# prefetch depth 2 / fast exp, each at one full 800 x 800 frame (bench.py roofline_hbm_frame)
set -u
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_encoding.py \
  tests/test_gpu_fullsize.py tests/test_gpu_fused_composite.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
for lib in nerf_amd/libnerf_amd.so var/lib_encblock.so var/lib_encwnt.so var/lib_comppf2.so var/lib_compfast.so; do
  NERF_AMD_LIB=nerf-experiments_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/frame_$(basename $lib .so)_$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/frame_$(basename $lib .so)_$rep.json'));f=d['roofline_hbm_frame'];print('$lib', round(f['frac'],3), {k:round(v['gbs']) for k,v in f['per_kernel'].items()})"
done
done
