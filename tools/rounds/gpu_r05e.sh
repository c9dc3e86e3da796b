#!/bin/bash
# round 5: weight-gradient column split (NERF_WGRAD_KSPLIT) parity + A/B, encode NT-store variant
set -u
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_encoding.py > $O/tests0.txt 2>&1 || { tail -30 $O/tests0.txt; exit 1; }
tail -1 $O/tests0.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_hashgrid.py \
  tests/test_gpu_fullsize.py tests/test_gpu_direct_sink.py tests/test_gpu_fused.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2; do
  for ks in 0 1; do
    NERF_WGRAD_KSPLIT=$ks timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 100 --warmup 10 > $O/bench_ks${ks}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_ks${ks}_$rep.json'));print('ks=$ks', d['ms_per_step'], d['kernel_functions'].get('linear_wgrad_x3_kernel'), d['kernels']['linear_wgrad_x3'])"
  done
done
for lib in nerf_amd/libnerf_amd.so var/lib_encold.so var/lib_encnt.so var/lib_compfast.so; do
  NERF_AMD_LIB=nerf-experiments_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/frame_$(basename $lib .so).json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/frame_$(basename $lib .so).json'));f=d['roofline_hbm_frame'];print('$lib', f['frac'], {k:round(v['gbs']) for k,v in f['per_kernel'].items()})"
done
for rep in 1 2; do
  for lib in nerf_amd/libnerf_amd.so var/lib_prio.so var/lib_sb2.so; do
    NERF_AMD_LIB=nerf-experiments_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 100 --warmup 10 > $O/bench_$(basename $lib .so)_$rep.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_$(basename $lib .so)_$rep.json'));k=d['kernel_functions'];print('$lib', d['ms_per_step'], k['mlp_fused_kernel<0>']['ms_per_step'], k['mlp_fused_kernel<1>']['ms_per_step'])"
  done
done
