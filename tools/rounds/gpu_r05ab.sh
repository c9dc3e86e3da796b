#!/bin/bash
# stand-alone encoding: rows per block 32 / 128 / 256 vs 64 (product), one full frame each
set -u
O=gpurun_out/r05ab; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
NERF_AMD_LIB=$L/var/lib_enc256.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "pe or encode or ipe" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
for v in prod enc32 enc128 enc256; do
  t=${v}_$rep
  NERF_AMD_LIB=$L/var/lib_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/frame_$t.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/frame_$t.json'));f=d['roofline_hbm_frame'];print('$t', round(f['frac'],3), {k:round(v['gbs']) for k,v in f['per_kernel'].items()})"
done
done
