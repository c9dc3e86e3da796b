#!/bin/bash
set -u
O=gpurun_out/r05o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug/dbg_w32.py 32768 262144 > $O/dbg.txt 2>&1 || { cat $O/dbg.txt; exit 1; }
grep -v amdgpu.ids $O/dbg.txt | grep -E "M=|bad=[1-9]" 
timeout -k 10 200 python -u tools/debug/time_w32.py 524288 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_w32.py -x -q --timeout 120 --timeout-method thread > $O/w32_tests.txt 2>&1 || { tail -30 $O/w32_tests.txt; exit 1; }
tail -2 $O/w32_tests.txt
for w in 0 1; do
  NERF_FUSED_W32=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_w$w.json 2> $O/bench_w$w.err || { tail -20 $O/bench_w$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_w$w.json'));k=d['kernels'];print('w32=$w', round(d['ms_per_step'],3), {n:round(v['ms_per_step'],3) for n,v in k.items()})"
done
