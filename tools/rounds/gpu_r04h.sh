#!/bin/bash
# Round-4 hash-grid corner arithmetic in 32 bits / fast fixed-point rounding: parity tests of every
# kernel that shares the corner code (stand-alone forward/backward, fused hash generation), a
# same-box A/B of the hash-grid kernels and the ingp step against the previous commit's hash-grid
# object (var/lib_hgprev.so), then the default bench line (frame render on the fused path).
# Usage (on the box): bash tools/gpu_r04h.sh <tag>
set -u
TAG=${1:-r04h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_hashgrid.py tests/test_gpu_fused_encoding.py tests/test_gpu_frame_render.py \
  -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "tests failed: $?"; tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for rep in 1 2; do
  for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so nerf-experiments_amd/var/lib_hgprev.so; do
    b=$(basename $lib .so)
    NERF_AMD_LIB=$lib timeout -k 10 120 python3 -u tools/hashgrid_bench.py --iters 10 > "$OUT/hg_${b}_$rep.txt" 2>&1 \
      || { echo "hashgrid bench $b failed"; tail "$OUT/hg_${b}_$rep.txt"; exit 1; }
    echo "hg $b: $(head -1 $OUT/hg_${b}_$rep.txt)"
    NERF_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload ingp --no-cpu-baseline --no-frame-roofline --steps 30 --warmup 5 \
      > "$OUT/ingp_${b}_$rep.json" 2> "$OUT/ingp_${b}_$rep.err" || { echo "ingp bench failed"; tail "$OUT/ingp_${b}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('ingp', sys.argv[2], round(d['value']/1e6,2), round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in d['kernel_functions'].items() if v['ms_per_step']>0.2})" "$OUT/ingp_${b}_$rep.json" $b
  done
done
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail "$OUT/bench_default.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('default', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'cpu', d['cpu_baseline']['value'], 'frame', d.get('frame_render',{}).get('ray_samples_per_s'), d.get('frame_render',{}).get('launches'))" "$OUT/bench_default.json"
echo done
