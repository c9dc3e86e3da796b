#!/bin/bash
# Round-4 check of the register-staged weight streams: parity tests of the touched kernels, the
# weight-gradient A/B (LDS-DMA stream vs register-staged transposed reads) and a same-box A/B of
# the fused kernels (default build vs NERF_FUSED_UNROLL2=0 vs the LDS-DMA weight ring) on the
# default mip step.  Usage (on the box): bash tools/gpu_r04d.sh <tag>
set -u
TAG=${1:-r04d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_wgrad_tr.py tests/test_gpu_wgrad_rays.py tests/test_gpu_direct_sink.py \
  tests/test_gpu_fused.py tests/test_gpu_fused_composite.py tests/test_gpu_fused_encoding.py tests/test_hashgrid.py \
  -x -q --timeout 240 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "tests failed: $?"; tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
NERF_WGRAD_TR=0 timeout -k 10 200 python -u tools/wgrad_ab.py --out "$OUT/a.pt" > "$OUT/ab_dma.txt" 2>&1 \
  || { echo "ab dma failed"; tail "$OUT/ab_dma.txt"; exit 1; }
timeout -k 10 200 python -u tools/wgrad_ab.py --out "$OUT/b.pt" --compare "$OUT/a.pt" > "$OUT/ab_tr.txt" 2>&1 \
  || { echo "ab tr failed"; tail "$OUT/ab_tr.txt"; exit 1; }
paste "$OUT/ab_dma.txt" "$OUT/ab_tr.txt" | cut -c1-220
for rep in 1 2; do
  for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so nerf-experiments_amd/var/lib_head.so nerf-experiments_amd/var/lib_unroll0.so nerf-experiments_amd/var/lib_wreg0.so; do
    NERF_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-frame-roofline --steps 100 \
      > "$OUT/$(basename $lib)_$rep.json" 2> "$OUT/$(basename $lib)_$rep.err" || { echo "failed $lib"; tail "$OUT/$(basename $lib)_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), round(d['ms_per_step'],3), d['final_loss'], {k: round(v['ms_per_step'],3) for k,v in d['kernel_functions'].items() if v['ms_per_step']>0.3})" "$OUT/$(basename $lib)_$rep.json" "$(basename $lib)"
  done
done
timeout -k 10 300 python3 -u bench.py --workload ingp --no-cpu-baseline --no-frame-roofline --steps 30 --warmup 5 \
  > "$OUT/bench_ingp.json" 2> "$OUT/bench_ingp.err" || { echo "ingp bench failed"; tail "$OUT/bench_ingp.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('ingp', round(d['value']/1e6,2), round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in d['kernels'].items()})" "$OUT/bench_ingp.json"
for v in "default" "fwd_thread" "parts16k"; do
  case $v in
    default) env_lib=""; lib=nerf-experiments_amd/nerf_amd/libnerf_amd.so ;;
    fwd_thread) env_lib="NERF_HG_FWD_LEVEL=0"; lib=nerf-experiments_amd/nerf_amd/libnerf_amd.so ;;
    parts16k) env_lib=""; lib=nerf-experiments_amd/var/lib_hgp16k.so ;;
  esac
  env $env_lib NERF_AMD_LIB=$lib timeout -k 10 120 python3 -u tools/hashgrid_bench.py --iters 10 > "$OUT/hg_$v.txt" 2>&1 \
    || { echo "hashgrid bench $v failed"; tail "$OUT/hg_$v.txt"; exit 1; }
  echo "$v: $(head -1 $OUT/hg_$v.txt)"
done
