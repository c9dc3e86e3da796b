#!/bin/bash
# Round-4 hash-grid backward position records + pipelined walk: parity tests of the hash-grid paths,
# then a same-box A/B of the hash-grid kernels and the ingp step over (label, env, library) variants.
# Usage (on the box): bash tools/gpu_r04i.sh <tag> [label=ENV=VAL@lib ...]
set -u
TAG=${1:-r04i}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
LIBDIR=nerf-experiments_amd
timeout -k 10 600 python -u -m pytest tests/test_hashgrid.py tests/test_gpu_fused_encoding.py \
  -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { echo "tests failed: $?"; tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=("cur=X=0@nerf_amd/libnerf_amd.so" "nopos=NERF_HG_POS=0@nerf_amd/libnerf_amd.so" "pipe0=X=0@var/lib_hgpipe0.so")
for rep in 1 2; do
  for v in "${VARIANTS[@]}"; do
    label=${v%%=*}; rest=${v#*=}; envkv=${rest%@*}; lib=$LIBDIR/${rest##*@}
    env "$envkv" NERF_AMD_LIB=$lib timeout -k 10 120 python3 -u tools/hashgrid_bench.py --iters 10 > "$OUT/hg_${label}_$rep.txt" 2>&1 \
      || { echo "hashgrid bench $label failed"; tail "$OUT/hg_${label}_$rep.txt"; exit 1; }
    echo "hg $label: $(sed -n 2p $OUT/hg_${label}_$rep.txt)"
    env "$envkv" NERF_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload ingp --no-cpu-baseline --no-frame-roofline --steps 30 --warmup 5 \
      > "$OUT/ingp_${label}_$rep.json" 2> "$OUT/ingp_${label}_$rep.err" || { echo "ingp bench $label failed"; tail "$OUT/ingp_${label}_$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('ingp', sys.argv[2], round(d['value']/1e6,2), round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in d['kernel_functions'].items() if v['ms_per_step']>0.2})" "$OUT/ingp_${label}_$rep.json" $label
  done
done
echo done
