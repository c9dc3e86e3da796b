#!/bin/bash
# A/B two builds of the library in one GPU call on the same box (microbench shapes).
# Usage: bash tools/ab_lib.sh <tag> <variant.so> <shape>...
set -u
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so "$VAR"; do
    for s in "$@"; do
      NERF_AMD_LIB=$lib timeout -k 10 120 python3 tools/microbench.py --only "$s" > "$OUT/$(basename $lib)_${s}_${rep}.json" 2>&1 \
        || { echo "failed $lib $s"; exit 1; }
      echo "$(basename $lib) $s $(cat $OUT/$(basename $lib)_${s}_${rep}.json)"
    done
  done
done
