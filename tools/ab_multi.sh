#!/bin/bash
# Time microbench shapes under several library builds in one GPU call (same box).
# Usage: bash tools/ab_multi.sh <tag> "<lib1> <lib2> ..." <shape>...
set -u
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in $LIBS; do
    for s in "$@"; do
      f="$OUT/$(basename $lib)_${s}_${rep}.json"
      NERF_AMD_LIB=$lib timeout -k 10 120 python3 tools/microbench.py --only "$s" > "$f" 2>/dev/null \
        || { echo "failed $lib $s"; exit 1; }
      echo "$(basename $lib) $s $(tail -1 $f)"
    done
  done
done
