#!/bin/bash
# Same-box A/B of library builds on the default bench step (kernel-function ms per step, loss):
# bash tools/ab_bench.sh <tag> <a.so> <b.so> [bench args...]
set -u
TAG=$1; A=$2; B=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$A" "$B"; do
    NERF_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-frame-roofline --steps 100 "$@" \
      > "$OUT/$(basename $lib)_$rep.json" 2> "$OUT/$(basename $lib)_$rep.err" || { echo "failed $lib"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), round(d['ms_per_step'],3), d['final_loss'], {k: round(v['ms_per_step'],3) for k,v in d['kernel_functions'].items() if v['ms_per_step']>0.3})" "$OUT/$(basename $lib)_$rep.json" "$(basename $lib)"
  done
done
