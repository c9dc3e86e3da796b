#!/bin/bash
# A/B the mip bench step across library variants on one box:
#   bash tools/ab_variants.sh <tag> <reps> <variant>...   (the in-tree library is always included first)
# A variant is a library path, or env:VAR=VALUE (the in-tree library with that environment setting).
# Writes gpurun_out/<tag>/<lib>_<rep>.json (bench.py's JSON line) and prints a summary line per run.
set -u
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
WL=${AB_WORKLOAD:-mip}   # AB_ARGS: extra bench.py arguments (e.g. --matmul-precision medium)
for rep in $(seq 1 "$REPS"); do
  for v in nerf-experiments_amd/nerf_amd/libnerf_amd.so "$@"; do
    lib=$v; envset=NERF_AB_NONE=1
    case "$v" in env:*) envset=${v#env:}; lib=nerf-experiments_amd/nerf_amd/libnerf_amd.so;; esac
    name=$(basename "$lib" .so); [ "$envset" != NERF_AB_NONE=1 ] && name="$name-$envset"
    f="$OUT/${name}_${rep}.json"
    env "$envset" NERF_AMD_LIB=$lib timeout -k 10 150 python3 bench.py --workload "$WL" --steps 60 --warmup 10 --no-cpu-baseline ${AB_ARGS:-} \
      --no-frame-roofline > "$f" 2> "$f.err" || { echo "failed $lib"; exit 1; }
    python3 - "$f" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
kf = d["kernel_functions"]
top = sorted(kf.items(), key=lambda kv: -kv[1]["ms_per_step"])[:6]
print(sys.argv[2].split("/")[-1], "%.3f ms/step" % d["ms_per_step"], "loss %.9g" % d["final_loss"],
      " ".join("%s=%.3f" % (k, v["ms_per_step"]) for k, v in top))
PY
  done
done
