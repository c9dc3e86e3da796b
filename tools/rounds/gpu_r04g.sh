#!/bin/bash
# Hash-grid backward A/B: the run-length merged walk (default) vs the strided walk, parity first.
set -u
OUT=gpurun_out/${1:-r04g}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_hashgrid.py -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/tests.txt" 2>&1 \
  || { echo "tests failed"; tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
for m in 1 0; do
  NERF_HG_MERGE=$m timeout -k 10 120 python3 -u tools/hashgrid_bench.py --iters 10 > "$OUT/hg_merge$m.txt" 2>&1 || { echo "hg bench failed"; exit 1; }
  echo "merge=$m"; grep -v amdgpu.ids "$OUT/hg_merge$m.txt" | head -6
  NERF_HG_MERGE=$m timeout -k 10 120 python3 -u tools/hashgrid_bench.py --iters 10 --spr 64 --rays 5120 > "$OUT/hg_merge${m}_coarse.txt" 2>&1 || { echo "hg bench failed"; exit 1; }
  grep -v amdgpu.ids "$OUT/hg_merge${m}_coarse.txt" | head -1
done
