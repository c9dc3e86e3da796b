#!/bin/bash
# Small-N weight-gradient kernel: parity tests, per-shape timing against the 128-tile kernel, step A/B.
set -u
OUT=gpurun_out/${1:-smalln}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
NERF_WGRAD_SMALLN=0 timeout -k 10 200 python -u tools/wgrad_ab.py --out /tmp/wa.pt > $OUT/wgrad_tile.txt 2>&1 || { echo "wgrad A failed"; tail $OUT/wgrad_tile.txt; exit 1; }
timeout -k 10 200 python -u tools/wgrad_ab.py --out /tmp/wb.pt --compare /tmp/wa.pt --rtol 1e-5 > $OUT/wgrad_smalln.txt 2>&1 || { echo "wgrad B failed"; tail $OUT/wgrad_smalln.txt; exit 1; }
grep "N4_" $OUT/wgrad_tile.txt $OUT/wgrad_smalln.txt
bash tools/ab_variants.sh ${1:-smalln}_ab 2 env:NERF_WGRAD_SMALLN=0
