#!/bin/bash
# per-shape timing of the small-N weight gradient against the 128-tile kernel (same box)
set -u
OUT=gpurun_out/${1:-smalln_t}; mkdir -p $OUT
NERF_WGRAD_SMALLN=0 timeout -k 10 200 python -u tools/wgrad_ab.py --out /tmp/wa.pt > $OUT/wgrad_tile.txt 2>&1 || { echo "A failed"; exit 1; }
timeout -k 10 200 python -u tools/wgrad_ab.py --out /tmp/wb.pt --compare /tmp/wa.pt --rtol 1e-5 > $OUT/wgrad_smalln.txt 2>&1 || { echo "B failed"; tail $OUT/wgrad_smalln.txt; exit 1; }
grep "N4_" $OUT/wgrad_tile.txt $OUT/wgrad_smalln.txt
