#!/bin/bash
# PMC passes over the hash-grid backward at the finest (hashed) and coarsest (bijective) levels.
set -u
OUT=gpurun_out/${1:-hgpmc_k}
bash tools/hashgrid_prof.sh $OUT/l15 --only 15 && bash tools/hashgrid_prof.sh $OUT/l0 --only 0 && \
python3 tools/pmc_summary.py hashgrid_bwd_kernel $OUT/l15/p1 $OUT/l15/p2 > $OUT/l15_summary.txt && \
python3 tools/pmc_summary.py hashgrid_bwd_kernel $OUT/l0/p1 $OUT/l0/p2 > $OUT/l0_summary.txt && cat $OUT/l15_summary.txt $OUT/l0_summary.txt
