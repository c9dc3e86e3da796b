#!/bin/bash
# PMC passes over the bucketed hash-grid backward (finest level alone) and its write traffic.
set -u
OUT=gpurun_out/${1:-hgpmc_b}
export NERF_HG_BUCKET=1
bash tools/hashgrid_prof.sh $OUT/l15 --only 15 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/l15/p3 -o run --output-format csv -- python3 tools/hashgrid_bench.py --iters 3 --only 15 > $OUT/l15/p3.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/l15/p4 -o run --output-format csv -- python3 tools/hashgrid_bench.py --iters 3 --only 15 > $OUT/l15/p4.log 2>&1 || { echo "fetch pass failed"; exit 1; }
for k in hashgrid_bucket_kernel hashgrid_bucket_add_kernel; do
  echo "== $k"; python3 tools/pmc_summary.py $k $OUT/l15/p1 $OUT/l15/p2 $OUT/l15/p3 $OUT/l15/p4
done > $OUT/summary.txt
cat $OUT/summary.txt
