#!/bin/bash
# PMC passes over the fused MLP forward microbenchmark (one counter group per pass).
set -u
OUT=${1:-gpurun_out/fprof}
shift || true
ARGS="$@"
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/fused_bench.py $ARGS > $OUT/time.txt 2>&1 || { cat $OUT/time.txt; exit 1; }
cat $OUT/time.txt
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 tools/fused_bench.py --iters 5 $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
echo done
