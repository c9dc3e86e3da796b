#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only, as MI355X_MICROARCH.md prescribes)
# over single-shape microbench runs.  Usage: tools/profile_counters.sh <outdir> <shape>...
set -u
OUT=${1:?outdir}; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
for shape in "$@"; do
  i=0
  for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
               "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --kernel-trace --pmc $group -d "$OUT/${shape}_p$i" -o run --output-format csv \
      -- python3 tools/microbench.py --only "$shape" > "$OUT/${shape}_p$i.log" 2>&1 || { echo "pass $i of $shape failed: $?"; exit 1; }
  done
done
echo done
