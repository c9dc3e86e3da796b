#!/bin/bash
# PMC of the stand-alone encoding / compositing kernels at one full frame (bench.py frame roofline)
set -u
O=gpurun_out/r05g; mkdir -p $O
export TMPDIR=/tmp
i=0
for group in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $group -d $O/p$i -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
