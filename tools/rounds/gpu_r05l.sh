#!/bin/bash
set -u
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 300 python -u tools/debug/dbg_w32.py 32768 262144 > $O/dbg.txt 2>&1 || { cat $O/dbg.txt; exit 1; }
grep -v amdgpu.ids $O/dbg.txt
bash tools/rounds/gpu_r05j.sh
