#!/bin/bash
set -u
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 300 python -u tools/debug/dbg_w32.py > $O/dbg.txt 2>&1; rc=$?
cat $O/dbg.txt | grep -v amdgpu.ids
exit $rc
