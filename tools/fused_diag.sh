#!/bin/bash
# Timing diagnostics of the fused forward: the baseline library and NERF_DIAG variants.
set -u
for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so nerf-experiments_amd/build/var/lib_*.so; do
  echo "$(basename $lib): $(NERF_AMD_LIB=$lib timeout -k 10 120 python3 tools/fused_bench.py 2>&1 | grep forward)"
done
