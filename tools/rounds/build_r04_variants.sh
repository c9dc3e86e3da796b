#!/bin/bash
# The round-4 A/B libraries (nerf-experiments_amd/var/, git-ignored, shipped to the GPU box):
# lib_unroll0 (NERF_FUSED_UNROLL2=0), lib_wreg0 (the LDS-DMA weight ring), lib_hgp16k (16384-entry
# hash-grid parts) and lib_head (the fused MLP kernel of commit 7f0a8c4, before this round's second
# session: 256-sample compositing and the hash-grid generator absent).
set -eu
cd "$(dirname "$0")/.."
bash tools/build_variant.sh unroll0 "-DNERF_FUSED_UNROLL2=0" | tail -1
bash tools/build_variant.sh wreg0 "-DNERF_FUSED_WREG=0" | tail -1
bash tools/build_variant.sh hgp16k "-DNERF_HG_PART_ENTRIES=16384" hashgrid | tail -1
cd nerf-experiments_amd
git show 7f0a8c4:nerf-experiments_amd/csrc/mlp_fused.hip > var/mlp_fused_head.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include -Icsrc \
  -c var/mlp_fused_head.hip -o var/mlp_fused_head.o 2>/dev/null
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o var/lib_head.so $(ls build/*.o | grep -v build/mlp_fused.o) var/mlp_fused_head.o
echo nerf-experiments_amd/var/lib_head.so
