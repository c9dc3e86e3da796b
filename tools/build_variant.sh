#!/bin/bash
# Build a variant of libnerf_amd.so with extra compile flags on one source (default mlp_fused.hip):
#   bash tools/build_variant.sh <name> "<flags>" [source-stem]
# -> nerf-experiments_amd/var/lib_<name>.so (travels to the GPU box; select with NERF_AMD_LIB=...;
#    a NERF_*_DIAG_* ablation build is refused by load() unless NERF_ALLOW_DIAG_BUILD=1)
set -eu
NAME=$1; FLAGS=$2; SRC=${3:-mlp_fused}
cd "$(dirname "$0")/../nerf-experiments_amd"
make -s -j8
mkdir -p var
OBJS=$(ls build/*.o | grep -v "build/$SRC.o")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include -Icsrc $FLAGS \
  -c csrc/$SRC.hip -o var/${SRC}_$NAME.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o var/lib_$NAME.so $OBJS var/${SRC}_$NAME.o
echo "nerf-experiments_amd/var/lib_$NAME.so"
