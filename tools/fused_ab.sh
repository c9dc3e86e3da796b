set -u
for lib in nerf-experiments_amd/nerf_amd/libnerf_amd.so nerf-experiments_amd/build/var/lib_ladder.so; do
  NERF_AMD_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
done
bash tools/fused_diag.sh
