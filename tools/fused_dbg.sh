for lib in nerf-experiments_amd/build/var/lib_*.so; do
  echo "== $lib"; NERF_AMD_LIB=$lib timeout -k 10 200 python -u tools/diag/fused_dbg.py 2>&1 | grep "^M=" | grep -v "nbad 0 "
done
