set -u
mkdir -p gpurun_out/fit1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fit1/tests.txt 2>&1; rc=$?
tail -25 gpurun_out/fit1/tests.txt
[ $rc -eq 0 ] || exit $rc
for w in n2v mip barf; do
  timeout -k 10 200 python -u bench.py --mode render --workload $w > gpurun_out/fit1/render_$w.json 2> gpurun_out/fit1/render_$w.err || { tail gpurun_out/fit1/render_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fit1/render_$w.json'));print('$w render', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', {k: round(v['ms_per_step'],3) for k,v in d['kernels'].items()})"
done
