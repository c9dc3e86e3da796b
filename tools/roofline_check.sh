set -u
mkdir -p gpurun_out/roof
for w in n2v mip barf; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/roof/$w.json 2> gpurun_out/roof/$w.err || { tail gpurun_out/roof/$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/roof/$w.json'));r=d['roofline'];print('$w', round(d['value']/1e6,2), r['kernel'][:24], r['bound'], round(r['achieved'],1), r['unit'], 'frac', round(r['frac'],3), 'AI', round(r['arithmetic_intensity'],1), 'ridge', round(r['ridge'],1), 'bytes', round(r['avg_bytes_per_launch']/1e6,1), 'traffic', r['traffic'])"
done
timeout -k 10 300 python -u bench.py --mode render --no-cpu-baseline > gpurun_out/roof/render.json 2> gpurun_out/roof/render.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/roof/render.json'));r=d['roofline'];print('render', round(d['value']/1e6,2), r['kernel'][:24], r['bound'], round(r['achieved'],1), r['unit'], 'frac', round(r['frac'],3), 'AI', round(r['arithmetic_intensity'],1))"
