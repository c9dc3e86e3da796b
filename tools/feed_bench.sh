# bench lines with the on-device ray feed (default) and with one resident batch (--feed fixed)
set -u
OUT=gpurun_out/${1:-feedb}
mkdir -p "$OUT"
for w in n2v mip barf; do
  for f in device fixed; do
    timeout -k 10 300 python -u bench.py --workload $w --feed $f --no-cpu-baseline > "$OUT/$w.$f.json" 2> "$OUT/$w.$f.err" \
      || { tail -20 "$OUT/$w.$f.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$w.$f.json'));print('$w $f', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms loss', round(d['final_loss'],4))"
  done
done
