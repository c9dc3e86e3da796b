#!/bin/bash
# the generated encoding rows stored nontemporal (NERF_FUSED_GEN_NT=1) vs production
set -u
O=gpurun_out/r05au; mkdir -p $O
export TMPDIR=/tmp
L=nerf-experiments_amd
run() {
  t=$1_$2
  NERF_ALLOW_DIAG_BUILD=1 NERF_AMD_LIB=$L/var/lib_$1.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 60 --warmup 10 \
    > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));k=d['kernel_functions'];print('$t', round(d['ms_per_step'],3), round(d['final_loss'],9), {n:round(v['ms_per_step'],3) for n,v in k.items() if 'fused' in n})"
}
for v in prod gnt; do run $v 1 || exit 1; done
for v in gnt prod; do run $v 2 || exit 1; done
for v in prod gnt; do run $v 3 || exit 1; done
for v in gnt prod; do run $v 4 || exit 1; done
