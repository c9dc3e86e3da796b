#!/bin/bash
# Multi-process rehearsal of bench.py's DP step on ONE GPU: 2 ranks share the device over gloo
# (the driver's N>1 runs use RCCL, one GPU per rank).
set -u
OUT=gpurun_out/${1:-dp}; mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
NERF_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  --no-frame-roofline > $OUT/bench_dp2_gloo.json 2> $OUT/bench_dp2_gloo.err || { echo "dp rehearsal failed"; tail -30 $OUT/bench_dp2_gloo.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench_dp2_gloo.json').read().strip().splitlines()[-1]);print(d['n_gpus'],d['value'],d['ms_per_step'],d['final_loss'],d['config']['parallelism'])"
