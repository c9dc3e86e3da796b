#!/bin/bash
# 32-sample-wave forward: diagnostic variants (no weight stream / no per-slot barrier / no stores)
# and SQ counters of the product build
set -u
O=gpurun_out/r05m; mkdir -p $O
export TMPDIR=/tmp
run() { # tag lib w32
  NERF_ALLOW_DIAG_BUILD=1 NERF_AMD_LIB=$2 NERF_FUSED_W32=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-frame-roofline --steps 40 --warmup 5 \
    > $O/bench_$1.json 2> $O/bench_$1.err || { tail -20 $O/bench_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$1.json'));k=d['kernels'];print('$1', round(d['ms_per_step'],3), {n:round(v['ms_per_step'],3) for n,v in k.items()})"
}
L=nerf-experiments_amd
run w16 $L/nerf_amd/libnerf_amd.so 0
run w32 $L/nerf_amd/libnerf_amd.so 1
run w32_nodma $L/var/lib_w32_NODMA.so 1
run w32_nobar $L/var/lib_w32_NOBARRIER.so 1
run w32_nostore $L/var/lib_w32_NOSTORE.so 1
i=0
for group in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  NERF_FUSED_W32=1 timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $group -d "$O/pmc_p$i" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-frame-roofline --steps 5 --warmup 2 > "$O/pmc_p$i.log" 2>&1 \
    || { echo "pmc pass $i failed"; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r05m/pmc_p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "mlp_fused" in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
