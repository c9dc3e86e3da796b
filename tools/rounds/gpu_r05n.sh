#!/bin/bash
set -u
O=gpurun_out/r05n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/debug/time_w32.py 524288 2>&1 | grep -v amdgpu.ids
for w in 0 1; do
W32_LIST=$w timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY \
  -d $O/pmc_w$w -o run --output-format csv -- python3 tools/debug/time_w32.py 524288 > $O/pmc_w$w.log 2>&1 || { tail $O/pmc_w$w.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for w in (0, 1):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r05n/pmc_w{w}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "mlp_fused" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    d = {c: sum(v) / len(v) for c, v in acc.items()}
    print(w, {c: round(v / 1e6, 2) for c, v in d.items()}, "VALU/MFMA", round(d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"], 2),
          "SALU/MFMA", round(d["SQ_INSTS_SALU"] / d["SQ_INSTS_MFMA"], 2), "LDS/MFMA", round(d["SQ_INSTS_LDS"] / d["SQ_INSTS_MFMA"], 2))
PY
