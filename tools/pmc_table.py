"""Per-dispatch average of every PMC counter of the kernels matching a name, over the passes of a
tools/fused_prof.sh (or profile_counters.sh) output directory.  Usage: python tools/pmc_table.py DIR [name]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "mlp_fused"
out = {}
for p in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if name in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
for k in sorted(out):
    print(f"{k:28s} {out[k]:.4g}")
