"""Average per-dispatch PMC values of one kernel from rocprofv3 --pmc pass directories.
Usage: python tools/pmc_summary.py <kernel-substring> <dir>/p1 <dir>/p2 ..."""
import collections
import csv
import sys

name = sys.argv[1]
for d in sys.argv[2:]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if name in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(d, k, f"{sum(v) / len(v):.4g}", f"n={len(v)}")
