#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter_collection CSVs per kernel (name substring) per shape.

    python tools/summarize_pmc.py <outdir> <kernel-substring> [json-out]

FETCH_SIZE/WRITE_SIZE are reported in KB by rocprofv3; on gfx950 FETCH_SIZE
undercounts by 2x (MI355X_MICROARCH.md, HBM section) — `hbm_bytes` applies that
correction: bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    out, ksub = sys.argv[1], sys.argv[2]
    res = {}
    for d in sorted(glob.glob(os.path.join(out, "*_p*"))):
        if not os.path.isdir(d):
            continue
        shape = os.path.basename(d).rsplit("_p", 1)[0]
        acc = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if ksub in row["Kernel_Name"]:
                        acc[(row["Dispatch_Id"], row["Counter_Name"])].append(float(row["Counter_Value"]))
        per = collections.defaultdict(list)
        for (disp, name), vals in acc.items():
            per[name].append(sum(vals))
        r = res.setdefault(shape, {})
        for name, vals in per.items():
            r[name] = sum(vals) / len(vals)
    for shape, r in res.items():
        if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
            r["hbm_bytes"] = (2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
