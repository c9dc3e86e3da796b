"""Per-launch PMC evidence for bench.py's roofline objects, from a tools/profile_bench.sh directory.

Reads the rocprofv3 passes <dir>/bench_p*/run_counter_collection.csv (FETCH_SIZE, WRITE_SIZE and
the SQ / GRBM instruction and cycle groups, each in its own pass) and writes, for every MFMA
kernel function bench.py can name as its roofline kernel,
  profiles/traffic_<workload>_<fn>.json   bytes per launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024
                                          (gfx950 FETCH_SIZE counts half of wide streaming reads,
                                          MI355X_MICROARCH.md HBM section)
  profiles/pmc_<workload>_<fn>.json       every other counter, averaged per launch
Kernel functions are named as rocprofv3 names them: the function, template arguments kept for the
fused MLP kernel (mlp_fused_kernel<0> = forward, <1> = input-gradient chain) and dropped for the
others (all instantiations of linear_nt_x3_glds_kernel are one function, as bench.py groups them).

    python tools/roofline_evidence.py gpurun_out/<tag>/prof_mip mip
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import evidence_tag  # noqa: E402

FNS = ("mlp_fused_kernel<0>", "mlp_fused_kernel<1>", "mlp_fused_kernel<2>", "mlp_fused_kernel<3>", "linear_nt_x3_glds_kernel", "linear_nt_x3_kernel", "linear_wgrad_smalln_kernel",
       "linear_wgrad_x3_tr_kernel", "linear_wgrad_x3_stream_kernel", "linear_wgrad_x3_kernel", "linear_nt_kernel",
       "linear_wgrad_kernel",
       "hashgrid_bwd_kernel", "hashgrid_fwd_kernel", "hashgrid_fwd_level_kernel", "hashgrid_fwd_tile_kernel",
       "hashgrid_bwd_walk_kernel", "hashgrid_gtr_kernel", "hashgrid_bucket_kernel", "hashgrid_bucket_add_kernel")


def fn_name(kernel_name: str) -> str:
    """'void (anonymous namespace)::mlp_fused_kernel<0>(FusedArgs)' -> 'mlp_fused_kernel<0>'."""
    s = kernel_name.replace("void ", "").replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in s:                      # cut at the argument list (first '(' outside template args)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    s = "".join(out).strip()
    if not s.startswith("mlp_fused_kernel"):
        s = re.sub(r"<.*>$", "", s)
    return s


def main(src: str, workload: str, dst: str = os.path.join(ROOT, "profiles")):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(glob.glob(f"{src}/bench_p*")):
        f = f"{d}/run_counter_collection.csv"
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            per[fn_name(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    written = []
    for fn in FNS:
        if fn not in per:
            continue
        c = {k: sum(v) / len(v) for k, v in per[fn].items()}
        launches = {k: len(v) for k, v in per[fn].items()}
        tag = evidence_tag(workload, fn)
        src_rel = os.path.relpath(src, ROOT)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            t = {"kernel": fn, "workload": workload,
                 "bytes_per_launch": (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0,
                 "FETCH_SIZE_KB": c["FETCH_SIZE"], "WRITE_SIZE_KB": c["WRITE_SIZE"],
                 "launches": [launches["FETCH_SIZE"], launches["WRITE_SIZE"]],
                 "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE, separate passes over "
                           "bench.py --steps 5 --warmup 2 (tools/profile_bench.sh); bytes = (2*FETCH_SIZE + "
                           "WRITE_SIZE)*1024 per launch, gfx950 correction of MI355X_MICROARCH.md",
                 "source": src_rel}
            with open(os.path.join(dst, f"traffic_{tag}.json"), "w") as fh:
                json.dump(t, fh, indent=1)
            written.append(f"traffic_{tag}.json")
        pm = {k: v for k, v in c.items() if k not in ("FETCH_SIZE", "WRITE_SIZE")}
        if pm:
            out = {"kernel": fn, "workload": workload, "per_launch": pm,
                   "launches": {k: launches[k] for k in pm}, "source": src_rel,
                   "notes": "per-launch averages; SQ_*_CYCLES and SQ_BUSY_CYCLES in the units rocprofv3 reports "
                            "(SQ cycle counters count quad-cycles, summed over SEs); SQ_VALU_MFMA_BUSY_CYCLES "
                            "advances 16 per v_mfma_f32_16x16x32_bf16 issued (= 16 x SQ_INSTS_MFMA for that "
                            "shape), so it counts MFMA work, not a utilisation fraction"}
            if "SQ_INSTS_MFMA" in pm and "SQ_VALU_MFMA_BUSY_CYCLES" in pm and pm["SQ_INSTS_MFMA"] > 0:
                out["mfma_busy_per_mfma"] = pm["SQ_VALU_MFMA_BUSY_CYCLES"] / pm["SQ_INSTS_MFMA"]
            with open(os.path.join(dst, f"pmc_{tag}.json"), "w") as fh:
                json.dump(out, fh, indent=1)
            written.append(f"pmc_{tag}.json")
    print("\n".join(written))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
